#!/bin/bash
# round 4: DD depth of the exact survivors in the seeded C3 / C4 searches
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for C in C3 C4; do
  timeout -k 10 200 python3 tools/bnb_tail_diag.py --config $C --seconds 15 --gl-hist \
      --width $([ $C = C3 ] && echo 64 || echo 128) > gpurun_out/r04n_$C.log 2>&1 || exit $?
  echo "$C"; tail -1 gpurun_out/r04n_$C.log
done
