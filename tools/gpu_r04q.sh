#!/bin/bash
# round 4: refinement chunk by arc-LP work (C4: 64 -> 320 paths per iteration): seeded C3 / C4 B&B
# at the new default and at the old 16 384 LPs
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for C in C4 C3; do
  W=$([ $C = C3 ] && echo 64 || echo 128)
  for CW in default old; do
    if [ $CW = old ]; then export SGUFP_CHUNK_WORK=$((16384 * $([ $C = C3 ] && echo 64 || echo 256) * 1000)); else unset SGUFP_CHUNK_WORK; fi
    timeout -k 10 200 python3 tools/bnb_tail_diag.py --config $C --seconds 20 --width $W \
        --out gpurun_out/r04q_${C}_$CW.json > gpurun_out/r04q_${C}_$CW.log 2>&1 || exit $?
    echo "$C $CW $(tail -1 gpurun_out/r04q_${C}_$CW.log)"
  done
done
