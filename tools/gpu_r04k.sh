#!/bin/bash
# round 4: pipelined coefficient staging in k_exact_leaf: parity + seeded C3 / C4 B&B
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 900 python -u -m pytest tests/test_bnb_parity.py tests/test_bnb.py -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/r04k_tests.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -2 gpurun_out/r04k_tests.log; ok $rc || exit $rc
for C in C3 C4; do
  SGUFP_EXACT_STATS=1 timeout -k 10 200 python3 tools/bnb_tail_diag.py --config $C --seconds 20 \
      --width $([ $C = C3 ] && echo 64 || echo 128) --out gpurun_out/r04k_$C.json > gpurun_out/r04k_$C.log 2>&1 || exit $?
  echo "$C"; tail -1 gpurun_out/r04k_$C.log
done
