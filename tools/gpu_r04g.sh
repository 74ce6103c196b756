#!/bin/bash
# round 4: exact phase with screening columns first -- parity, then A/B of the screen width
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_bnb_parity.py -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/r04g_tests.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -2 gpurun_out/r04g_tests.log; ok $rc || exit $rc
for sc in 0 256; do
  SGUFP_EXACT_SCREEN=$sc SGUFP_EXACT_STATS=1 timeout -k 10 200 python3 tools/bnb_tail_diag.py --config C3 --seconds 20 \
    --out gpurun_out/r04g_s$sc.json > gpurun_out/r04g_s$sc.log 2>&1 || exit $?
  tail -1 gpurun_out/r04g_s$sc.log
done
