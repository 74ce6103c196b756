#!/bin/bash
# round 4: leaf kernel v2 (scalar leaf words, early-stop checks every 4 blocks): parity + C3 B&B
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_bnb_parity.py tests/test_bnb.py -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/r04h_tests.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -2 gpurun_out/r04h_tests.log; ok $rc || exit $rc
SGUFP_EXACT_SCREEN=0 SGUFP_EXACT_STATS=1 timeout -k 10 200 python3 tools/bnb_tail_diag.py --config C3 --seconds 20 \
    --out gpurun_out/r04h.json > gpurun_out/r04h.log 2>&1 || exit $?
tail -1 gpurun_out/r04h.log
timeout -k 10 200 python3 tools/relax_diag.py --config C4 --nodes 8192 > gpurun_out/r04h_relax_diag.log 2>&1 || exit $?
cat gpurun_out/r04h_relax_diag.log | tail -12
