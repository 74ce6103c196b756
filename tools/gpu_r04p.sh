#!/bin/bash
# round 4: leaf sizing 8 layers / 16 leaves per wave: parity suites, then the round-end bench + counters
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_bnb_parity.py tests/test_bnb.py -x -q \
    --timeout 300 --timeout-method thread > gpurun_out/r04p_tests.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -2 gpurun_out/r04p_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_bench_r04.sh
