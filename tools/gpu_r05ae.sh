#!/bin/bash
# round-5 end: B&B test files with the final library, then the profiling passes (tools/gpu_bench_r05.sh)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_bnb.py tests/test_bnb_parity.py tests/test_nx_phase.py -x -q --timeout 600 --timeout-method thread -m gpu \
    > gpurun_out/r05ae_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r05ae_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_bench_r05.sh
