#!/bin/bash
# round 4: B&B tests after the seen-list release, then a kernel trace of the seeded C3 search
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_bnb.py tests/test_solver_protocol.py -x -q -m gpu --timeout 300 \
    --timeout-method thread > gpurun_out/r04s_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r04s_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04s_trace -o run -- \
    python3 tools/bnb_tail_diag.py --config C3 --seconds 20 --out gpurun_out/r04s_c3.json > gpurun_out/r04s_c3.log 2>&1 || exit $?
tail -1 gpurun_out/r04s_c3.log
