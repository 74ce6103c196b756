#!/bin/bash
# round 5: cut-parallel optimality phase of non-exact DDs -- engagement diagnostics and parity
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/nx_diag.py C4 > gpurun_out/r05g_diag.log 2>&1
rc=$?; grep -E "incumbent|\[exact\]" gpurun_out/r05g_diag.log | head -20; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests/test_nx_phase.py -v --timeout 300 --timeout-method thread -m gpu \
    > gpurun_out/r05g_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed" gpurun_out/r05g_tests.log | tail -2
grep -E "FAILED" gpurun_out/r05g_tests.log | head -10
exit $rc
