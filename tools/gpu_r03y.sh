#!/bin/bash
# round 3: segmented chain groups (one tail depth per group) with the one-quiet-sweep stop
# -- subproblem / B&B / restricted GPU tests, then timing
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_subproblem.py tests/test_bnb.py tests/test_restricted.py tests/test_host_api.py -m gpu -x -v --timeout 170 --timeout-method thread > gpurun_out/r03y_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r03y_tests.log; exit 1; }
tail -1 gpurun_out/r03y_tests.log
for c in "C3 64 26" "C4 256 32" "C4 256 32 --gen-lb" "C5 512 4"; do
  set -- $c
  timeout -k 10 200 python -u tools/sub_bench.py --cfg $1 --scenarios $2 --paths $3 $4 --reps 3 > gpurun_out/r03y_$1$4.log 2>&1 || { tail gpurun_out/r03y_$1$4.log; exit 1; }
  echo "$1 $4: $(tail -1 gpurun_out/r03y_$1$4.log)"
done
L=$PWD/sgufp_solver_amd/lib_var/trace/libsgufp_hip.so
SGUFP_LIB_PATH=$L timeout -k 10 120 python -u tools/sub_bench.py --cfg C3 --scenarios 64 --paths 26 --reps 0 > gpurun_out/r03y_trace_c3.log 2>&1 || exit 1
grep SUB gpurun_out/r03y_trace_c3.log | head -3
