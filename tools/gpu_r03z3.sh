#!/bin/bash
# round 3: skip chain groups without arcs of a sweep half (+ the invalidation rewrite)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_subproblem.py tests/test_bnb.py -m gpu -x -q --timeout 170 --timeout-method thread > gpurun_out/r03z3_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r03z3_tests.log; exit 1; }
tail -1 gpurun_out/r03z3_tests.log
for c in "C3 64 26" "C4 256 32" "C4 256 32 --gen-lb" "C5 512 4"; do
  set -- $c
  for v in new base; do
    if [ $v = new ]; then L=; else L=$PWD/sgufp_solver_amd/lib_var/$v/libsgufp_hip.so; fi
    SGUFP_LIB_PATH=$L timeout -k 10 200 python -u tools/sub_bench.py --cfg $1 --scenarios $2 --paths $3 $4 --reps 3 > gpurun_out/r03z3_${v}_$1$4.log 2>&1 || { tail gpurun_out/r03z3_${v}_$1$4.log; exit 1; }
    echo "$v $1 $4: $(tail -1 gpurun_out/r03z3_${v}_$1$4.log)"
  done
done
L=$PWD/sgufp_solver_amd/lib_var/trace/libsgufp_hip.so
SGUFP_LIB_PATH=$L timeout -k 10 120 python -u tools/sub_bench.py --cfg C3 --scenarios 64 --paths 26 --reps 0 > gpurun_out/r03z3_trace_c3.log 2>&1 || exit 1
grep SUB gpurun_out/r03z3_trace_c3.log | head -3
