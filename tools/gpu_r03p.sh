#!/bin/bash
# round 3: single-wave Bellman-Ford sweeps over register groups two at a time (lib_var/pair)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
P=$PWD/sgufp_solver_amd/lib_var/pair/libsgufp_hip.so
SGUFP_LIB_PATH=$P timeout -k 10 300 python -u -m pytest tests/test_subproblem.py -m gpu -x -q --timeout 170 --timeout-method thread > gpurun_out/r03p_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r03p_tests.log; exit 1; }
tail -1 gpurun_out/r03p_tests.log
for c in "C3 64 26" "C4 256 32" "C4 256 32 --gen-lb"; do
  set -- $c
  for v in main pair; do
    if [ $v = main ]; then L=; else L=$P; fi
    SGUFP_LIB_PATH=$L timeout -k 10 200 python -u tools/sub_bench.py --cfg $1 --scenarios $2 --paths $3 $4 --reps 3 > gpurun_out/r03p_${v}_$1$4.log 2>&1 || { tail gpurun_out/r03p_${v}_$1$4.log; exit 1; }
    echo "$v $1 $4: $(tail -1 gpurun_out/r03p_${v}_$1$4.log)"
  done
done
SGUFP_LIB_PATH=$PWD/sgufp_solver_amd/lib_var/trpair/libsgufp_hip.so timeout -k 10 120 python -u tools/sub_bench.py --cfg C3 --scenarios 64 --paths 26 --reps 0 > gpurun_out/r03p_trace_c3.log 2>&1 || exit 1
grep SUB gpurun_out/r03p_trace_c3.log | head -3
