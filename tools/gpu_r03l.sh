#!/bin/bash
# round 3: invalidation -- dead nodes stop jumping (lib_var/live) vs the committed kernel
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
P=$PWD/sgufp_solver_amd/lib_var/live/libsgufp_hip.so
SGUFP_LIB_PATH=$P timeout -k 10 300 python -u -m pytest tests/test_subproblem.py -m gpu -x -q --timeout 170 --timeout-method thread > gpurun_out/r03l_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r03l_tests.log; exit 1; }
tail -1 gpurun_out/r03l_tests.log
for c in "C3 64 26" "C4 256 32" "C5 512 4"; do
  set -- $c
  for v in main live; do
    if [ $v = main ]; then L=; else L=$P; fi
    SGUFP_LIB_PATH=$L timeout -k 10 200 python -u tools/sub_bench.py --cfg $1 --scenarios $2 --paths $3 --reps 3 > gpurun_out/r03l_${v}_$1.log 2>&1 || { tail gpurun_out/r03l_${v}_$1.log; exit 1; }
    echo "$v $1: $(tail -1 gpurun_out/r03l_${v}_$1.log)"
  done
done
for v in trmain trlive; do
SGUFP_LIB_PATH=$PWD/sgufp_solver_amd/lib_var/$v/libsgufp_hip.so timeout -k 10 120 python -u tools/sub_bench.py --cfg C3 --scenarios 64 --paths 26 --reps 0 > gpurun_out/r03l_${v}_c3.log 2>&1 || exit 1
echo $v; grep SUB gpurun_out/r03l_${v}_c3.log | head -2
done
