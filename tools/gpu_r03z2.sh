#!/bin/bash
# round 3: invalidation unroll depth (kInvU 2 / 4 / 8) on the subproblem benches
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_subproblem.py -m gpu -x -q --timeout 170 --timeout-method thread > gpurun_out/r03z2_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r03z2_tests.log; exit 1; }
tail -1 gpurun_out/r03z2_tests.log
for c in "C3 64 26" "C4 256 32" "C5 512 4"; do
  set -- $c
  for v in new u2 u8 base; do
    if [ $v = new ]; then L=; else L=$PWD/sgufp_solver_amd/lib_var/$v/libsgufp_hip.so; fi
    SGUFP_LIB_PATH=$L timeout -k 10 200 python -u tools/sub_bench.py --cfg $1 --scenarios $2 --paths $3 --reps 3 > gpurun_out/r03z2_${v}_$1.log 2>&1 || { tail gpurun_out/r03z2_${v}_$1.log; exit 1; }
    echo "$v $1: $(tail -1 gpurun_out/r03z2_${v}_$1.log)"
  done
done
