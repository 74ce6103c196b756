#!/bin/bash
# round 3: 32-bit Bellman-Ford keys in the subproblem -- subproblem GPU tests, then A/B timing
# (SGUFP_SUB_KEY64=1 forces the 64-bit keys) on C3 26 x 64, C4 32 x 256 and C5 4 x 512 (lb 0)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_subproblem.py tests/test_bnb.py -m gpu -x -v --timeout 170 --timeout-method thread > gpurun_out/r03j_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r03j_tests.log; exit 1; }
tail -2 gpurun_out/r03j_tests.log
for k in 1 0; do
  for c in "C3 64 26" "C4 256 32" "C5 512 4"; do
    set -- $c
    SGUFP_SUB_KEY64=$k timeout -k 10 200 python -u tools/sub_bench.py --cfg $1 --scenarios $2 --paths $3 --reps 3 > gpurun_out/r03j_k${k}_$1.log 2>&1 || { tail gpurun_out/r03j_k${k}_$1.log; exit 1; }
    echo "key64=$k $1: $(tail -1 gpurun_out/r03j_k${k}_$1.log)"
  done
done
