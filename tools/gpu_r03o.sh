#!/bin/bash
# round 3: Bellman-Ford stops after a quiet sweep that follows a non-stale one (single wave): tests + timing
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_subproblem.py tests/test_bnb.py -m gpu -x -v --timeout 170 --timeout-method thread > gpurun_out/r03o_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r03o_tests.log; exit 1; }
tail -2 gpurun_out/r03o_tests.log
for d in 0; do
  for c in "C3 64 26" "C4 256 32" "C4 256 32 --gen-lb"; do
    set -- $c
    SGUFP_SUB_PREDS_LDS=$d timeout -k 10 200 python -u tools/sub_bench.py --cfg $1 --scenarios $2 --paths $3 $4 --reps 3 > gpurun_out/r03o_d${d}_$1$4.log 2>&1 || { tail gpurun_out/r03o_d${d}_$1$4.log; exit 1; }
    echo "preds_lds=$d $1 $4: $(tail -1 gpurun_out/r03o_d${d}_$1$4.log)"
  done
done
