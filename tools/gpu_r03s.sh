#!/bin/bash
# round 3: register predecessors in the eight-wave (large-network) subproblem kernel --
# subproblem / B&B GPU tests, then C5 4 x 512 A/B (SGUFP_SUB_PREDS_LDS=1: LDS chain records)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_subproblem.py tests/test_bnb.py -m gpu -x -v --timeout 170 --timeout-method thread > gpurun_out/r03s_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r03s_tests.log; exit 1; }
tail -1 gpurun_out/r03s_tests.log
for d in 1 0; do
  SGUFP_SUB_PREDS_LDS=$d timeout -k 10 200 python -u tools/sub_bench.py --cfg C5 --scenarios 512 --paths 4 --reps 2 > gpurun_out/r03s_d$d.log 2>&1 || { tail gpurun_out/r03s_d$d.log; exit 1; }
  echo "preds_lds=$d C5: $(tail -1 gpurun_out/r03s_d$d.log)"
done
timeout -k 10 200 python -u tools/sub_bench.py --cfg C4 --scenarios 256 --paths 32 --reps 3 > gpurun_out/r03s_c4.log 2>&1 || { tail gpurun_out/r03s_c4.log; exit 1; }
echo "C4: $(tail -1 gpurun_out/r03s_c4.log)"
