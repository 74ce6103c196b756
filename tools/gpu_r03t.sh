#!/bin/bash
# round 3: 12-byte chain records with 32-bit keys (two large-network scenarios per CU, twelve
# small ones) -- subproblem / B&B / restricted GPU tests, then timing
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_subproblem.py tests/test_bnb.py tests/test_restricted.py -m gpu -x -v --timeout 170 --timeout-method thread > gpurun_out/r03t_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r03t_tests.log; exit 1; }
tail -1 gpurun_out/r03t_tests.log
for c in "C3 64 26" "C4 256 32" "C4 256 32 --gen-lb" "C5 512 4"; do
  set -- $c
  timeout -k 10 200 python -u tools/sub_bench.py --cfg $1 --scenarios $2 --paths $3 $4 --reps 3 > gpurun_out/r03t_$1$4.log 2>&1 || { tail gpurun_out/r03t_$1$4.log; exit 1; }
  echo "$1 $4: $(tail -1 gpurun_out/r03t_$1$4.log)"
done
