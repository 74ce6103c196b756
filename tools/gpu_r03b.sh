#!/bin/bash
# round 3: full GPU suite, subproblem timing after the scratch removal, bounded B&B on C3 / C5
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --durations=15 --timeout 170 --timeout-method thread > gpurun_out/r03b_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r03b_tests.log; exit 1; }
tail -3 gpurun_out/r03b_tests.log
timeout -k 10 120 python -u tools/sub_bench.py --cfg C3 --scenarios 64 --paths 26 --reps 3 > gpurun_out/r03b_sub.log 2>&1 && \
timeout -k 10 120 python -u tools/sub_bench.py --cfg C5 --scenarios 512 --paths 4 --reps 2 >> gpurun_out/r03b_sub.log 2>&1 || { cat gpurun_out/r03b_sub.log; exit 1; }
cat gpurun_out/r03b_sub.log
timeout -k 10 400 python -u tools/bnb_explore.py C3:1:64:zero:none:120 C5:1:512:zero:none:150 > gpurun_out/r03b_bnb.json 2> gpurun_out/r03b_bnb.err
rc=$?; cat gpurun_out/r03b_bnb.json; tail -4 gpurun_out/r03b_bnb.err; exit $rc
