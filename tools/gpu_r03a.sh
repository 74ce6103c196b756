#!/bin/bash
# round 3: GPU suite + exploratory B&B runs (bounded rounds)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03a_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r03a_tests.log; exit 1; }
tail -3 gpurun_out/r03a_tests.log
timeout -k 10 400 python -u tools/bnb_explore.py T4:1:64:zero:7004.265625:120 C2:1:1:zero:29299:240 > gpurun_out/r03a_bnb.json 2> gpurun_out/r03a_bnb.err
rc=$?; cat gpurun_out/r03a_bnb.json; tail -5 gpurun_out/r03a_bnb.err; exit $rc
