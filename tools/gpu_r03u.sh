#!/bin/bash
# round 3: the subproblem kernel variants agree bit for bit (32 / 64-bit keys, 12 / 16-byte
# chain records, register / LDS predecessors)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_subproblem.py -m gpu -x -v -k variants --timeout 200 --timeout-method thread > gpurun_out/r03u_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r03u_tests.log; exit 1; }
tail -3 gpurun_out/r03u_tests.log
