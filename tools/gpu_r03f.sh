#!/bin/bash
# round 3: subproblem chain partition -- subproblem + B&B tests, timing, B&B on C3
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-r03f}
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_subproblem.py tests/test_bnb.py tests/test_restricted.py -m gpu -x -v --timeout 170 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
timeout -k 10 120 python -u tools/sub_bench.py --cfg C3 --scenarios 64 --paths 26 --reps 3 > gpurun_out/${TAG}_sub.log 2>&1 && \
timeout -k 10 120 python -u tools/sub_bench.py --cfg C4 --scenarios 256 --paths 32 --reps 2 >> gpurun_out/${TAG}_sub.log 2>&1 || { cat gpurun_out/${TAG}_sub.log; exit 1; }
cat gpurun_out/${TAG}_sub.log
timeout -k 10 300 python3 bench.py --mode bnb --bnb-config C3 --nodes 1024 --bnb-seconds 20 > gpurun_out/${TAG}_bnb_c3.json 2> gpurun_out/${TAG}_bnb_c3.err || { tail gpurun_out/${TAG}_bnb_c3.err; exit 1; }
cat gpurun_out/${TAG}_bnb_c3.json
