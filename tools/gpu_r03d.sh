#!/bin/bash
# round 3: device-resident refinement loop -- B&B / host-API / subproblem GPU tests, then the
# device B&B on C3 under a kernel trace and on C5 (cut generation in the loop) with a budget
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-r03d}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_bnb.py tests/test_host_api.py tests/test_restricted.py -m gpu -x -v --timeout 170 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_bnb_stats -o run -- python3 bench.py --mode bnb --bnb-config C3 --nodes 1024 --bnb-seconds 20 > gpurun_out/${TAG}_bnb_c3.json 2> gpurun_out/${TAG}_bnb_c3.err || { tail gpurun_out/${TAG}_bnb_c3.err; exit 1; }
cat gpurun_out/${TAG}_bnb_c3.json
timeout -k 10 300 python3 bench.py --mode bnb --bnb-config C5 --nodes 1024 --bnb-seconds 30 > gpurun_out/${TAG}_bnb_c5.json 2> gpurun_out/${TAG}_bnb_c5.err || { tail gpurun_out/${TAG}_bnb_c5.err; exit 1; }
cat gpurun_out/${TAG}_bnb_c5.json
