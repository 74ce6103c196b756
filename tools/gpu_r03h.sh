#!/bin/bash
# round 3: production k_relax without clock stamps -- parity suite + headline timing
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 170 --timeout-method thread > gpurun_out/r03h_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r03h_tests.log; exit 1; }
tail -2 gpurun_out/r03h_tests.log
timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --bnb-leg-seconds 0 --c5-nodes 0 --sub-paths 0 --no-cpu > gpurun_out/r03h_bench.json 2> gpurun_out/r03h_bench.err || { tail gpurun_out/r03h_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r03h_bench.json')); print(d['value'], d['roofline']['avg_launch_ms'])"
