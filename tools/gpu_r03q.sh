#!/bin/bash
# round 3: optimality-cut screening depth in the seeded device B&B (C3, incumbent from the
# restricted-DD heuristic, 20 s each), then a kernel trace of the default depth
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for sc in 4 16 64; do
  SGUFP_SCREEN=$sc timeout -k 10 200 python3 bench.py --mode bnb --bnb-config C3 --nodes 1024 --bnb-seconds 20 --bnb-heuristic 64 > gpurun_out/r03q_s$sc.json 2> gpurun_out/r03q_s$sc.err || { tail gpurun_out/r03q_s$sc.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r03q_s$sc.json')); print($sc, d['value'], d['subproblems_per_s'], d['counters']['pruned_optimality'], d['counters']['exact'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03q_stats -o run -- python3 bench.py --mode bnb --bnb-config C3 --nodes 1024 --bnb-seconds 20 --bnb-heuristic 64 > gpurun_out/r03q_prof.json 2> gpurun_out/r03q_prof.err || { tail gpurun_out/r03q_prof.err; exit 1; }
cat gpurun_out/r03q_stats/run_kernel_stats.csv | head -8
