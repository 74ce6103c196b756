#!/bin/bash
# round 6: warm-start statistics with the generated lower bounds kept (SGUFP_SUB_STATS: augmentations,
# flow / potential passes per scenario, fallbacks) on the C5 B&B (feasible scenarios, 64-bit keys)
# and the seeded C3 / C4 B&B; kernel shares of the unseeded C4 and the C5 B&B legs
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
SGUFP_SUB_STATS=1 timeout -k 10 200 python3 bench.py --mode bnb --bnb-config C5 --bnb-lb gen --nodes 1024 --round-seconds 5 --bnb-seconds 30 \
  > gpurun_out/r06x_bnb5_gen.json 2> gpurun_out/r06x_bnb5_gen.log || exit 11
SGUFP_SUB_STATS=1 timeout -k 10 200 python3 bench.py --mode bnb --bnb-config C3 --bnb-lb gen --nodes 1024 --round-seconds 5 --bnb-heuristic 64 --bnb-seconds 20 \
  > gpurun_out/r06x_bnb3_gen.json 2> gpurun_out/r06x_bnb3_gen.log || exit 12
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06x_bnb_stats -o run -- python3 bench.py --mode bnb --bnb-config C4 --bnb-lb zero --nodes 1024 --round-seconds 5 --bnb-seconds 20 > gpurun_out/r06x_bnb_stats.log 2>&1 || exit 13
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06x_bnb5_stats -o run -- python3 bench.py --mode bnb --bnb-config C5 --bnb-lb zero --nodes 1024 --round-seconds 5 --bnb-seconds 30 > gpurun_out/r06x_bnb5_stats.log 2>&1 || exit 14
rm -f gpurun_out/r06x_*_stats/run_kernel_trace.csv
