#!/bin/bash
# round 6: warm-start statistics of the C5 B&B with its generated lower bounds kept (feasible
# scenarios, 64-bit-key kernels): SGUFP_SUB_STATS prints every 200 subproblem launches, 45 s
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
SGUFP_SUB_STATS=1 timeout -k 10 200 python3 bench.py --mode bnb --bnb-config C5 --bnb-lb gen --nodes 1024 --round-seconds 5 --bnb-seconds 60 \
  > gpurun_out/r06y_bnb5_gen.json 2> gpurun_out/r06y_bnb5_gen.log
