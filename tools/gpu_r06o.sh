#!/bin/bash
# round 6: the seeded C4 leg's HBM traffic per kernel (FETCH_SIZE / WRITE_SIZE passes) with the leaf
# byte-model counters (SGUFP_EXACT_STATS: cumulative pass-blocks and staged row-blocks), kernel trace
# of the same command
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
BNBS="--mode bnb --bnb-config C4 --bnb-lb zero --nodes 1024 --round-seconds 5 --bnb-heuristic 128"
SGUFP_EXACT_STATS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06o_bnbs_stats -o run -- python3 bench.py $BNBS --bnb-seconds 12 > gpurun_out/r06o_bnbs_stats.log 2>&1 || exit 11
SGUFP_EXACT_STATS=1 timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r06o_bnbs_fetch -o run -- python3 bench.py $BNBS --bnb-seconds 12 > gpurun_out/r06o_bnbs_fetch.log 2>&1 || exit 12
SGUFP_EXACT_STATS=1 timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/r06o_bnbs_write -o run -- python3 bench.py $BNBS --bnb-seconds 12 > gpurun_out/r06o_bnbs_write.log 2>&1 || exit 13
python3 tools/compact_pmc.py gpurun_out/r06o_bnbs_fetch/*counter_collection.csv gpurun_out/r06o_bnbs_write/*counter_collection.csv
