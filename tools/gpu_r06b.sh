#!/bin/bash
# round 6, second box: (1) the cut-parallel non-exact phase on the headline step (SGUFP_NX_MIN=1,
# SGUFP_NX_SKIP 0 / 8 / 16) against the default; (2) the seeded C4 leg with the exact phase's
# counters (SGUFP_EXACT_STATS=1: passes, blocks swept, leaves open after 16 / 64 blocks);
# (3) FETCH_SIZE / WRITE_SIZE of the seeded leg's kernels (k_exact_leaf's HBM bytes).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
ONLY="--no-cpu --no-parity --sub-paths 0 --c5-nodes 0 --bnb-seeded-width 0 --bnb-leg-seconds 0 --c5-bnb-seconds 0 --bnb-parity-rounds 0 --bnb-gen-seconds 0 --cpp-leg-seconds 0 --bnb-parity-survivor-pool 0"
BNBS="--mode bnb --bnb-config C4 --bnb-lb zero --nodes 1024 --round-seconds 5 --bnb-heuristic 128"
timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 $ONLY > gpurun_out/r06b_head_default.json 2> gpurun_out/r06b_head_default.log || exit 11
for skip in 0 8 16; do
  SGUFP_NX_MIN=1 SGUFP_NX_SKIP=$skip timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 $ONLY > gpurun_out/r06b_head_nx$skip.json 2> gpurun_out/r06b_head_nx$skip.log || exit 12
done
SGUFP_EXACT_STATS=1 timeout -k 10 200 python3 bench.py $BNBS --bnb-seconds 20 > gpurun_out/r06b_bnbs_estats.json 2> gpurun_out/r06b_bnbs_estats.log || exit 13
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06b_bnbs_stats -o run -- python3 bench.py $BNBS --bnb-seconds 20 > gpurun_out/r06b_bnbs_stats.log 2>&1 || exit 14
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r06b_bnbs_fetch -o run -- python3 bench.py $BNBS --bnb-seconds 10 > gpurun_out/r06b_bnbs_fetch.log 2>&1 || exit 15
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/r06b_bnbs_write -o run -- python3 bench.py $BNBS --bnb-seconds 10 > gpurun_out/r06b_bnbs_write.log 2>&1 || exit 16
python3 tools/compact_pmc.py gpurun_out/r06b_bnbs_fetch/*counter_collection.csv gpurun_out/r06b_bnbs_write/*counter_collection.csv
