#!/bin/bash
# round 6: the rest of r06k's tests (C5 / C4 generated lower bounds, the non-exact phase, the C++
# host driver); the seeded C4 leg with open-leaf compaction (SGUFP_LEAF_SPLIT 16, default) and
# without (0) plus its kernel shares (rocprofv3 --stats); the cut-parallel non-exact phase on the
# headline step (SGUFP_NX_MIN=1, SGUFP_NX_SKIP 0 / 8 / 16) against the default
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
( while sleep 50; do date >> gpurun_out/r06l_heartbeat.log; done ) &
HB=$!
T="python3 -u -m pytest -x -v --timeout 600 --timeout-method thread"
timeout -k 10 600 $T tests/test_bnb_parity.py -k "c5_generated or c4_generated" tests/test_nx_phase.py tests/test_host_api.py \
  > gpurun_out/r06l_tests.log 2>&1 || { kill $HB; exit 12; }
BNBS="--mode bnb --bnb-config C4 --bnb-lb zero --nodes 1024 --round-seconds 5 --bnb-heuristic 128"
for sp in 16 0; do
  SGUFP_LEAF_SPLIT=$sp SGUFP_EXACT_STATS=1 timeout -k 10 200 python3 bench.py $BNBS --bnb-seconds 20 > gpurun_out/r06l_bnbs_split$sp.json 2> gpurun_out/r06l_bnbs_split$sp.log || { kill $HB; exit 13; }
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06l_bnbs_stats -o run -- python3 bench.py $BNBS --bnb-seconds 20 > gpurun_out/r06l_bnbs_stats.log 2>&1 || { kill $HB; exit 14; }
ONLY="--no-cpu --no-parity --sub-paths 0 --c5-nodes 0 --bnb-seeded-width 0 --bnb-leg-seconds 0 --c5-bnb-seconds 0 --bnb-parity-rounds 0 --bnb-gen-seconds 0 --cpp-leg-seconds 0 --bnb-parity-survivor-pool 0"
timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 $ONLY > gpurun_out/r06l_head_default.json 2> gpurun_out/r06l_head_default.log || { kill $HB; exit 15; }
for skip in 0 8 16; do
  SGUFP_NX_MIN=1 SGUFP_NX_SKIP=$skip timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 $ONLY > gpurun_out/r06l_head_nx$skip.json 2> gpurun_out/r06l_head_nx$skip.log || { kill $HB; exit 16; }
done
kill $HB
