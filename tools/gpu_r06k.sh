#!/bin/bash
# round 6: (1) the work lists' group counts (exact marks, coarse successor marks = wl2) (SGUFP_SUB_TRACE printf, cold C4 32 x 256) against the
# full sweeps; (2) B&B parity with the round-6 leaf passes and lower-bound warm starts (C3 seeded,
# M1, exact-phase variants, generated lower bounds, the non-exact phase) and the C++ host driver;
# (3) the seeded C4 leg with open-leaf compaction (SGUFP_LEAF_SPLIT 16, default) and without (0)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
( while sleep 50; do date >> gpurun_out/r06k_heartbeat.log; done ) &
HB=$!
A=$PWD/sgufp_solver_amd/lib_alt
for v in trace tracewl2 tracenowl; do
  SGUFP_LIB_PATH=$A/$v/libsgufp_hip.so timeout -k 10 120 python3 tools/sub_bench.py --cfg C4 --scenarios 256 --paths 32 --reps 1 > gpurun_out/r06k_$v.log 2>&1 || { kill $HB; exit 11; }
done
for v in wl2; do
  SGUFP_LIB_PATH=$A/$v/libsgufp_hip.so timeout -k 10 120 python3 tools/sub_bench.py --cfg C4 --scenarios 256 --paths 32 --reps 3 > gpurun_out/r06k_sub_$v.log 2>&1 || { kill $HB; exit 11; }
  SGUFP_LIB_PATH=$A/$v/libsgufp_hip.so SGUFP_SUB_STATS=1 timeout -k 10 200 python3 bench.py --mode bnb --bnb-config C4 --bnb-lb zero --nodes 1024 --round-seconds 5 --bnb-seconds 20 > gpurun_out/r06k_bnb_$v.json 2> gpurun_out/r06k_bnb_$v.log || { kill $HB; exit 11; }
done
T="python3 -u -m pytest -x -v --timeout 600 --timeout-method thread"
timeout -k 10 700 $T tests/test_bnb_parity.py -k "c3_seeded or m1 or variants or generated" tests/test_nx_phase.py tests/test_host_api.py \
  > gpurun_out/r06k_tests.log 2>&1 || { kill $HB; exit 12; }
BNBS="--mode bnb --bnb-config C4 --bnb-lb zero --nodes 1024 --round-seconds 5 --bnb-heuristic 128"
for sp in 16 0; do
  SGUFP_LEAF_SPLIT=$sp SGUFP_EXACT_STATS=1 timeout -k 10 200 python3 bench.py $BNBS --bnb-seconds 20 > gpurun_out/r06k_bnbs_split$sp.json 2> gpurun_out/r06k_bnbs_split$sp.log || { kill $HB; exit 13; }
done
kill $HB
