#!/bin/bash
# round 6: balanced leaf passes (a pass's leaves split evenly over its waves) -- the seeded C4 leg
# against lib_alt/nobal (-DSGUFP_LEAF_BALANCE=0) and the per-wave clock split (lib_alt/leafclk);
# then B&B parity, the non-exact phase and the C++ host API with the tree's library
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
A=$PWD/sgufp_solver_amd/lib_alt
BNBS="--mode bnb --bnb-config C4 --bnb-lb zero --nodes 1024 --round-seconds 5 --bnb-heuristic 128"
for v in bal nobal; do
  L=""; [ $v = nobal ] && L=$A/nobal/libsgufp_hip.so
  SGUFP_LIB_PATH=$L timeout -k 10 200 python3 bench.py $BNBS --bnb-seconds 20 > gpurun_out/r06q_bnbs_$v.json 2> gpurun_out/r06q_bnbs_$v.log || exit 11
done
SGUFP_LIB_PATH=$A/leafclk/libsgufp_hip.so SGUFP_EXACT_STATS=1 timeout -k 10 200 python3 bench.py $BNBS --bnb-seconds 12 \
  > gpurun_out/r06q_leafclk.json 2> gpurun_out/r06q_leafclk.log || exit 12
T="python3 -u -m pytest -x -v --timeout 500 --timeout-method thread"
timeout -k 10 600 $T tests/test_bnb_parity.py -k "c3_seeded or m1 or variants" > gpurun_out/r06q_parity.log 2>&1 || exit 13
timeout -k 10 300 $T tests/test_nx_phase.py tests/test_host_api.py > gpurun_out/r06q_tests.log 2>&1
