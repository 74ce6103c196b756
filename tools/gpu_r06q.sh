#!/bin/bash
# round 6: leaf-pass variants on the seeded C4 leg (20 s each): the tree's library (balanced passes,
# fast exact loop with lazy walks, staging pipeline), v2 (no staging pipeline: no scratch reload
# inside the leaf loop), v3 (v2 with the walk's info from LDS), v4 (balanced, general loop), nobal
# (general loop, unbalanced); the per-wave clock split of v2 (lib_alt/leafclk); then B&B parity and
# the non-exact phase on the tree's library and on v2
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
A=$PWD/sgufp_solver_amd/lib_alt
BNBS="--mode bnb --bnb-config C4 --bnb-lb zero --nodes 1024 --round-seconds 5 --bnb-heuristic 128"
for v in tree v2 v3 v4 nobal; do
  L=""; [ $v != tree ] && L=$A/$v/libsgufp_hip.so
  SGUFP_LIB_PATH=$L timeout -k 10 200 python3 bench.py $BNBS --bnb-seconds 20 > gpurun_out/r06q_bnbs_$v.json 2> gpurun_out/r06q_bnbs_$v.log || exit 11
done
SGUFP_LIB_PATH=$A/leafclk/libsgufp_hip.so SGUFP_EXACT_STATS=1 timeout -k 10 200 python3 bench.py $BNBS --bnb-seconds 12 \
  > gpurun_out/r06q_leafclk.json 2> gpurun_out/r06q_leafclk.log || exit 12
T="python3 -u -m pytest -x -v --timeout 500 --timeout-method thread"
timeout -k 10 420 $T tests/test_bnb_parity.py -k "c3_seeded or m1 or variants" > gpurun_out/r06q_parity.log 2>&1 || exit 13
SGUFP_LIB_PATH=$A/v2/libsgufp_hip.so timeout -k 10 300 $T tests/test_bnb_parity.py -k "c3_seeded or m1" > gpurun_out/r06q_parity_v2.log 2>&1 || exit 14
timeout -k 10 200 $T tests/test_nx_phase.py tests/test_host_api.py > gpurun_out/r06q_tests.log 2>&1
