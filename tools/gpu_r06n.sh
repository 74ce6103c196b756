#!/bin/bash
# round 6: leaf-pass variants on the seeded C4 leg -- base (the tree's library), leafA (info bytes and
# the last layer's rows in registers, one barrier fewer, no staging pipeline), leafB (the same with
# the pipeline), leafC (info in registers only), leafD (one barrier fewer only); then B&B parity and
# the non-exact phase on leafA
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
A=$PWD/sgufp_solver_amd/lib_alt
BNBS="--mode bnb --bnb-config C4 --bnb-lb zero --nodes 1024 --round-seconds 5 --bnb-heuristic 128"
for v in base leafA leafB leafC leafD; do
  L=""; [ $v != base ] && L=$A/$v/libsgufp_hip.so
  SGUFP_LIB_PATH=$L timeout -k 10 200 python3 bench.py $BNBS --bnb-seconds 20 > gpurun_out/r06n_bnbs_$v.json 2> gpurun_out/r06n_bnbs_$v.log || exit 11
done
SGUFP_LIB_PATH=$A/leafA/libsgufp_hip.so timeout -k 10 600 python3 -u -m pytest -x -v --timeout 500 --timeout-method thread \
  tests/test_bnb_parity.py -k "c3_seeded or m1 or variants or c4_seeded" > gpurun_out/r06n_tests.log 2>&1 || exit 12
SGUFP_LIB_PATH=$A/leafA/libsgufp_hip.so timeout -k 10 200 python3 -u -m pytest -x -v --timeout 150 --timeout-method thread \
  tests/test_nx_phase.py > gpurun_out/r06n_nx.log 2>&1
