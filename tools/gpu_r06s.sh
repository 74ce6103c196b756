#!/bin/bash
# round 6: leaf pairs (SGUFP_LEAF_FAST=2: both leaves' coefficient reads issued before either walk)
# with and without the staging pipeline, against the tree's library, on the seeded C4 leg; the
# 64-scenario P1 / P3 instances (generated lower bounds) closed by the device B&B vs HiGHS
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
A=$PWD/sgufp_solver_amd/lib_alt
BNBS="--mode bnb --bnb-config C4 --bnb-lb zero --nodes 1024 --round-seconds 5 --bnb-heuristic 128"
for v in tree f2p0 f2; do
  L=""; [ $v != tree ] && L=$A/$v/libsgufp_hip.so
  SGUFP_LIB_PATH=$L timeout -k 10 200 python3 bench.py $BNBS --bnb-seconds 20 > gpurun_out/r06s_bnbs_$v.json 2> gpurun_out/r06s_bnbs_$v.log || exit 11
done
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_bnb.py -k "lower_bounds" \
  > gpurun_out/r06s_p.log 2>&1
