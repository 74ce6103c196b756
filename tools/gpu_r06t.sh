#!/bin/bash
# round 6: sweep steps skipped when no lane of their register slot has a residual arc in that
# direction (lib_alt/skip) against the tree's library: C4 32 x 256 and C5 4 x 512 cold
# micro-benches, the unseeded C4 B&B (pass counts on stderr), the C5 B&B
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
A=$PWD/sgufp_solver_amd/lib_alt
BNB="--mode bnb --bnb-config C4 --bnb-lb zero --nodes 1024 --round-seconds 5"
for v in tree skip; do
  L=""; [ $v != tree ] && L=$A/$v/libsgufp_hip.so
  SGUFP_LIB_PATH=$L timeout -k 10 120 python3 tools/sub_bench.py --cfg C4 --scenarios 256 --paths 32 --reps 3 > gpurun_out/r06t_sub4_$v.log 2>&1 || exit 11
  SGUFP_LIB_PATH=$L timeout -k 10 200 python3 tools/sub_bench.py --cfg C5 --scenarios 512 --paths 4 --reps 2 > gpurun_out/r06t_sub5_$v.log 2>&1 || exit 12
  SGUFP_LIB_PATH=$L SGUFP_SUB_STATS=1 timeout -k 10 200 python3 bench.py $BNB --bnb-seconds 20 > gpurun_out/r06t_bnb_$v.json 2> gpurun_out/r06t_bnb_$v.log || exit 13
  SGUFP_LIB_PATH=$L timeout -k 10 200 python3 bench.py --mode bnb --bnb-config C5 --bnb-lb zero --nodes 1024 --round-seconds 5 --bnb-seconds 30 > gpurun_out/r06t_bnb5_$v.json 2> gpurun_out/r06t_bnb5_$v.log || exit 14
done
