#!/bin/bash
# round 6: work-list Bellman-Ford in the subproblem (single-wave kernels) -- the subproblem
# tests (warm == cold on the verify build, kernel variants, HiGHS objectives), then A/B against
# full sweeps (lib_alt/nowl, -DSGUFP_SUB_NO_WL): the C4 32 x 256 micro-bench, the unseeded C4
# B&B and the seeded one with the generated lower bounds (pass counts on stderr)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T="python3 -u -m pytest -x -v --timeout 300 --timeout-method thread"
NOWL=$PWD/sgufp_solver_amd/lib_alt/nowl/libsgufp_hip.so
BNB="--mode bnb --bnb-config C4 --bnb-lb zero --nodes 1024 --round-seconds 5"
BNBG="--mode bnb --bnb-config C4 --bnb-lb gen --nodes 1024 --round-seconds 5 --bnb-heuristic 128"
timeout -k 10 700 $T tests/test_subproblem.py > gpurun_out/r06j_tests.log 2>&1 || exit 11
for v in wl nowl; do
  L=""; [ $v = nowl ] && L=$NOWL
  SGUFP_LIB_PATH=$L timeout -k 10 200 python3 tools/sub_bench.py --cfg C4 --scenarios 256 --paths 32 --reps 3 > gpurun_out/r06j_sub_$v.log 2>&1 || exit 12
  SGUFP_LIB_PATH=$L SGUFP_SUB_STATS=1 timeout -k 10 200 python3 bench.py $BNB --bnb-seconds 20 > gpurun_out/r06j_bnb_$v.json 2> gpurun_out/r06j_bnb_$v.log || exit 13
  SGUFP_LIB_PATH=$L SGUFP_SUB_STATS=1 timeout -k 10 200 python3 bench.py $BNBG --bnb-seconds 20 > gpurun_out/r06j_bnbg_$v.json 2> gpurun_out/r06j_bnbg_$v.log || exit 14
done
