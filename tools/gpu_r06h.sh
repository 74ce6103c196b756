#!/bin/bash
# round 6: scalar-branch leaf loop (uniform masks, +inf past the pool, v_min_f64) and the
# subproblem's stop after the first infeasible scenario -- parity, then timings
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T="python3 -u -m pytest -x -v --timeout 400 --timeout-method thread"
BNBS="--mode bnb --bnb-config C4 --bnb-lb zero --nodes 1024 --round-seconds 5 --bnb-heuristic 128"
BNBG="--mode bnb --bnb-config C4 --bnb-lb gen --nodes 1024 --round-seconds 5 --bnb-heuristic 128"
timeout -k 10 900 $T tests/test_bnb_parity.py -k "c3_seeded or m1 or variants or c3_generated" \
  tests/test_subproblem.py -k "c3_seeded or m1 or variants or c3_generated or lower_bounds or matches_highs or benchmark_scenario" \
  > gpurun_out/r06h_tests.log 2>&1 || exit 11
for sp in 16 0; do
  SGUFP_LEAF_SPLIT=$sp SGUFP_EXACT_STATS=1 timeout -k 10 200 python3 bench.py $BNBS --bnb-seconds 20 > gpurun_out/r06h_bnbs_split$sp.json 2> gpurun_out/r06h_bnbs_split$sp.log || exit 12
done
timeout -k 10 200 python3 bench.py $BNBG --bnb-seconds 20 > gpurun_out/r06h_bnbg.json 2> gpurun_out/r06h_bnbg.log || exit 13
SGUFP_SUB_SKIP=0 timeout -k 10 200 python3 bench.py $BNBG --bnb-seconds 20 > gpurun_out/r06h_bnbg_noskip.json 2> gpurun_out/r06h_bnbg_noskip.log || exit 14
