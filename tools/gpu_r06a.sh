#!/bin/bash
# round 6, first box: the new GPU tests (dd view state, warm-slot checks, warm starts with
# lower bounds, non-exact survivors at 2e4 / 1e5 cuts), then the seeded C4 B&B with the
# generated lower bounds (subproblem statistics on stderr).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
( while sleep 50; do date >> gpurun_out/r06a_heartbeat.log; done ) &
HB=$!
T="python3 -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_subproblem.py -k "lower_bounds" \
  > gpurun_out/r06a_tests.log 2>&1 || { kill $HB; exit 11; }
SGUFP_SUB_STATS=1 timeout -k 10 300 python3 bench.py --mode bnb --bnb-config C4 --bnb-lb gen --nodes 1024 --round-seconds 5 \
  --bnb-heuristic 128 --bnb-seconds 20 > gpurun_out/r06a_bnb_gen_seeded.json 2> gpurun_out/r06a_bnb_gen_seeded.log || { kill $HB; exit 12; }
SGUFP_SUB_STATS=1 timeout -k 10 300 python3 bench.py --mode bnb --bnb-config C4 --bnb-lb gen --nodes 1024 --round-seconds 5 \
  --bnb-seconds 20 > gpurun_out/r06a_bnb_gen.json 2> gpurun_out/r06a_bnb_gen.log || { kill $HB; exit 13; }
timeout -k 10 1300 $T --timeout 1500 tests/test_bnb_parity.py -k "survivors" -s > gpurun_out/r06a_survivors.log 2>&1
rc=$?
kill $HB
exit $rc
