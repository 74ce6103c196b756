#!/bin/bash
# round 6: (1) where a leaf pass's block time goes (lib_alt/leafclk: -DSGUFP_LEAF_CLOCKS, per-wave
# cycles of staging + barrier, leaf loop, flags + barrier; seeded C4 12 s); (2) the non-exact
# phase's survivors at 2e4 / 1e5 optimality cuts (the kept root children, no incumbent) against
# ref_dd relaxp; (3) the non-exact phase's fixtures and the C++ host driver
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
( while sleep 50; do date >> gpurun_out/r06p_heartbeat.log; done ) &
HB=$!
BNBS="--mode bnb --bnb-config C4 --bnb-lb zero --nodes 1024 --round-seconds 5 --bnb-heuristic 128"
SGUFP_LIB_PATH=$PWD/sgufp_solver_amd/lib_alt/leafclk/libsgufp_hip.so SGUFP_EXACT_STATS=1 timeout -k 10 200 python3 bench.py $BNBS --bnb-seconds 12 \
  > gpurun_out/r06p_leafclk.json 2> gpurun_out/r06p_leafclk.log || { kill $HB; exit 11; }
timeout -k 10 800 python3 -u -m pytest -x -v -s --timeout 1500 --timeout-method thread tests/test_bnb_parity.py -k "c4_survivors" \
  > gpurun_out/r06p_survivors.log 2>&1
rc=$?
if [ $rc -ne 0 ]; then kill $HB; exit $rc; fi
timeout -k 10 150 python3 -u -m pytest -x -v --timeout 140 --timeout-method thread tests/test_nx_phase.py tests/test_host_api.py \
  > gpurun_out/r06p_tests.log 2>&1
rc=$?
kill $HB
exit $rc
