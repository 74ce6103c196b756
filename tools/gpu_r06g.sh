#!/bin/bash
# round 6: C3 survivors at 6e4 cuts; the B&B with the generated lower bounds against ref_dd
# (C3, C5, C4 at a 5e3-cut feasibility pool); the C++ host driver against the Python one
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
( while sleep 50; do date >> gpurun_out/r06g_heartbeat.log; done ) &
HB=$!
T="python3 -u -m pytest -v -s --timeout 1000 --timeout-method thread"
timeout -k 10 500 $T tests/test_bnb_parity.py -k "generated" tests/test_host_api.py > gpurun_out/r06g_tests.log 2>&1
rc1=$?
if [ $rc1 -ge 124 ]; then kill $HB; exit $rc1; fi   # a time limit / abort / fault: no further GPU step
timeout -k 10 600 $T tests/test_bnb_parity.py -k "c3_survivors" > gpurun_out/r06g_survivors.log 2>&1
rc2=$?
kill $HB
exit $((rc1 + rc2))
