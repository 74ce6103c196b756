#!/bin/bash
# round-6 end, GPU suite part B: test_bnb_parity.py with the long checks (SGUFP_GPU_LONG=1) (round-by-round B&B parity, timed-pool and
# survivor checks, generated lower bounds), final library
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
( while sleep 50; do date >> gpurun_out/r06_suite_heartbeat_b.log; done ) &
HB=$!
sha256sum sgufp_solver_amd/lib/libsgufp_hip.so > gpurun_out/r06_suite_b.log
SGUFP_GPU_LONG=1 timeout -k 10 1100 python3 -u -m pytest tests/test_bnb_parity.py -m gpu -v -s --durations=0 --timeout 1000 --timeout-method thread \
  >> gpurun_out/r06_suite_b.log 2>&1
rc=$?
kill $HB
exit $rc
