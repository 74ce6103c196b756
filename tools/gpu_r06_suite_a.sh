#!/bin/bash
# round-6 end, GPU suite part A (every -m gpu test outside test_bnb_parity.py) + smoke, final library
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
( while sleep 50; do date >> gpurun_out/r06_suite_heartbeat.log; done ) &
HB=$!
sha256sum sgufp_solver_amd/lib/libsgufp_hip.so > gpurun_out/r06_suite_a.log
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -v --durations=30 --timeout 600 --timeout-method thread --ignore=tests/test_bnb_parity.py \
  >> gpurun_out/r06_suite_a.log 2>&1
rc=$?
if [ $rc -lt 124 ]; then
  timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06_smoke.log 2>&1
fi
kill $HB
exit $rc
