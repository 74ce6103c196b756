#!/bin/bash
# round-6 end: the GPU suite exactly as the driver runs it (pytest tests -x -q -m gpu, default
# environment) with its wall time, then smoke -- final library
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
( while sleep 50; do date >> gpurun_out/r06_suite_default_heartbeat.log; done ) &
HB=$!
sha256sum sgufp_solver_amd/lib/libsgufp_hip.so > gpurun_out/r06_suite_default.log
t0=$(date +%s)
timeout -k 10 1050 python3 -u -m pytest tests -x -v -m gpu --durations=15 --timeout 600 --timeout-method thread >> gpurun_out/r06_suite_default.log 2>&1
rc=$?
echo "wall_s $(( $(date +%s) - t0 )) rc $rc" >> gpurun_out/r06_suite_default.log
if [ $rc -lt 124 ]; then
  timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06_smoke.log 2>&1
fi
kill $HB
exit $rc
