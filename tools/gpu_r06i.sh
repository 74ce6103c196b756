#!/bin/bash
# round 6 (re-entry): the whole GPU suite with the committed library, smoke, the default bench line
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
( while sleep 50; do date >> gpurun_out/r06i_heartbeat.log; done ) &
HB=$!
timeout -k 10 1500 python3 -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread \
  > gpurun_out/r06i_tests.log 2>&1 || { kill $HB; exit 11; }
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06i_smoke.log 2>&1 || { kill $HB; exit 12; }
timeout -k 10 600 python3 bench.py > gpurun_out/r06i_bench.json 2> gpurun_out/r06i_bench.log
rc=$?
kill $HB
exit $rc
