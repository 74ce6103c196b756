#!/bin/bash
# round 4: 8-cut batches in half-filled contexts: the whole GPU suite + smoke, then the bench line
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04w_tests.log 2>&1
rc=$?; echo "gpu suite rc=$rc"; tail -2 gpurun_out/r04w_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04w_smoke.log 2>&1 || exit $?
tail -1 gpurun_out/r04w_smoke.log
timeout -k 10 600 python3 bench.py > gpurun_out/r04w_bench.json 2> gpurun_out/r04w_bench.err || exit $?
tail -c 300 gpurun_out/r04w_bench.json
