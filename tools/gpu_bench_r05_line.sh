#!/bin/bash
# round-5 end: the bench line (reads the r05 counters from profiles/ when the library matches)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 1150 python3 bench.py > gpurun_out/bench_r05.json 2> gpurun_out/bench_r05.err || exit $?
tail -c 3000 gpurun_out/bench_r05.json
