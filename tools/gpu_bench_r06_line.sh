#!/bin/bash
# round-6 end: the bench line (reads the r06 counters from profiles/ when the library matches)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 1100 python3 bench.py > gpurun_out/bench_r06.json 2> gpurun_out/bench_r06.err || exit $?
tail -c 3000 gpurun_out/bench_r06.json
