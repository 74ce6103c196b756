#!/bin/bash
# round 5: completion study -- M1 / 64 seeded with opt - 10 (main.cpp:75) for 10 minutes; the
# progress lines (frontier, incumbent, pool, counters) every 2 s give the trend if it does not close
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python3 -u tools/bnb_try.py M1:1:64:0:10 > gpurun_out/r05w_m1.log 2>&1
rc=$?; echo "rc=$rc (124: the 10-minute limit)"; tail -4 gpurun_out/r05w_m1.log | cut -c1-600
[ $rc -eq 0 ] || [ $rc -eq 124 ] || exit $rc
exit 0
