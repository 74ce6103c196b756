#!/bin/bash
# round 5: completion study, long run -- M1 / 64 seeded with opt - 10 (main.cpp:75) for up to 19 minutes
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 1130 python3 -u tools/bnb_try.py M1:1:64:0:10 > gpurun_out/r05af_m1.log 2>&1
rc=$?; echo "rc=$rc (124: the time limit)"; tail -3 gpurun_out/r05af_m1.log | cut -c1-600
[ $rc -eq 0 ] || [ $rc -eq 124 ] || exit $rc
exit 0
