#!/bin/bash
# round 3: full B&B to completion on the M configs (64 scenarios), seeded opt-10 and unseeded
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u tools/bnb_explore.py M1:1:64:zero:9211.781250000002:240 M1:1:64:zero:none:240 M2:1:16:zero:15204.250000000005:240 > gpurun_out/r03e_bnb.json 2> gpurun_out/r03e_bnb.err
rc=$?; cat gpurun_out/r03e_bnb.json; tail -3 gpurun_out/r03e_bnb.err; exit $rc
