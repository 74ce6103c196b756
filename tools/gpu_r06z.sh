#!/bin/bash
# round 6: where the seeded C4 leg's dominant kernels wait -- SQ_WAIT_ANY (parked: waitcnt /
# barrier), SQ_WAIT_INST_ANY (issue stall), SQ_WAIT_INST_LDS, SQ_ACTIVE_INST_ANY over SQ_WAVE_CYCLES
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
BNBS="--mode bnb --bnb-config C4 --bnb-lb zero --nodes 1024 --round-seconds 5 --bnb-heuristic 128"
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS \
  --output-format csv -d gpurun_out/r06z_bnbs_wait -o run -- python3 bench.py $BNBS --bnb-seconds 8 > gpurun_out/r06z_bnbs_wait.log 2>&1 || exit 11
python3 tools/compact_pmc.py gpurun_out/r06z_bnbs_wait/*counter_collection.csv
