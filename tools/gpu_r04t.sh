#!/bin/bash
# round 4: subproblem LDS counters (C4 32 paths x 256 scenarios, 8-byte chain records)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY \
    --output-format csv -d gpurun_out/r04_sub_pmc -o run -- python3 tools/sub_bench.py --cfg C4 --paths 32 --scenarios 256 --reps 2 \
    > gpurun_out/r04_sub_pmc.log 2>&1 || exit $?
tail -1 gpurun_out/r04_sub_pmc.log
