#!/bin/bash
# round 3: optimality-cut screening depth in the device B&B (C3, 20 s each)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for sc in 4 16 64; do
  SGUFP_SCREEN=$sc timeout -k 10 200 python3 bench.py --mode bnb --bnb-config C3 --nodes 1024 --bnb-seconds 20 > gpurun_out/r03i_bnb_s$sc.json 2> gpurun_out/r03i_bnb_s$sc.err || { tail gpurun_out/r03i_bnb_s$sc.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r03i_bnb_s$sc.json')); print($sc, d['value'], d['subproblems_per_s'], d['counters']['exact_closed'], d['counters']['pruned_optimality'])"
done
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d gpurun_out/r03i_subpmc -o run -- python3 tools/sub_bench.py --cfg C3 --scenarios 64 --paths 26 --reps 1 > gpurun_out/r03i_subpmc.log 2>&1 || { tail gpurun_out/r03i_subpmc.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU SQ_BUSY_CYCLES SQ_WAVES --output-format csv -d gpurun_out/r03i_subpmc2 -o run -- python3 tools/sub_bench.py --cfg C3 --scenarios 64 --paths 26 --reps 1 > gpurun_out/r03i_subpmc2.log 2>&1 || { tail gpurun_out/r03i_subpmc2.log; exit 1; }
echo pmc done
