#!/bin/bash
# round 5 final: seeded C3 / 64 B&B (width-64 heuristic) under rocprofv3 kernel stats -- k_relax's
# longest launch and the rate
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/r05aa_prof" -o run -- \
    python3 "$GRAFT_REPO_ROOT/bench.py" --mode bnb --bnb-config C3 --bnb-lb zero --bnb-seconds 20 --nodes 1024 --round-seconds 5 \
    --bnb-heuristic 64 > "$GRAFT_REPO_ROOT/gpurun_out/r05aa_c3.json" 2> "$GRAFT_REPO_ROOT/gpurun_out/r05aa_c3.err"
rc=$?; cd "$GRAFT_REPO_ROOT"; echo "rc=$rc"
python3 -c "import json;d=json.loads(open('gpurun_out/r05aa_c3.json').read().splitlines()[-1]);print(d['relaxations_per_s'], d['subproblems_per_s'], d['counters'])"
head -8 gpurun_out/r05aa_prof/run_kernel_stats.csv | cut -d, -f1-7 | cut -c1-220
rm -f gpurun_out/r05aa_prof/run_kernel_trace.csv
exit $rc
