#!/bin/bash
# round 5: where the unseeded C4 B&B leg's time goes (kernel shares, GPU busy vs wall)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/r05ab_prof" -o run -- \
    python3 "$GRAFT_REPO_ROOT/bench.py" --mode bnb --bnb-config C4 --bnb-lb zero --bnb-seconds 20 --nodes 1024 --round-seconds 5 \
    > "$GRAFT_REPO_ROOT/gpurun_out/r05ab_c4.json" 2> "$GRAFT_REPO_ROOT/gpurun_out/r05ab_c4.err"
rc=$?; cd "$GRAFT_REPO_ROOT"; echo "rc=$rc"
python3 -c "import json;d=json.loads(open('gpurun_out/r05ab_c4.json').read().splitlines()[-1]);print(d['relaxations_per_s'], d['subproblems_per_s'], d['seconds'], d['rounds'], d['counters'])"
python3 tools/trace_busy.py gpurun_out/r05ab_prof/run_kernel_trace.csv 2>&1 | tail -15
rm -f gpurun_out/r05ab_prof/run_kernel_trace.csv
exit $rc
