#!/bin/bash
# round 5: the unseeded C4 B&B (bench leg `bnb`): subproblem statistics and kernel time shares
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
SGUFP_SUB_STATS=1 timeout -k 10 200 python3 bench.py --mode bnb --bnb-config C4 --bnb-lb zero --bnb-seconds 20 --nodes 1024 \
    --round-seconds 5 > gpurun_out/r05p_bnb.json 2> gpurun_out/r05p_bnb.err || exit $?
grep "\[sub\]" gpurun_out/r05p_bnb.err | tail -3; tail -c 400 gpurun_out/r05p_bnb.json
SGUFP_SUB_STATS=1 timeout -k 10 200 python3 bench.py --mode bnb --bnb-config C4 --bnb-lb zero --bnb-seconds 20 --nodes 1024 \
    --round-seconds 5 --bnb-heuristic 128 > gpurun_out/r05p_bnbs.json 2> gpurun_out/r05p_bnbs.err || exit $?
grep "\[sub\]" gpurun_out/r05p_bnbs.err | tail -2
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/r05p_prof" -o run -- \
    python3 "$GRAFT_REPO_ROOT/bench.py" --mode bnb --bnb-config C4 --bnb-lb zero --bnb-seconds 20 --nodes 1024 --round-seconds 5 \
    > "$GRAFT_REPO_ROOT/gpurun_out/r05p_prof.log" 2>&1 || exit $?
cd "$GRAFT_REPO_ROOT"; head -12 gpurun_out/r05p_prof/run_kernel_stats.csv | cut -c1-160
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/r05p_prof/run_kernel_trace.csv")))
st = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows)
busy = 0; cur_s, cur_e = st[0]
for s, e in st[1:]:
    if s > cur_e:
        busy += cur_e - cur_s; cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += cur_e - cur_s
span = st[-1][1] - st[0][0]
print(f"kernels busy {busy/1e9:.2f} s of a {span/1e9:.2f} s span ({busy/span:.2%}), {len(rows)} dispatches")
PY
rm -f gpurun_out/r05p_prof/run_kernel_trace.csv
