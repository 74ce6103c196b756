#!/bin/bash
# round 5: C3 survivors at a 60k-cut pool (parity), then where the C5 B&B's GPU time goes
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
cd /tmp && SGUFP_SUB_STATS=1 SGUFP_EXACT_STATS=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$GRAFT_REPO_ROOT/gpurun_out/r05v_prof" -o run -- \
    python3 "$GRAFT_REPO_ROOT/bench.py" --mode bnb --bnb-config C5 --bnb-lb zero --bnb-seconds 20 --nodes 1024 --round-seconds 5 \
    > "$GRAFT_REPO_ROOT/gpurun_out/r05v_c5.json" 2> "$GRAFT_REPO_ROOT/gpurun_out/r05v_c5.err"
rc2=$?; cd "$GRAFT_REPO_ROOT"; echo "c5 rc=$rc2"; f=$(ls gpurun_out/r05v_prof/*kernel_stats.csv gpurun_out/r05v_prof/*/*kernel_stats.csv 2>/dev/null | head -1)
[ -n "$f" ] && head -16 "$f" | cut -c1-200
python3 -c "import json;d=json.loads(open('gpurun_out/r05v_c5.json').read().splitlines()[-1]);print(d['relaxations_per_s'], d['subproblems_per_s'], d['counters'])"
grep '\[sub\]' gpurun_out/r05v_c5.err | tail -1; grep 'non-exact' gpurun_out/r05v_c5.err | tail -1 | cut -c1-400
[ $rc2 -eq 0 ] || exit $rc2
timeout -k 10 700 python -u -m pytest tests/test_bnb_parity.py -k "survivors" -v --timeout 600 \
    --timeout-method thread -m gpu > gpurun_out/r05v_parity.log 2>&1
rc=$?; echo "parity rc=$rc"; grep -E "passed|failed" gpurun_out/r05v_parity.log | tail -2
grep -E "FAILED|^E " gpurun_out/r05v_parity.log | head -6 | cut -c1-600
exit $rc
