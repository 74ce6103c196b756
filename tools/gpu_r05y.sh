#!/bin/bash
# round 5: the cut row summed in LDS (phase 5): subproblem + B&B tests, micro-bench, B&B legs, phase clocks
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_subproblem.py tests/test_bnb.py -x -q --timeout 240 --timeout-method thread -m gpu \
    > gpurun_out/r05y_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r05y_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 tools/sub_bench.py --cfg C4 --scenarios 256 --paths 32 --reps 3 > gpurun_out/r05y_c4.log 2>&1 || exit $?
timeout -k 10 150 python3 tools/sub_bench.py --cfg C5 --scenarios 512 --paths 4 --reps 2 > gpurun_out/r05y_c5.log 2>&1 || exit $?
echo "C4 $(tail -2 gpurun_out/r05y_c4.log | head -1) | C5 $(tail -2 gpurun_out/r05y_c5.log | head -1)"
export SGUFP_LIB_PATH=$PWD/sgufp_solver_amd/lib_alt/nolacc/libsgufp_hip.so
timeout -k 10 120 python3 tools/sub_bench.py --cfg C4 --scenarios 256 --paths 32 --reps 3 > gpurun_out/r05y_c4n.log 2>&1 || exit $?
timeout -k 10 150 python3 tools/sub_bench.py --cfg C5 --scenarios 512 --paths 4 --reps 2 > gpurun_out/r05y_c5n.log 2>&1 || exit $?
unset SGUFP_LIB_PATH
echo "nolacc: C4 $(tail -2 gpurun_out/r05y_c4n.log | head -1) | C5 $(tail -2 gpurun_out/r05y_c5n.log | head -1)"
for c in C4 C5; do
  for h in 0 128; do
    [ $c = C5 ] && [ $h = 128 ] && continue
    SGUFP_SUB_STATS=1 timeout -k 10 200 python3 bench.py --mode bnb --bnb-config $c --bnb-lb zero --bnb-seconds 15 \
        --nodes 1024 --round-seconds 5 --bnb-heuristic $h > gpurun_out/r05y_${c}_h$h.json 2> gpurun_out/r05y_${c}_h$h.err || exit $?
    echo "$c h=$h bnb: $(python3 -c "import json;d=json.loads(open('gpurun_out/r05y_${c}_h$h.json').read().splitlines()[-1]);print(d['relaxations_per_s'], d['subproblems_per_s'])") $(grep '\[sub\]' gpurun_out/r05y_${c}_h$h.err | tail -1)"
  done
done
SGUFP_LIB_PATH=$PWD/sgufp_solver_amd/lib_alt/phases/libsgufp_hip.so timeout -k 10 200 python3 bench.py --mode bnb --bnb-config C4 \
    --bnb-lb zero --bnb-seconds 10 --nodes 1024 --round-seconds 5 > gpurun_out/r05y_ph.json 2> gpurun_out/r05y_ph.err || exit $?
python3 - <<'PY'
import re, collections
acc = collections.defaultdict(lambda: [0] * 9)
for l in open("gpurun_out/r05y_ph.json"):
    m = re.search(r"SUBPH warm=(\d) chains (\d+) flow (\d+) potentials (\d+) dual (\d+) \(ticks\) repair bf (\d+) aug (\d+) inv (\d+) chk (\d+)", l)
    if m:
        a = acc[m.group(1)]
        a[0] += 1
        for k in range(8): a[k + 1] += int(m.group(k + 2))
for w, a in acc.items():
    n = a[0]
    print(f"warm={w}: {n} scenarios, mean ticks (10 ns): chains {a[1]/n:.0f} flow {a[2]/n:.0f} potentials {a[3]/n:.0f} dual {a[4]/n:.0f}"
          f" | repair bf {a[5]/n:.0f} aug {a[6]/n:.0f} inv {a[7]/n:.0f} chk {a[8]/n:.0f}")
PY
