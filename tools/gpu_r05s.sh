#!/bin/bash
# round 5: per-path chain lists (k_sub_paths): subproblem + B&B tests, C4 B&B legs, phase clocks
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_subproblem.py tests/test_bnb.py -x -v --timeout 240 --timeout-method thread -m gpu \
    > gpurun_out/r05s_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed" gpurun_out/r05s_tests.log | tail -2; [ $rc -eq 0 ] || exit $rc
for h in 0 128; do
  SGUFP_SUB_STATS=1 timeout -k 10 200 python3 bench.py --mode bnb --bnb-config C4 --bnb-lb zero --bnb-seconds 20 \
      --nodes 1024 --round-seconds 5 --bnb-heuristic $h > gpurun_out/r05s_h$h.json 2> gpurun_out/r05s_h$h.err || exit $?
  echo "h=$h: $(python3 -c "import json;d=json.loads(open('gpurun_out/r05s_h$h.json').read().splitlines()[-1]);print(d['relaxations_per_s'], d['subproblems_per_s'])") $(grep '\[sub\]' gpurun_out/r05s_h$h.err | tail -1)"
done
SGUFP_LIB_PATH=$PWD/sgufp_solver_amd/lib_alt/phases/libsgufp_hip.so timeout -k 10 200 python3 bench.py --mode bnb --bnb-config C4 \
    --bnb-lb zero --bnb-seconds 10 --nodes 1024 --round-seconds 5 > gpurun_out/r05s_ph.json 2> gpurun_out/r05s_ph.err || exit $?
python3 - <<'PY'
import re, collections
acc = collections.defaultdict(lambda: [0] * 9)
for l in open("gpurun_out/r05s_ph.json"):
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
