#!/bin/bash
# round 5: warm-repair sub-phase clocks (lib_alt/phases)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
SGUFP_LIB_PATH=$PWD/sgufp_solver_amd/lib_alt/phases/libsgufp_hip.so timeout -k 10 200 python3 bench.py --mode bnb --bnb-config C4 \
    --bnb-lb zero --bnb-seconds 10 --nodes 1024 --round-seconds 5 > gpurun_out/r05t_ph.json 2> gpurun_out/r05t_ph.err || exit $?
python3 - <<'PY'
import re, collections
acc = collections.defaultdict(lambda: [0] * 9)
for l in open("gpurun_out/r05t_ph.json"):
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
