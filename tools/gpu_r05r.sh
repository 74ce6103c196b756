#!/bin/bash
# round 5: where a warm-started scenario's time goes (phase clocks, lib_alt/phases)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
SGUFP_LIB_PATH=$PWD/sgufp_solver_amd/lib_alt/phases/libsgufp_hip.so timeout -k 10 200 python3 bench.py --mode bnb --bnb-config C4 \
    --bnb-lb zero --bnb-seconds 10 --nodes 1024 --round-seconds 5 > gpurun_out/r05r_bnb.json 2> gpurun_out/r05r_bnb.err || exit $?
grep -c SUBPH gpurun_out/r05r_bnb.json
python3 - <<'PY'
import re, collections
acc = collections.defaultdict(lambda: [0, 0, 0, 0, 0, 0])
for l in open("gpurun_out/r05r_bnb.json"):
    m = re.search(r"SUBPH warm=(\d) chains (\d+) flow (\d+) potentials (\d+) dual (\d+) starts (\d+)", l)
    if m:
        a = acc[m.group(1)]
        a[0] += 1
        for k in range(5): a[k + 1] += int(m.group(k + 2))
for w, a in acc.items():
    n = a[0]
    print(f"warm={w}: {n} scenarios, mean ticks (10 ns): chains {a[1]/n:.0f} flow {a[2]/n:.0f} potentials {a[3]/n:.0f} "
          f"dual {a[4]/n:.0f} chain_starts {a[5]/n:.0f}")
PY
