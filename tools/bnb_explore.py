"""Exploratory device B&B runs with progress (frontier, incumbent, pool, counters).

    python tools/bnb_explore.py CFG:SEED:S:LB:KNOWN:BUDGET[:BATCH[:ROUND_S]] ...

LB = zero | gen (the generator's sink lower bounds), KNOWN = seed incumbent (a number, or
"none" for DOUBLE_MIN), BUDGET = seconds (0: until the frontier is empty).  One JSON line
per case on stdout, progress on stderr.
"""
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from sgufp_solver_amd import instance  # noqa: E402
from sgufp_solver_amd.pools import DOUBLE_MIN  # noqa: E402
from sgufp_solver_amd.solver import DDSolver  # noqa: E402

for arg in sys.argv[1:]:
    f = arg.split(":")
    cfg, seed, S, lbm, known, budget = f[0], int(f[1]), int(f[2]), f[3], f[4], float(f[5])
    batch = int(f[6]) if len(f) > 6 else 1024
    round_s = float(f[7]) if len(f) > 7 else 20.0
    inst = instance.generate(instance.CONFIGS[cfg], seed, scenarios=S)
    if lbm == "zero":
        inst.lb[:] = 0
    p = os.path.join(tempfile.mkdtemp(), "net.txt")
    inst.write(p)
    z0 = DOUBLE_MIN if known == "none" else float(known)
    s = DDSolver(p, max_batch=batch, verbose=False, progress=10.0, time_budget=budget, round_seconds=round_s)
    t0 = time.time()
    sol = s.start_solver(z0)
    sec = time.time() - t0
    print(json.dumps({"case": arg, "known": z0, "solution": sol, "complete": s.complete, "seconds": round(sec, 2),
                      "rounds": s.rounds, "frontier": s.eng.frontier_size(),
                      "pool": [s.eng.cuts_count(1), s.eng.cuts_count(0)], **s.counters}), flush=True)
    s.eng.close()
