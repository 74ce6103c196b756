"""Exploratory B&B runs on the device (prints per-instance optimum, rounds, counters, time)."""
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

EF = json.load(open(os.path.join(ROOT, "tests", "golden", "extensive_form.json")))
cases = [a.split(":") for a in sys.argv[1:]] or [["C1", "1", "1", "0", "10"]]
for cfg, seed, S, bn, gap in cases:
    key = f"{cfg}-{seed}-{S}"
    if key not in EF and gap == "inf":
        EF[key] = {"optimum": float("nan")}
    if key not in EF:
        from oracle import extensive_form as ef
        EF[key] = {"optimum": ef.solve(instance.generate(instance.CONFIGS[cfg], int(seed), scenarios=int(S)))}
    known = EF[key]["optimum"] - float(gap) if gap != "inf" else DOUBLE_MIN
    inst = instance.generate(instance.CONFIGS[cfg], int(seed), scenarios=int(S))
    d = tempfile.mkdtemp()
    p = os.path.join(d, "net.txt")
    inst.write(p)
    t = time.time()
    s = DDSolver(p, max_batch=4096, batch_nodes=int(bn), progress=2.0, max_rounds=int(os.environ.get("MAXR", "0")))
    t0 = time.time()
    try:
        sol, sec = s.start(known)
    except RuntimeError as e:
        sol, sec = None, time.time() - t0
        print(str(e), flush=True)
    print(json.dumps({"case": key, "batch": int(bn), "known": known, "ef": EF[key]["optimum"], "optimum": sol,
                      "seconds": sec, "pool": [s.eng.cuts_count(1), s.eng.cuts_count(0)],
                      "rounds": s.rounds, **s.counters}), flush=True)
    s.eng.close()
