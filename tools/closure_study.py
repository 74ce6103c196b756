"""Closing times of the device B&B on 64-scenario instances between T4 and M1 (generated lower
bounds kept), seeded with opt - 10 (main.cpp:75) and unseeded, against the HiGHS optimum of the
extensive form computed on the CPU beforehand.

    closure_study.py budget name arcs layers width deg f seed opt_hex [name ...]
"""
import json
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from sgufp_solver_amd import instance  # noqa: E402
from sgufp_solver_amd.pools import DOUBLE_MIN  # noqa: E402
from sgufp_solver_amd.solver import DDSolver  # noqa: E402


def main(argv):
    budget = float(argv[0])
    specs = argv[1:]
    for k in range(0, len(specs), 8):
        name, arcs, layers, width, deg, f, seed, opt_hex = specs[k:k + 8]
        cfg = instance.InstanceConfig(name, int(arcs), int(layers), int(width), int(deg), float(f), 64)
        inst = instance.generate(cfg, int(seed))
        opt = float.fromhex(opt_hex)
        path = os.path.join(tempfile.mkdtemp(prefix="sgufp_close_"), "net.txt")
        inst.write(path)
        for seeding in ("opt-10", "none"):
            known = opt - 10.0 if seeding == "opt-10" else DOUBLE_MIN
            s = DDSolver(path, max_batch=1024, verbose=False, round_seconds=5.0, time_budget=budget, progress=30.0)
            t0 = time.perf_counter()
            z = s.start_solver(known)
            sec = time.perf_counter() - t0
            rec = {"name": name, "seed": int(seed), "vbar": len(inst.vbar), "seeding": seeding, "complete": s.complete,
                   "solution": z, "opt": opt, "match": abs(z - opt) <= 1e-5 * max(1.0, abs(opt)), "seconds": round(sec, 2),
                   "rounds": s.rounds, "frontier_left": s.eng.frontier_size(), "counters": s.counters}
            s.eng.close()
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main(sys.argv[1:])
