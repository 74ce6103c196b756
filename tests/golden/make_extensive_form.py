"""Extensive-form optima (oracle/extensive_form.py, HiGHS milp) of the seeded instances the
end-to-end B&B tests solve; written to tests/golden/extensive_form.json.

    python tests/golden/make_extensive_form.py [name ...]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle import extensive_form as ef  # noqa: E402
from sgufp_solver_amd import instance  # noqa: E402

# (config, seed, scenarios)
CASES = [("C1", 1, 1), ("C1", 2, 1), ("C1", 3, 1), ("C1", 4, 2), ("C1", 5, 3), ("C2", 1, 1), ("C2", 3, 2),
         # 64 scenarios, generated lower bounds (the closure study's instances between T4 and M1)
         ("P1", 1, 64), ("P1", 3, 64), ("P3", 2, 64), ("P3", 3, 64)]
# lower bounds 0 (suffix "z"): the 64-scenario end-to-end case of tests/test_bnb.py
CASES_LB0 = [("T4", 1, 64)]
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "extensive_form.json")


def key(cfg, seed, S):
    return f"{cfg}-{seed}-{S}"


def main(argv):
    data = json.load(open(OUT)) if os.path.exists(OUT) else {}
    for cfg, seed, S in CASES:
        k = key(cfg, seed, S)
        if argv and k not in argv:
            continue
        t = time.time()
        v = ef.solve(instance.generate(instance.CONFIGS[cfg], seed, scenarios=S))
        data[k] = {"optimum": v, "optimum_hex": v.hex(), "seconds": round(time.time() - t, 2)}
        print(k, data[k], flush=True)
        json.dump(data, open(OUT, "w"), indent=1, sort_keys=True)
    for cfg, seed, S in CASES_LB0:
        k = key(cfg, seed, S) + "z"
        if argv and k not in argv:
            continue
        inst = instance.generate(instance.CONFIGS[cfg], seed, scenarios=S)
        inst.lb[:] = 0
        t = time.time()
        v = ef.solve(inst)
        data[k] = {"optimum": v, "optimum_hex": v.hex(), "seconds": round(time.time() - t, 2)}
        print(k, data[k], flush=True)
        json.dump(data, open(OUT, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main(sys.argv[1:])
