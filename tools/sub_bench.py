"""Subproblem micro-benchmark (study tool): k_sub_scenario + k_sub_reduce over P random full
matchings of a generated instance, timed with the C ABI call (HBM-resident tables,
paths uploaded per call), and checked against a first run for determinism.

    python tools/sub_bench.py --cfg C3 --scenarios 64 --paths 26 --reps 3
"""
import argparse
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import subproblem_oracle as so  # noqa: E402
from sgufp_solver_amd import engine as E  # noqa: E402
from sgufp_solver_amd import instance  # noqa: E402
from tests.test_subproblem import _full_matching, _path_of  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfg", default="C3")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--scenarios", type=int, default=64)
    ap.add_argument("--paths", type=int, default=26)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--gen-lb", action="store_true")
    a = ap.parse_args()
    inst = instance.generate(instance.CONFIGS[a.cfg], a.seed, scenarios=a.scenarios)
    if not a.gen_lb:
        inst.lb[:] = 0
    d = tempfile.mkdtemp(prefix="sgufp_subb_")
    path = os.path.join(d, "net.txt")
    inst.write(path)
    L, la, vb = E.probe_network(path)
    net = so.from_instance(inst, la)
    rng = np.random.default_rng(7)
    paths = [_path_of(inst, net, _full_matching(net, rng, 1.0)) for _ in range(a.paths)]
    eng = E.Engine(path, 0, 64)
    ref = None
    for r in range(a.reps + 1):
        t0 = time.perf_counter()
        typ, rhs, rows, om = eng.subproblem(paths)
        dt = time.perf_counter() - t0
        st, obj, dual = eng.subproblem_detail(len(paths))
        if ref is None:
            ref = (typ.copy(), rhs.copy(), rows.copy(), obj.copy())
        else:
            assert (typ == ref[0]).all() and (rhs == ref[1]).all() and (rows == ref[2]).all() and (obj == ref[3]).all()
        print(f"rep {r}: {dt * 1e3:.2f} ms for {len(paths)} paths x {a.scenarios} scenarios "
              f"(types {np.bincount(typ + 1, minlength=3).tolist()}, status {np.bincount(st.ravel(), minlength=3).tolist()}, "
              f"obj sum {float(obj.sum()):.1f})", flush=True)
    eng.close()
    import hashlib
    h = hashlib.sha256()
    for x in ref:
        h.update(np.ascontiguousarray(x).tobytes())
    print(f"digest {h.hexdigest()[:16]}")


if __name__ == "__main__":
    main()
