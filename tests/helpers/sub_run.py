"""Subprocess helper for tests/test_subproblem.py: run the device subproblem on seeded
random full matchings and save the per-(path, scenario) results.  The library is the one
SGUFP_LIB_PATH names (the verify build re-runs every warm Bellman-Ford cold)."""
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main(cfg, seed, S, n_paths, out):
    from sgufp_solver_amd import engine as E
    from sgufp_solver_amd import instance
    inst = instance.generate(instance.CONFIGS[cfg], seed, scenarios=S)
    inst.lb[:] = 0                       # feasible: full max-reward flows, many augmentations
    d = tempfile.mkdtemp(prefix="sgufp_subv_")
    path = os.path.join(d, "net.txt")
    inst.write(path)
    _, la, _ = E.probe_network(path)
    rng = np.random.default_rng(1000 + seed)
    paths = [instance.random_matching_path(inst, la, rng) for _ in range(n_paths)]
    eng = E.Engine(path, 0, 64)
    typ, rhs, rows, obj_mean = eng.subproblem(paths)
    st, obj, dual = eng.subproblem_detail(len(paths))
    eng.close()
    np.savez(out, typ=typ, rhs=rhs, rows=rows, obj_mean=obj_mean, st=st, obj=obj, dual=dual,
             lib=np.array(E.LIB_PATH))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), sys.argv[5])
