"""Subprocess helper for tests/test_subproblem.py: run the device subproblem on seeded
random full matchings and save the per-(path, scenario) results.  The library is the one
SGUFP_LIB_PATH names (the verify build re-runs every warm Bellman-Ford cold, and every warm
start's repair cold).

    sub_run.py cfg seed S n_paths out.npz [warm | warmgen]

warm: the paths are solved cold into ring slots 0 .. n-1, then B&B-like neighbours of them
(the decisions of the last DD layers redrawn, as the exact leaves of one cutset differ) are
solved warm from those slots and, for comparison, cold.  warmgen: the same with the
generator's lower bounds kept (64-bit-key kernels; some scenarios infeasible)."""
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def valid_path(path) -> bool:
    used = set()
    for d in path:
        if d >= 0:
            if d in used:
                return False
            used.add(d)
    return True


def neighbour(inst, la, base, rng, k):
    """base with the decisions of its last k layers redrawn (a valid matching)."""
    from sgufp_solver_amd import instance
    for _ in range(200):
        q = instance.random_matching_path(inst, la, rng)
        cand = list(base[:len(base) - k]) + list(q[len(base) - k:])
        if valid_path(cand) and cand != list(base):
            return cand
    return list(base)


def main(cfg, seed, S, n_paths, out, mode=""):
    from sgufp_solver_amd import engine as E
    from sgufp_solver_amd import instance
    inst = instance.generate(instance.CONFIGS[cfg], seed, scenarios=S)
    if mode != "warmgen":
        inst.lb[:] = 0                   # feasible: full max-reward flows, many augmentations
    d = tempfile.mkdtemp(prefix="sgufp_subv_")
    path = os.path.join(d, "net.txt")
    inst.write(path)
    _, la, _ = E.probe_network(path)
    rng = np.random.default_rng(1000 + seed)
    paths = [instance.random_matching_path(inst, la, rng) for _ in range(n_paths)]
    eng = E.Engine(path, 0, 64)
    res = {}
    if mode in ("warm", "warmgen"):
        n = n_paths
        eng.subproblem(paths, [-1] * n, list(range(n)))
        res["seed_st"], res["seed_obj"], _ = eng.subproblem_detail(n)
        nb = [neighbour(inst, la, p, rng, 7 + 3 * (k % 3)) for k, p in enumerate(paths)]
        # one unrelated path starts from a far donor too
        nb[-1] = instance.random_matching_path(inst, la, rng)
        typ, rhs, rows, obj_mean = eng.subproblem(nb, list(range(n)), [n + k for k in range(n)])
        st, obj, dual = eng.subproblem_detail(n)
        res["warm_aug"], res["warm_passes"] = eng.subproblem_stats(n)
        ctyp, crhs, crows, cobj_mean = eng.subproblem(nb)
        res["cold_st"], res["cold_obj"], res["cold_dual"] = eng.subproblem_detail(n)
        res["cold_aug"], res["cold_passes"] = eng.subproblem_stats(n)
        res["cold_typ"], res["cold_obj_mean"] = ctyp, cobj_mean
        res["cold_rhs"], res["cold_rows"] = crhs, crows
        res["paths"] = np.array(nb, dtype=np.int16)
    else:
        typ, rhs, rows, obj_mean = eng.subproblem(paths)
        st, obj, dual = eng.subproblem_detail(len(paths))
    eng.close()
    np.savez(out, typ=typ, rhs=rhs, rows=rows, obj_mean=obj_mean, st=st, obj=obj, dual=dual,
             lib=np.array(E.LIB_PATH), **res)


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), sys.argv[5],
         sys.argv[6] if len(sys.argv) > 6 else "")
