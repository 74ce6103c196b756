"""Which single optimality cut prunes which bench node (post-F DD)?  Study for the
optimality-cut screening: hit rate of static cut rankings vs the reference order."""
import collections
import json
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from sgufp_solver_amd import engine as E  # noqa: E402
from sgufp_solver_amd import frontier, instance, pools  # noqa: E402

inst = instance.generate(instance.CONFIGS["C4"], 1, scenarios=1)
d = tempfile.mkdtemp()
net = f"{d}/net.txt"
inst.write(net)
pool = pools.synthetic_pool(inst, 16, 64, 1)
F = [c for c in pool if c.type == 1]
O = [c for c in pool if c.type == 0]
eng = E.Engine(net, 0, 4096)
fr = frontier.bfs_frontier(eng, 4096)
eng.add_cuts(pool)
eng.upload(fr)
eng.relax_async(pools.DOUBLE_MIN)
eng.sync()
st, ex, lb, ub, nc = eng.results_arrays()
inc = float(np.percentile(ub[(st == 0) | (st == 3)], 40))
eng.relax_async(inc)
eng.sync()
full, _, _, _, _ = eng.results_arrays()
_, _, _, sweeps = eng.stats()
print("full status", dict(zip(*np.unique(full, return_counts=True))), "sweeps mean", sweeps.mean(), flush=True)
hit = np.zeros((len(O), fr.n), dtype=bool)
for j, c in enumerate(O):
    eng.clear_cuts()
    eng.add_cuts(F + [c])
    eng.relax_async(inc)
    eng.sync()
    s, _, _, _, _ = eng.results_arrays()
    hit[j] = s == 2
pr = full == 2
print("pruned nodes", pr.sum(), "prunable by a single cut", (hit[:, pr].any(axis=0)).sum(), flush=True)
print("cuts pruning >0 nodes", (hit.sum(axis=1) > 0).sum(), "per-cut hits", sorted(hit.sum(axis=1).tolist(), reverse=True)[:20])


def ub_static(c):
    best = collections.defaultdict(float)
    for (i, q, jj, v) in c.coeff:
        best[(i, q)] = max(best[(i, q)], v)
    return c.rhs + sum(best.values())


def screens(order):
    need = []
    for n in np.where(pr)[0]:
        k = next((t for t, j in enumerate(order) if hit[j, n]), None)
        need.append(k + 1 if k is not None else -1)
    need = np.array(need)
    ok = need > 0
    return ok.mean(), need[ok].mean() if ok.any() else 0, np.percentile(need[ok], 90) if ok.any() else 0


ref_order = list(range(len(O)))[::-1]        # newest first
print("reference order: frac, mean screens, p90", screens(ref_order))
print("static UB order:", screens(list(np.argsort([ub_static(c) for c in O]))))
print("rhs order:", screens(list(np.argsort([c.rhs for c in O]))))
print("oracle (most hits first):", screens(list(np.argsort(-hit.sum(axis=1)))))
