"""Study tool: does the order of the open nodes in a k_relax launch matter?  Builds the
bench workload (C4, 16F+64O pool, BFS frontier, 40th-percentile incumbent), relaxes it
once for per-node costs, then times k_relax with the frontier order, sorted by a record
proxy (global layer, ub) and sorted by the measured cost (an upper bound on what any
ordering can gain).

    python tools/order_diag.py --nodes 8192
"""
import argparse
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from sgufp_solver_amd import engine as E  # noqa: E402
from sgufp_solver_amd import frontier, instance, pools  # noqa: E402


def timed(eng, batch, inc, reps=5):
    eng.upload(batch)
    eng.set_timing(True)
    eng.relax_async(inc)
    eng.sync()
    ts = []
    for _ in range(reps):
        eng.relax_async(inc)
        eng.sync()
        ts.append(eng.last_timing()[0])
    return float(np.mean(ts))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=8192)
    a = ap.parse_args()
    inst = instance.generate(instance.CONFIGS["C4"], 1)
    d = tempfile.mkdtemp()
    net = os.path.join(d, "net.txt")
    inst.write(net)
    pool = pools.synthetic_pool(inst, 16, 64, 1)
    eng = E.Engine(net, 0, a.nodes)
    full = frontier.bfs_frontier(eng, a.nodes)
    eng.add_cuts(pool)
    probe = E.batch_slice(full, np.arange(min(1024, full.n)))
    eng.upload(probe)
    eng.relax_async(pools.DOUBLE_MIN)
    eng.sync()
    st, ex, lb, ub, nc = eng.results_arrays()
    fin = ub[(st == 0) | (st == 3)]
    inc = float(np.percentile(fin, 40))
    eng.upload(full)
    eng.relax_async(inc)
    eng.sync()
    dn, da, dl, sw = eng.stats()
    st, ex, lb, ub2, nc = eng.results_arrays()
    cost = sw * (14.0 * da + 8.0 * dn) + 6.0 * da
    n = full.n
    print(f"n={n} cost mean {cost.mean():.3g} cv {cost.std() / cost.mean():.2f} max/mean {cost.max() / cost.mean():.1f}")
    for q in range(8):
        sl = slice(q * n // 8, (q + 1) * n // 8)
        print(f"  eighth {q}: cost share {cost[sl].sum() / cost.sum():.3f}  mean gl {full.gl[sl].mean():.1f}  "
              f"mean sweeps {sw[sl].mean():.1f}")
    print("corr(cost, gl)", np.corrcoef(cost, full.gl)[0, 1], "corr(cost, ub)", np.corrcoef(cost, full.ub)[0, 1],
          "corr(cost, nstates)", np.corrcoef(cost, np.diff(full.states_off))[0, 1])
    base = timed(eng, full, inc)
    by_cost = timed(eng, E.batch_slice(full, np.argsort(-cost, kind="stable")), inc)
    by_ub = timed(eng, E.batch_slice(full, np.argsort(-full.ub, kind="stable")), inc)
    by_gl = timed(eng, E.batch_slice(full, np.argsort(full.gl, kind="stable")), inc)
    rnd = timed(eng, E.batch_slice(full, np.random.default_rng(0).permutation(n)), inc)
    print(f"k_relax ms: frontier order {base:.2f}  by measured cost {by_cost:.2f}  by ub desc {by_ub:.2f}  "
          f"by gl asc {by_gl:.2f}  random {rnd:.2f}")
    eng.close()


if __name__ == "__main__":
    main()
