"""Study tool: how well does the DD built for a record predict its relaxation time?
Relaxes the bench workload once with per-wave clocks, correlates each record's wave time
with what is known right after the build (DD nodes, arcs, layers), then times k_relax in
dispatch orders sorted by those sizes and by the measured time itself (the bound on
what a build-then-sweep split with longest-first dispatch could gain).

    SGUFP_RELAX_ORDER=0 python tools/cost_diag.py --nodes 8192
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


def timed(eng, batch, inc, reps=3):
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
    inst = instance.generate(instance.CONFIGS["C4"], 1, scenarios=1)
    d = tempfile.mkdtemp()
    net = os.path.join(d, "net.txt")
    inst.write(net)
    eng = E.Engine(net, 0, a.nodes)
    full = frontier.bfs_frontier(eng, a.nodes)
    eng.add_cuts(pools.synthetic_pool(inst, 16, 64, 1))
    eng.upload(full)
    eng.relax_async(pools.DOUBLE_MIN)
    eng.sync()
    st, ex, lb, ub, nc = eng.results_arrays()
    inc = float(np.percentile(ub[(st == 0) | (st == 3)], 40))
    eng.set_timing(True)
    eng.relax_async(inc)
    eng.sync()
    ticks, _ = eng.debug()
    t = ticks.astype(np.float64) / 100.0
    dn, da, dl, sw = (x.astype(np.float64) for x in eng.stats())
    st, ex, lb, ub, nc = eng.results_arrays()
    ph = eng.phases() / 100.0
    build = ph[:, 0]
    print(f"n={full.n} wave us mean {t.mean():.0f} cv {t.std() / t.mean():.2f} max/mean {t.max() / t.mean():.1f}")
    feats = {"dd nodes": dn, "dd arcs": da, "layers": dl, "nodes*layers": dn * dl, "build us": build,
             "sweeps (after)": sw, "gl": full.gl.astype(np.float64)}
    for k, v in feats.items():
        print(f"  corr(time, {k}) = {np.corrcoef(t, v)[0, 1]:+.3f}")
    print("status counts", dict(zip(*np.unique(st, return_counts=True))))
    res = {"batch order": timed(eng, full, inc)}
    for k in ("dd nodes", "dd arcs", "build us"):
        res[f"by {k} desc"] = timed(eng, E.batch_slice(full, np.argsort(-feats[k], kind="stable")), inc)
    res["by measured time desc"] = timed(eng, E.batch_slice(full, np.argsort(-t, kind="stable")), inc)
    print("k_relax ms: " + ", ".join(f"{k} {v:.2f}" for k, v in res.items()))
    eng.close()


if __name__ == "__main__":
    main()
