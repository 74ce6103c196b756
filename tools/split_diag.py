"""Study tool: would a build+feasibility+screen / exact-optimality split of k_relax pack
better?  Needs a library built from dd_kernels.hip with the screen-margin diagnostics
(phase slot 7 = ticks at the end of the screen, slot 6 = screen bound - incumbent as f64
bits; see the round-2 notes in DESIGN.md).  Simulates list scheduling of the measured
per-record wave times on 2048 wave slots: one launch in the current pseudo-random order
versus two launches (all records up to the screen, then the survivors' exact phase
ordered by a predictor).

    SGUFP_LIB_PATH=... python tools/split_diag.py --nodes 8192
"""
import argparse
import heapq
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from sgufp_solver_amd import engine as E  # noqa: E402
from sgufp_solver_amd import frontier, instance, pools  # noqa: E402

SLOTS = 2048


def makespan(costs):
    h = [0.0] * SLOTS
    for c in costs:
        t = heapq.heappop(h)
        heapq.heappush(h, t + c)
    return max(h)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=8192)
    a = ap.parse_args()
    inst = instance.generate(instance.CONFIGS["C4"], 1, scenarios=1)
    d = tempfile.mkdtemp()
    net = os.path.join(d, "net.txt")
    inst.write(net)
    eng = E.Engine(net, 0, a.nodes)
    fr = frontier.bfs_frontier(eng, a.nodes)
    eng.add_cuts(pools.synthetic_pool(inst, 16, 64, 1))
    eng.upload(fr)
    eng.relax_async(pools.DOUBLE_MIN)
    eng.sync()
    st, ex, lb, ub, nc = eng.results_arrays()
    inc = float(np.percentile(ub[(st == 0) | (st == 3)], 40))
    eng.set_timing(True)
    for _ in range(2):
        eng.relax_async(inc)
        eng.sync()
    print(f"k_relax {eng.last_timing()[0]:.2f} ms")
    ticks, _ = eng.debug()
    t = ticks.astype(np.float64) / 100.0
    ph = eng.phases()
    tscr = ph[:, 7].astype(np.float64) / 100.0
    margin = ph[:, 6].astype(np.uint64).view(np.float64)
    st, ex, lb, ub, nc = eng.results_arrays()
    dn, da, dl, sw = (x.astype(np.float64) for x in eng.stats())
    surv = (tscr > 0) & (t - tscr > 50.0)   # screened and not proven by the screen
    screened = tscr > 0
    print(f"n={len(t)} screened {screened.sum()} survivors of the screen {surv.sum()}; wave us mean {t.mean():.0f}")
    b = np.where(surv, t - tscr, 0.0)
    acost = np.where(surv, tscr, t)
    print(f"phase A us mean {acost.mean():.0f}, phase B us mean over survivors {b[surv].mean():.0f}")
    for k, v in {"margin": margin, "ub": fr.ub, "dd arcs": da, "tscr": tscr}.items():
        m = surv & np.isfinite(v)
        print(f"  corr(B, {k}) over survivors = {np.corrcoef(b[m], v[m])[0, 1]:+.3f}")
    rng = np.random.default_rng(0)
    perm = rng.permutation(len(t))
    one = makespan(t[perm])
    lpt = makespan(np.sort(t)[::-1])
    A = makespan(acost[perm])
    bs = b[surv]
    res = {"one launch random": one, "one launch LPT (measured)": lpt}
    for k, key in {"B by margin desc": -margin[surv], "B random": rng.random(bs.size),
                   "B LPT (measured)": -bs}.items():
        res[f"A + {k}"] = A + makespan(bs[np.argsort(key, kind="stable")])
    for k, v in res.items():
        print(f"  {k}: {v / 1e3:.2f} ms")
    eng.close()


if __name__ == "__main__":
    main()
