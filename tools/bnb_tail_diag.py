#!/usr/bin/env python3
"""Where the device B&B's round time goes (GPU; profiling library for per-wave ticks).

    SGUFP_LIB_PATH=sgufp_solver_amd/lib_prof/libsgufp_hip.so python tools/bnb_tail_diag.py --config C3 --seconds 20

Runs the seeded search (restricted-DD heuristic of --width on the root, as bench.py's
bnb_seeded leg) and, per round: wall time, k_relax launch time (hipEvents), the popped
records' wave times (wall_clock64 ticks, 100 MHz) by status, cuts swept, and how full the
launch kept the GPU (sum of wave times / (launch time x resident wave slots)).
"""
import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--width", type=int, default=64)
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--seconds", type=float, default=20.0)
    ap.add_argument("--round-seconds", type=float, default=5.0)
    ap.add_argument("--slots", type=int, default=2048, help="resident k_relax waves (2 per SIMD x 1024 SIMDs)")
    ap.add_argument("--round-iters", type=int, default=0)
    ap.add_argument("--out", default=None)
    ap.add_argument("--gl-hist", action="store_true", help="histogram of the DD layers of the exact survivors")
    ap.add_argument("--no-trace", action="store_true", help="search without the round trace (as the bench legs run)")
    a = ap.parse_args()
    from sgufp_solver_amd import engine as E
    from sgufp_solver_amd import instance
    from sgufp_solver_amd.pools import DOUBLE_MAX, DOUBLE_MIN, NodeRecord
    from sgufp_solver_amd.restricted import RestrictedExplorer
    inst = instance.generate(instance.CONFIGS[a.config], a.seed)
    inst.lb[:] = 0
    d = tempfile.mkdtemp()
    net = os.path.join(d, "net.txt")
    inst.write(net)
    eng = E.Engine(net, 0, a.batch)
    eng.set_timing(True)
    eng.bnb_set_trace(not a.no_trace)
    root = NodeRecord(0, DOUBLE_MIN, DOUBLE_MAX, [], [])
    z = RestrictedExplorer(eng, a.width).incumbent([root], DOUBLE_MIN) if a.width else DOUBLE_MIN
    eng.frontier_clear()
    eng.frontier_push([root])
    t0 = time.perf_counter()
    t_hist = {}
    rows = []
    seen_paths = {}
    dup = 0
    diving = True
    while time.perf_counter() - t0 < a.seconds and eng.frontier_size():
        eng.bnb_set_limits(a.round_iters, a.round_seconds)
        b = 64 if diving else a.batch
        gls = None
        if a.gl_hist:
            fs = eng.frontier_size()
            nb = min(b, fs)
            gls = eng.frontier_peek(fs - nb, nb).gl.astype(np.int64)
        tr = time.perf_counter()
        z, st = eng.bnb_step(z, b)
        wall = time.perf_counter() - tr
        if st.exact:
            diving = False
        n = int(st.popped)
        waves = eng.bnb_trace(3) if not a.no_trace else []
        popped = eng.bnb_trace(0) if not a.no_trace else []
        for sub in (eng.bnb_trace(1) if not a.no_trace else []):
            key = hash(tuple(sub[4]))
            dup += 1 if key in seen_paths else 0
            seen_paths[key] = 1
        ticks = np.array([w[3] for w in waves])
        redo = np.array([w[1] for w in waves])
        sw = np.array([w[2] for w in waves])
        stt = np.array([p[1] for p in popped])
        if gls is not None and len(gls) == len(stt):
            # DD layers of the records that reached the subproblem (exact DDs): total - gl + 1
            for t in (eng.info.total_layers - gls[stt == 3] + 1):
                t_hist[int(t)] = t_hist.get(int(t), 0) + 1
        ms = ticks / 1e5
        launch = float(st.ms_relax)
        fill = float(ms.sum() / max(1e-9, launch * min(a.slots, max(n, 1)))) if launch else 0.0
        by = {}
        for s in np.unique(stt):
            m = stt == s
            by[int(s)] = {"n": int(m.sum()), "wave_ms_mean": round(float(ms[m].mean()), 3),
                          "wave_ms_max": round(float(ms[m].max()), 3), "sweeps_mean": round(float(sw[m].mean()), 1),
                          "redo_mean": round(float(redo[m].mean()), 2), "redo_frac": round(float((redo[m] > 0).mean()), 3)}
        rows.append({"round": len(rows), "popped": n, "wall_ms": round(wall * 1e3, 2), "k_relax_ms": round(launch, 2),
                     "wave_ms_max": round(float(ms.max()), 3) if len(ms) else 0.0,
                     "wave_ms_mean": round(float(ms.mean()), 3) if len(ms) else 0.0,
                     "fill": round(fill, 3), "subproblems": int(st.subproblems), "iters": int(st.refine_iters),
                     "pool": eng.cuts_count(0) + eng.cuts_count(1), "resumed": int(st.resumed),
                     "deferred": int(st.deferred), "by_status": by})
        print(json.dumps(rows[-1]), flush=True)
    tot = {k: sum(r[k] for r in rows) for k in ("wall_ms", "k_relax_ms", "popped", "subproblems", "resumed")}
    tot["relaxations_per_s"] = round(tot["popped"] / (tot["wall_ms"] / 1e3), 1)
    tot["k_relax_share"] = round(tot["k_relax_ms"] / tot["wall_ms"], 3)
    tot["duplicate_subproblem_paths"] = dup
    tot["round_iters"] = a.round_iters
    if a.gl_hist:
        tot["exact_dd_layers_hist"] = dict(sorted(t_hist.items()))
    print(json.dumps({"total": tot}))
    if a.out:
        with open(a.out, "w") as fh:
            json.dump({"rounds": rows, "total": tot}, fh)


if __name__ == "__main__":
    main()
