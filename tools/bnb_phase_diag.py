#!/usr/bin/env python3
"""Where k_relax spends a B&B record's time under a grown Benders pool (GPU, lib_prof).

    SGUFP_LIB_PATH=sgufp_solver_amd/lib_prof/libsgufp_hip.so python tools/bnb_phase_diag.py --pool 20000

Runs the seeded device search until the pool holds --pool cuts, then relaxes the batch the
next round would pop (the staged-batch path, same kernel) and prints, per status: records,
global layer, DD size, exactness, cuts swept, wave time and the k_relax phase split (build,
narrow sweep, tail layers, last layer, post / replay, redo, finish, epilog).
"""
import argparse
import json
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--width", type=int, default=64)
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--pool", type=int, default=20000)
    a = ap.parse_args()
    from oracle import bnb_parity as bp
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
    root = NodeRecord(0, DOUBLE_MIN, DOUBLE_MAX, [], [])
    z = RestrictedExplorer(eng, a.width).incumbent([root], DOUBLE_MIN) if a.width else DOUBLE_MIN
    eng.frontier_clear()
    eng.frontier_push([root])
    diving = True
    for _ in range(2000):
        if eng.cuts_count(0) + eng.cuts_count(1) >= a.pool or not eng.frontier_size():
            break
        eng.bnb_set_limits(0, 5.0)
        z, st = eng.bnb_step(z, 64 if diving else a.batch)
        diving = diving and not st.exact
    snap = bp.snapshot_top(eng, a.batch)
    eng.set_timing(True)
    eng.upload(snap)
    eng.relax_async(z)
    eng.sync()
    ms = eng.last_timing()[0]
    st, ex, lb, ub, nc = eng.results_arrays()
    dn, da, dl, sw = eng.stats()
    ticks, redo = eng.debug()
    ph = eng.phases() / 100.0
    us = ticks / 100.0
    names = ["build", "narrow", "tail", "last", "post", "redo", "finish", "epilog"]
    out = {"pool": eng.cuts_count(0) + eng.cuts_count(1), "incumbent": z, "records": int(snap.n),
           "k_relax_ms": round(ms, 2), "wave_us_sum_per_2048": round(float(us.sum()) / 2048 / 1e3, 2), "by_status": {}}
    gl = snap.gl.astype(np.int64)
    for s in np.unique(st):
        m = st == s
        out["by_status"][int(s)] = {
            "n": int(m.sum()), "gl_mean": round(float(gl[m].mean()), 1), "exact": int(ex[m].sum()),
            "dd_nodes_mean": round(float(dn[m].mean()), 1), "dd_layers_mean": round(float(dl[m].mean()), 1),
            "sweeps_mean": round(float(sw[m].mean()), 1), "wave_us_mean": round(float(us[m].mean()), 1),
            "us_per_sweep": round(float(np.mean(us[m] / np.maximum(sw[m], 1))), 3),
            "redo_mean": round(float((redo[m] & 0xFF).mean()), 2),
            "phase_us": {nm: round(float(ph[m, k].mean()), 1) for k, nm in enumerate(names)}}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
