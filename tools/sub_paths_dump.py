#!/usr/bin/env python3
"""Study tool (GPU): dump the exact-leaf paths the device B&B sends to the scenario
subproblem, in solve order, for the warm-start study (tools/warm_study.cpp).

    python tools/sub_paths_dump.py --config C3 --seconds 15 --out gpurun_out/paths_c3.npz

Runs the seeded search (restricted-DD heuristic on the root, as bench.py's bnb_seeded leg)
with the round trace on and stores, per subproblem: round, record slot, path.
"""
import argparse
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
    ap.add_argument("--seconds", type=float, default=15.0)
    ap.add_argument("--out", required=True)
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
    eng.bnb_set_trace(True)
    root = NodeRecord(0, DOUBLE_MIN, DOUBLE_MAX, [], [])
    z = RestrictedExplorer(eng, a.width).incumbent([root], DOUBLE_MIN) if a.width else DOUBLE_MIN
    eng.frontier_clear()
    eng.frontier_push([root])
    t0 = time.perf_counter()
    rnd, rec, plen, flat = [], [], [], []
    r = 0
    diving = True
    while time.perf_counter() - t0 < a.seconds and eng.frontier_size():
        eng.bnb_set_limits(0, 5.0)
        z, st = eng.bnb_step(z, 64 if diving else a.batch)
        if st.exact:
            diving = False
        for sub in eng.bnb_trace(1):
            rnd.append(r)
            rec.append(sub[0])
            plen.append(len(sub[4]))
            flat.extend(sub[4])
        r += 1
        print(f"round {r} subproblems {len(rec)} frontier {eng.frontier_size()}", flush=True)
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    L = max(plen) if plen else 0
    paths = np.full((len(plen), L), -1, dtype=np.int16)
    o = 0
    for i, n in enumerate(plen):
        paths[i, :n] = flat[o:o + n]
        o += n
    layer_arcs = eng.processing_order()[0]
    np.savez_compressed(a.out, round=np.array(rnd, np.int32), record=np.array(rec, np.int32),
                        plen=np.array(plen, np.int32), paths=paths,
                        layer_arcs=np.asarray(layer_arcs, np.int32),
                        config=a.config, seed=a.seed)
    print(f"wrote {a.out}: {len(plen)} subproblem paths over {r} rounds", flush=True)
    eng.close()


if __name__ == "__main__":
    main()
