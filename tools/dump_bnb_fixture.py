#!/usr/bin/env python3
"""GPU side of the device-B&B fixture (tests/golden/make_bnb_golden.py is the CPU side).

Runs the device search (sgufp_bnb_step) on a seeded instance for a few rounds, then writes
what the next round would see -- the network, the pool the subproblem built (rows as
(i, q, j, v) cuts, F list then O list in insertion order), a sample of the records the next
round pops, the incumbent -- and the cuts of one exact record's refinement loop replayed on
the device (oracle/bnb_parity.refine_replay), under <out>/.  The reference's outputs for
these inputs are generated in the container (ref_dd relax / refine), never on the box.

    python tools/dump_bnb_fixture.py --config C3 --seed 1 --width 64 --rounds 8 --out gpurun_out/bnb_c3
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from oracle import bnb_parity as bp  # noqa: E402
from sgufp_solver_amd import engine as E  # noqa: E402
from sgufp_solver_amd import instance, pools  # noqa: E402
from sgufp_solver_amd.pools import DOUBLE_MAX, DOUBLE_MIN, NodeRecord  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--width", type=int, default=64)
    ap.add_argument("--rounds", type=int, default=3, help="rounds after the first subproblem")
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--records", type=int, default=96)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    inst = instance.generate(instance.CONFIGS[a.config], a.seed)
    inst.lb[:] = 0
    net = os.path.join(a.out, "net.txt")
    inst.write(net)
    eng = E.Engine(net, 0, max(a.batch, a.records))
    root = NodeRecord(0, DOUBLE_MIN, DOUBLE_MAX, [], [])
    z = DOUBLE_MIN
    if a.width:
        from sgufp_solver_amd.restricted import RestrictedExplorer
        z = RestrictedExplorer(eng, a.width).incumbent([root], z)
    eng.frontier_clear()
    eng.frontier_push([root])
    # dive until the batch the next round pops holds exact records (refinement loops), then
    # a.rounds more rounds so that the pool holds the subproblem's cuts
    exact_seen, extra_rounds = False, 0
    for _ in range(400):
        eng.bnb_set_limits(2, 5.0)      # two refinement iterations per round: a pool of hundreds
        z, st = eng.bnb_step(z, a.batch)
        exact_seen = exact_seen or st.subproblems > 0
        if exact_seen:
            extra_rounds += 1
            if extra_rounds >= a.rounds:
                break
    pool = bp.pool_of(eng)
    top = bp.snapshot_top(eng, max(a.records, 1))
    recs = E.batch_to_records(top)
    pools.write_pool(os.path.join(a.out, "cuts.txt"), pool)
    pools.write_nodes(os.path.join(a.out, "nodes.txt"), recs)
    # one exact record's refinement loop with the subproblem's own cuts
    res = eng.relax(recs, z)
    eng.close()
    exact = [k for k, r in enumerate(res) if r.status == E.NEEDS_SUBPROBLEM]
    extra = []
    if exact:
        pe = E.Engine(net, 0, 4)
        bp.load_pool(pe, pool)
        extra, states = bp.refine_replay(pe, recs[exact[0]], z, 16)
        pe.close()
    pools.write_pool(os.path.join(a.out, "extra_cuts.txt"), extra)
    meta = {"config": a.config, "seed": a.seed, "scenarios": int(inst.scenarios), "heuristic_width": a.width,
            "rounds": a.rounds, "batch": a.batch, "incumbent": z.hex(), "n_feas": sum(c.type == 1 for c in pool),
            "n_opt": sum(c.type == 0 for c in pool), "records": len(recs), "exact_records": exact,
            "extra_cuts": len(extra),
            "status_counts": {str(k): int(v) for k, v in zip(*np.unique([r.status for r in res], return_counts=True))}}
    with open(os.path.join(a.out, "meta.json"), "w") as fh:
        json.dump(meta, fh, indent=1)
    print(json.dumps(meta))


if __name__ == "__main__":
    main()
