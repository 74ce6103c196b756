"""Fixture case with a V-bar node of 20 out-arcs (state sets of 21 > 16 entries), produced by
the reference compiled in this container:

    make -C oracle && python tests/golden/make_wide.py

The generator's configs never give a V-bar node more than a handful of out-arcs, so neither
the relaxed nor the restricted fixtures exercised state sets wider than 16 (a coefficient
table of 4 cuts x 21 states is wider than one 64-lane wave).  Here: source -> 4 sources ->
4 feeders (V-bar) -> hub (V-bar, 20 out-arcs) -> 20 pre-sink nodes (V-bar) -> sink.  Everything else follows make_golden.py (getActualCut pools, frontier
from the reference's own LIFO expansion, per-incumbent NodeExplorer::process outcomes) and
make_restricted.py (RestrictedDDNew under the pool), appended to both manifests.  Only data
is committed."""
from __future__ import annotations

import gzip
import json
import os
import shutil
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)

from sgufp_solver_amd import instance, pools  # noqa: E402
import make_restricted as MR  # noqa: E402

REF = os.path.join(ROOT, "oracle", "_ref", "ref_dd")
DMIN = pools.DOUBLE_MIN
NAME = "w1_s1_wide"


def wide_instance(seed: int = 1) -> instance.Instance:
    # the hub sits next to the sink side, so its layers come early in the V-bar order (demand
    # points first, Network.cpp:132-186) and the last five (exactly expanded) layers belong
    # to the small feeders: a 21-state node there would expand to millions of DD nodes
    rng = np.random.Generator(np.random.PCG64(seed))
    src = [1, 2, 3, 4]
    feed = [5, 6, 7, 8]
    hub = 9
    pre = list(range(10, 30))
    sink = 30
    arcs = [(0, s) for s in src]
    for f in feed:
        for s in sorted(int(x) for x in rng.choice(len(src), size=2, replace=False)):
            arcs.append((src[s], f))
    for s in src:
        if not any(t == s for t, _ in arcs[len(src):]):
            arcs.append((s, feed[0]))
    arcs += [(f, hub) for f in feed]
    arcs += [(f, pre[int(rng.integers(0, len(pre)))]) for f in feed]
    arcs += [(hub, p) for p in pre] + [(p, sink) for p in pre]
    arcs = list(dict.fromkeys(arcs))
    order = rng.permutation(len(arcs))
    arcs = [arcs[i] for i in order]
    m = len(arcs)
    tails = np.array([a[0] for a in arcs], dtype=np.int32)
    heads = np.array([a[1] for a in arcs], dtype=np.int32)
    ub = rng.integers(5, 51, size=(m, 1)).astype(np.int32)
    lb = np.zeros((m, 1), dtype=np.int32)
    r = rng.integers(-5, 31, size=m).astype(np.int32)
    return instance.Instance(n=sink + 1, tails=tails, heads=heads, lb=lb, ub=ub, reward=r[:, None].copy(),
                             vbar=feed + [hub] + pre)


def gz(tmp):
    with open(tmp, "rb") as fi, gzip.open(tmp + ".gz", "wb", compresslevel=9) as fo:
        shutil.copyfileobj(fi, fo)
    os.remove(tmp)


def main():
    if not os.path.exists(REF):
        sys.exit("build oracle/_ref/ref_dd first (make -C oracle)")
    d = os.path.join(HERE, NAME)
    shutil.rmtree(d, ignore_errors=True)
    os.makedirs(d)
    inst = wide_instance()
    net = os.path.join(d, "net.txt")
    inst.write(net)
    pool = pools.synthetic_pool(inst, 4, 12, 4243)
    cuts = os.path.join(d, "cuts.txt")
    pools.write_pool(cuts, pool)
    empty = os.path.join(d, "_empty.txt")
    pools.write_pool(empty, [])
    nodes_path = os.path.join(d, "nodes.txt")
    MR.run([REF, "dfs", net, empty, DMIN.hex(), "120", nodes_path])
    os.remove(empty)
    nodes = pools.read_nodes(nodes_path)
    nodes = [pools.NodeRecord(0, DMIN, pools.DOUBLE_MAX, [], [])] + nodes
    pools.write_nodes(nodes_path, nodes)
    incs = [DMIN, -961.0, -912.0]   # quartile and median of the bounds at DMIN
    outs = []
    for k, inc in enumerate(incs):
        tmp = os.path.join(d, f"ref_{k}.txt")
        MR.run([REF, "relax", net, cuts, nodes_path, inc.hex(), tmp])
        gz(tmp)
        outs.append({"incumbent": inc.hex(), "file": f"ref_{k}.txt.gz"})
    MR.run([REF, "order", net, os.path.join(d, "order.txt")])
    mpath = os.path.join(HERE, "manifest.json")
    man = [c for c in json.load(open(mpath)) if c["name"] != NAME]
    man.append({"name": NAME, "config": "wide", "seed": 1, "scenarios": 1, "n_feas": 4, "n_opt": 12,
                "frontier": "dfs", "nodes": len(nodes), "runs": outs})
    with open(mpath, "w") as fh:
        json.dump(man, fh, indent=1)
    # restricted runs over the same records
    rd = os.path.join(HERE, "restricted", NAME)
    shutil.rmtree(rd, ignore_errors=True)
    os.makedirs(rd)
    pools.write_nodes(os.path.join(rd, "nodes.txt"), nodes)
    runs, k = [], 0
    for w in (4, 16, 128):
        tmp = os.path.join(rd, f"restricted_{k}.txt")
        MR.run([REF, "restricted", net, cuts, os.path.join(rd, "nodes.txt"), DMIN.hex(), str(w), tmp])
        lbs = sorted(lb for st, ex, lb, p in MR.parse(tmp) if st == 0 and lb > DMIN)
        gz(tmp)
        runs.append({"width": w, "incumbent": DMIN.hex(), "file": f"restricted_{k}.txt.gz"})
        k += 1
        if lbs:
            inc = lbs[len(lbs) // 2]
            tmp = os.path.join(rd, f"restricted_{k}.txt")
            MR.run([REF, "restricted", net, cuts, os.path.join(rd, "nodes.txt"), inc.hex(), str(w), tmp])
            gz(tmp)
            runs.append({"width": w, "incumbent": inc.hex(), "file": f"restricted_{k}.txt.gz"})
            k += 1
    rpath = os.path.join(HERE, "restricted_manifest.json")
    rman = [c for c in json.load(open(rpath)) if c["name"] != NAME]
    rman.append({"name": NAME, "source": NAME, "nodes": len(nodes), "deep": 0, "runs": runs})
    with open(rpath, "w") as fh:
        json.dump(rman, fh, indent=1)
    print(NAME, len(nodes), "nodes,", len(runs), "restricted runs")


if __name__ == "__main__":
    main()
