"""Golden traces of the RelaxedDDNew surface (DD.h:797-808), call by call.

    make -C oracle               # oracle/_ref/ref_dd from /root/reference
    python tests/golden/make_dd_api.py

For a few fixture cases (their network, pool and first records) and incumbents, the
reference's own RelaxedDDNew is driven by `ref_dd api` (oracle/ref_driver.cpp): buildTree,
every pool cut newest first with the value each apply call returns, getSolution after every
4th cut and at the end, and getCutset(ub) of a non-exact tree.  One run per case uses an
empty pool: buildTree(root) + getCutset(DOUBLE_MAX), what DDSolver::startSolver does
(DDSolver.cpp:788-791).  Only the data lands in tests/golden/dd_api/.
"""
from __future__ import annotations

import gzip
import json
import os
import shutil
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from sgufp_solver_amd import pools  # noqa: E402

REF = os.path.join(ROOT, "oracle", "_ref", "ref_dd")
OUT = os.path.join(HERE, "dd_api")
DMIN = pools.DOUBLE_MIN
# case, records taken, incumbents
CASES = [
    ("c1_s1_bfs", 40, [DMIN, 0.0]),
    ("c2_s2_dfs", 40, [DMIN, 300.0]),
    ("c2_s5_feas_only", 40, [DMIN]),
    ("c3_s1_dfs", 32, [DMIN, 300.0]),
    ("c3_s4_dfs", 32, [300.0]),
    ("w1_s1_wide", 24, [DMIN]),
]


def run_api(net, cuts, nodes, inc, out):
    r = subprocess.run([REF, "api", net, cuts, nodes, inc.hex(), out], capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(r.stderr)


def main():
    os.makedirs(OUT, exist_ok=True)
    man = []
    tmp = tempfile.mkdtemp()
    for name, take, incs in CASES:
        d = os.path.join(HERE, name)
        nodes = pools.read_nodes(os.path.join(d, "nodes.txt"))[:take]
        root = pools.NodeRecord(0, DMIN, pools.DOUBLE_MAX, [], [])
        sel = os.path.join(OUT, f"{name}_nodes.txt")
        pools.write_nodes(sel, [root] + nodes)
        empty = os.path.join(tmp, "empty.txt")
        with open(empty, "w") as fh:
            fh.write("0\n")
        runs = []
        for k, inc in enumerate(incs + [None]):
            cuts = os.path.join(d, "cuts.txt") if inc is not None else empty
            fname = f"{name}_{k}.txt.gz"
            raw = os.path.join(tmp, fname[:-3])
            run_api(os.path.join(d, "net.txt"), cuts, sel, DMIN if inc is None else inc, raw)
            with open(raw, "rb") as fi, gzip.open(os.path.join(OUT, fname), "wb") as fo:
                shutil.copyfileobj(fi, fo)
            runs.append({"incumbent": (DMIN if inc is None else inc).hex(), "pool": "cuts.txt" if inc is not None else "",
                         "file": fname})
        man.append({"name": name, "nodes": f"{name}_nodes.txt", "runs": runs})
    with open(os.path.join(OUT, "manifest.json"), "w") as fh:
        json.dump(man, fh, indent=1)
    print(f"wrote {len(man)} cases to {OUT}")


if __name__ == "__main__":
    main()
