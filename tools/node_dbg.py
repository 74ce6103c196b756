"""Relax a single golden-case node with the current library and print its outcome."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import golden_io  # noqa: E402
from sgufp_solver_amd import engine as E, pools  # noqa: E402

name, fname, idx = sys.argv[1], sys.argv[2], int(sys.argv[3])
case = [c for c in golden_io.manifest() if c["name"] == name][0]
run = [r for r in case["runs"] if r["file"] == fname][0]
d = golden_io.case_dir(name)
e = E.Engine(f"{d}/net.txt", 0, 256)
e.add_cuts(pools.read_pool(f"{d}/cuts.txt"))
nodes = pools.read_nodes(f"{d}/nodes.txt")
for batch in ([nodes[idx]], nodes):
    got = e.relax(batch, float.fromhex(run["incumbent"]))
    g = got[0] if len(batch) == 1 else got[idx]
    ticks, rinfo = e.debug()
    k = 0 if len(batch) == 1 else idx
    dn, da, dl, sw = e.stats()
    print(f"batch={len(batch)} status={g.status} exact={g.exact} ub={g.ub!r} children={len(g.children)} "
          f"sweeps={sw[k]} redo={int(rinfo[k]) & 0xFF} mirror={(int(rinfo[k]) >> 31) & 1}")
want = golden_io.parse_results_text(golden_io.read_golden(name, fname))[idx]
print(f"want status={want.status} ub={want.ub!r} children={len(want.children)}")
