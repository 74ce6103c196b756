"""Fixture of the device B&B under its own Benders pool, CPU side.

    bash-on-the-box: python tools/dump_bnb_fixture.py --config C3 --seed 1 --width 64 --out gpurun_out/bnb_c3_seeded
    here:            make -C oracle && python tests/golden/make_bnb_golden.py gpurun_out/bnb_c3_seeded

The GPU run (tools/dump_bnb_fixture.py) writes what a round of the device search would see
after it reached exact leaves: the network, the global pool -- every cut made by the
device scenario subproblem (k_sub_scenario, the reference's GuroSolver::solveSubProblem,
grb.cpp:236-281) in insertion order --, the records the next round pops and the incumbent,
plus the cuts of one exact record's refinement loop (NodeExplorer.cpp:957-969).  This
script runs the reference's own RelaxedDDNew (oracle/_ref/ref_dd, built from
/root/reference) on those inputs -- "relax" at the round's incumbent and at DOUBLE_MIN,
"refine" with the loop's cuts -- and files the case in manifest.json / refine_manifest.json
like make_golden.py's cases.  The pool is stored gzipped (cuts.txt.gz).  Only data lands in
the repository.
"""
from __future__ import annotations

import gzip
import json
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from sgufp_solver_amd import pools  # noqa: E402

REF = os.path.join(ROOT, "oracle", "_ref", "ref_dd")


def gz(src, dst):
    with open(src, "rb") as fi, gzip.open(dst, "wb", compresslevel=9) as fo:
        fo.write(fi.read())


def run(cmd):
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"{cmd}: {r.stderr}")


def main():
    src = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "bnb_c3_seeded")
    with open(os.path.join(src, "meta.json")) as fh:
        meta = json.load(fh)
    name = f"bnb_{meta['config'].lower()}_s{meta['seed']}"
    d = os.path.join(HERE, name)
    shutil.rmtree(d, ignore_errors=True)
    os.makedirs(d)
    for f in ("net.txt", "nodes.txt", "extra_cuts.txt"):
        shutil.copy(os.path.join(src, f), os.path.join(d, f))
    tmp = os.path.join(d, "_cuts.txt")
    shutil.copy(os.path.join(src, "cuts.txt"), tmp)
    net, nodes, extra = (os.path.join(d, f) for f in ("net.txt", "nodes.txt", "extra_cuts.txt"))
    z = float.fromhex(meta["incumbent"])
    runs = []
    for k, inc in enumerate([z, pools.DOUBLE_MIN]):
        out = os.path.join(d, f"ref_{k}.txt")
        run([REF, "relax", net, tmp, nodes, inc.hex(), out])
        gz(out, out + ".gz")
        os.remove(out)
        runs.append({"incumbent": inc.hex(), "file": f"ref_{k}.txt.gz"})
    refine = []
    if meta.get("extra_cuts", 0) > 0:
        out = os.path.join(d, "refine_0.txt")
        run([REF, "refine", net, tmp, nodes, z.hex(), extra, out])
        gz(out, out + ".gz")
        os.remove(out)
        refine.append({"incumbent": z.hex(), "file": "refine_0.txt.gz"})
    run([REF, "order", net, os.path.join(d, "order.txt")])
    gz(tmp, os.path.join(d, "cuts.txt.gz"))
    os.remove(tmp)
    entry = {"name": name, "config": meta["config"], "seed": meta["seed"], "scenarios": meta["scenarios"],
             "n_feas": meta["n_feas"], "n_opt": meta["n_opt"], "frontier": "device-bnb",
             "nodes": meta["records"], "runs": runs,
             "source": "device B&B pool and frontier (tools/dump_bnb_fixture.py, "
                       f"heuristic width {meta['heuristic_width']}, incumbent {meta['incumbent']})"}
    mp = os.path.join(HERE, "manifest.json")
    with open(mp) as fh:
        manifest = [c for c in json.load(fh) if c["name"] != name]
    manifest.append(entry)
    with open(mp, "w") as fh:
        json.dump(manifest, fh, indent=1)
    rp = os.path.join(HERE, "refine_manifest.json")
    with open(rp) as fh:
        rm = json.load(fh)
    rm.pop(name, None)
    if refine:
        rm[name] = refine
    with open(rp, "w") as fh:
        json.dump(rm, fh, indent=1)
    print(name, entry["nodes"], "records,", meta["n_feas"] + meta["n_opt"], "cuts,", meta["extra_cuts"], "loop cuts")


if __name__ == "__main__":
    main()
