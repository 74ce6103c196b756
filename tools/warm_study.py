#!/usr/bin/env python3
"""Study tool (CPU): feed the B&B's subproblem paths (tools/sub_paths_dump.py) to
tools/warm_study.cpp and print its counts.

    python tools/warm_study.py gpurun_out/r05a_paths_c3.npz --s0 0 --ns 4 --max-paths 300
"""
import argparse
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("npz")
    ap.add_argument("--s0", type=int, default=0)
    ap.add_argument("--ns", type=int, default=2)
    ap.add_argument("--max-paths", type=int, default=200)
    ap.add_argument("--first", type=int, default=0, help="skip the first paths")
    ap.add_argument("--mode", choices=["path", "scen", "nearest"], default="path",
                    help="path: warm from the previous path (same scenario); scen: from the previous scenario")
    ap.add_argument("--order", choices=["solve", "record"], default="solve",
                    help="solve: the B&B's order; record: grouped by (round, record)")
    a = ap.parse_args()
    from sgufp_solver_amd import instance
    z = np.load(a.npz)
    inst = instance.generate(instance.CONFIGS[str(z["config"])], int(z["seed"]))
    inst.lb[:] = 0
    idx = np.arange(len(z["plen"]))[a.first:]
    if a.order == "record":
        idx = idx[np.lexsort((idx, z["record"][idx], z["round"][idx]))]
    idx = idx[:a.max_paths]
    exe = os.path.join(tempfile.gettempdir(), "warm_study")
    src = os.path.join(ROOT, "tools", "warm_study.cpp")
    if not os.path.exists(exe) or os.path.getmtime(exe) < os.path.getmtime(src):
        subprocess.run(["g++", "-O2", "-std=c++17", src, "-o", exe], check=True)
    S = inst.scenarios
    lines = [f"{inst.n} {inst.m} {S}"]
    for e in range(inst.m):
        parts = [str(int(inst.tails[e])), str(int(inst.heads[e]))]
        for s in range(S):
            parts += ["0", str(int(inst.ub[e, s])), str(int(inst.reward[e, s]))]
        lines.append(" ".join(parts))
    lines.append(f"{len(inst.vbar)} " + " ".join(str(v) for v in inst.vbar))
    la = z["layer_arcs"]
    lines.append(f"{len(la)} " + " ".join(str(int(x)) for x in la))
    lines.append(str(len(idx)))
    for i in idx:
        n = int(z["plen"][i])
        lines.append(f"{int(z['record'][i])} {n} " + " ".join(str(int(x)) for x in z["paths"][i, :n]))
    fin = os.path.join(tempfile.gettempdir(), "warm_study_in.txt")
    with open(fin, "w") as fh:
        fh.write("\n".join(lines) + "\n")
    r = subprocess.run([exe, fin, str(a.s0), str(a.ns), str(len(idx)), a.mode], capture_output=True, text=True)
    sys.stdout.write(r.stdout)
    sys.stderr.write(r.stderr)
    sys.exit(r.returncode)


if __name__ == "__main__":
    main()
