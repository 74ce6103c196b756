"""Golden fixtures for the restricted DD (Inavap::RestrictedDDNew, DD.cpp:3090-3505, under the
cut phases of NodeExplorer::processX3, NodeExplorer.cpp:605-656), produced by the reference
compiled in this container:

    make -C oracle && python tests/golden/make_restricted.py

For each case: the network and cut pool of an existing fixture case, its open nodes plus
deep records (prefixes of the restricted DDs' own max paths that stop at one of the last
state-update layers, so that exact restricted trees and short restricted tails occur), and
per (width, incumbent) the reference's outcome (restricted_<k>.txt.gz, oracle/_ref/ref_dd
"restricted").  The second incumbent of a case is the median bound of the first run, so
both outcomes occur.  Only data is committed."""
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
DMIN = pools.DOUBLE_MIN
DMAX = pools.DOUBLE_MAX

CASES = [("c1_s2_dfs", [4, 16, 128]), ("c2_s4_opt_only", [8, 128]), ("c2_s5_feas_only", [128]), ("c3_s1_dfs", [16, 128])]


def run(cmd):
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"{cmd}: {r.stderr}")


def update_sets(net_path):
    """stateUpdateMap of the reference loader (Network.cpp:100-121): layer -> sorted states."""
    from sgufp_solver_amd import engine as E
    L, la, vb = E.probe_network(net_path)
    with open(net_path) as fh:
        tok = fh.read().split()
    n, m, S = int(tok[0]), int(tok[1]), int(tok[2])
    pos = 3
    tails, heads = [], []
    for _ in range(m):
        tails.append(int(tok[pos])); heads.append(int(tok[pos + 1]))
        pos += 2 + 3 * S
    outs = {}
    for a in range(m):
        outs.setdefault(tails[a], []).append(a)
    ups, i = {}, 0
    for q in vb:
        q = int(q)
        ups.setdefault(i, sorted(set(outs.get(q, [])) | {-1}))
        i += sum(1 for a in range(m) if heads[a] == q)
    return L, ups


def parse(path):
    """restricted outputs: per node (status, exact, lb, path)"""
    with gzip.open(path, "rt") if path.endswith(".gz") else open(path) as fh:
        lines = fh.read().splitlines()
    out, k = [], 1
    while k < len(lines):
        q = lines[k].split()
        k += 1
        st, ex, lb, nc, np_ = int(q[1]), int(q[2]), float.fromhex(q[3]), int(q[4]), int(q[5])
        path = [int(x) for x in lines[k].split()] if np_ else []
        k += (1 if np_ else 0) + nc
        out.append((st, ex, lb, path))
    return out


def main():
    out_root = os.path.join(HERE, "restricted")
    os.makedirs(out_root, exist_ok=True)
    manifest = []
    for name, widths in CASES:
        src = os.path.join(HERE, name)
        d = os.path.join(out_root, name)
        os.makedirs(d, exist_ok=True)
        net, cuts = os.path.join(src, "net.txt"), os.path.join(src, "cuts.txt")
        L, ups = update_sets(net)
        base = pools.read_nodes(os.path.join(src, "nodes.txt"))[:80]
        probe = os.path.join(d, "probe_nodes.txt")
        pools.write_nodes(probe, base)
        tmp = os.path.join(d, "probe.txt")
        run([REF, "restricted", net, cuts, probe, DMIN.hex(), "128", tmp])
        res = parse(tmp)
        os.remove(tmp)
        os.remove(probe)
        deep = []
        for st, ex, lb, path in res[:30]:
            if len(path) != L:
                continue
            for gl in range(L - 1, max(0, L - 6), -1):
                if gl in ups:
                    deep.append(pools.NodeRecord(gl, DMIN, DMAX, list(ups[gl]), list(path[:gl])))
        nodes = base + deep
        pools.write_nodes(os.path.join(d, "nodes.txt"), nodes)
        runs, k = [], 0
        for w in widths:
            incs = [DMIN]
            tmp = os.path.join(d, f"restricted_{k}.txt")
            run([REF, "restricted", net, cuts, os.path.join(d, "nodes.txt"), DMIN.hex(), str(w), tmp])
            lbs = sorted(lb for st, ex, lb, p in parse(tmp) if st == 0 and lb > DMIN)
            with open(tmp, "rb") as fi, gzip.open(tmp + ".gz", "wb", compresslevel=9) as fo:
                shutil.copyfileobj(fi, fo)
            os.remove(tmp)
            runs.append({"width": w, "incumbent": DMIN.hex(), "file": f"restricted_{k}.txt.gz"})
            k += 1
            if lbs:
                inc = lbs[len(lbs) // 2]
                tmp = os.path.join(d, f"restricted_{k}.txt")
                run([REF, "restricted", net, cuts, os.path.join(d, "nodes.txt"), inc.hex(), str(w), tmp])
                with open(tmp, "rb") as fi, gzip.open(tmp + ".gz", "wb", compresslevel=9) as fo:
                    shutil.copyfileobj(fi, fo)
                os.remove(tmp)
                runs.append({"width": w, "incumbent": inc.hex(), "file": f"restricted_{k}.txt.gz"})
                k += 1
        manifest.append({"name": name, "source": name, "nodes": len(nodes), "deep": len(deep), "runs": runs})
    with open(os.path.join(HERE, "restricted_manifest.json"), "w") as fh:
        json.dump(manifest, fh, indent=1)


if __name__ == "__main__":
    main()
