"""Restricted decision diagram (Inavap::RestrictedDDNew, /root/reference/DD.cpp:3090-3505) under
the restricted cut phases of NodeExplorer::processX3 (NodeExplorer.cpp:605-656): compile with a
width limit, feasibility cuts then optimality cuts of the pool (newest first), the max path.

CPU: the clean-room restatement (oracle/dd_oracle.cpp "restricted") reproduces the reference's
own output (tests/golden/restricted/, made by oracle/_ref/ref_dd, see make_restricted.py)
byte for byte.  GPU: k_restrict through the C ABI, bit-exact on status, exactness, the bound's
bit pattern, the max path and the exact cutset (states, solution vector, global layer)."""
import os
import struct
import subprocess

import pytest

from tests import golden_io

CASES = [(c["name"], r) for c in golden_io.restricted_manifest() for r in c["runs"]]
IDS = [f"{c}-w{r['width']}-{r['file']}" for c, r in CASES]


@pytest.mark.parametrize("name,run", CASES, ids=IDS)
def test_oracle_restricted_matches_reference(oracle_bin, tmp_path, name, run):
    d = golden_io.restricted_dir(name)
    src = golden_io.case_dir(name)
    out = tmp_path / "r.txt"
    subprocess.run([oracle_bin, "restricted", f"{src}/net.txt", f"{src}/cuts.txt", f"{d}/nodes.txt", run["incumbent"],
                    str(run["width"]), str(out)], check=True)
    assert out.read_text() == golden_io.read_restricted(name, run["file"])


def test_restricted_fixtures_cover_every_outcome():
    seen = set()
    for name, run in CASES:
        for st, ex, lb, path, kids in golden_io.parse_restricted_text(golden_io.read_restricted(name, run["file"])):
            seen.add((st, ex))
    assert {(0, 0), (0, 1), (1, 0), (2, 0), (2, 1)} <= seen


def _bits(x):
    return struct.unpack("<Q", struct.pack("<d", x))[0]


@pytest.mark.gpu
@pytest.mark.parametrize("name,run", CASES, ids=IDS)
def test_restricted_matches_reference(name, run):
    from sgufp_solver_amd import engine as E
    from sgufp_solver_amd import pools
    src = golden_io.case_dir(name)
    d = golden_io.restricted_dir(name)
    nodes = pools.read_nodes(os.path.join(d, "nodes.txt"))
    e = E.Engine(os.path.join(src, "net.txt"), 0, max(256, len(nodes)))
    e.add_cuts(pools.read_pool(os.path.join(src, "cuts.txt")))
    got = e.restricted(nodes, float.fromhex(run["incumbent"]), int(run["width"]))
    e.close()
    want = golden_io.parse_restricted_text(golden_io.read_restricted(name, run["file"]))
    assert len(got) == len(want)
    bad = []
    for k, (g, w) in enumerate(zip(got, want)):
        gs, gx, glb, gp, gk = g
        ws, wx, wlb, wp, wk = w
        if (gs, gx) != (ws, wx) or _bits(glb) != _bits(wlb) or gp != wp:
            bad.append(f"node {k}: got {(gs, gx, glb.hex(), len(gp))} want {(ws, wx, wlb.hex(), len(wp))}")
            continue
        if len(gk) != len(wk):
            bad.append(f"node {k}: {len(gk)} cutset nodes, want {len(wk)}")
            continue
        for a, b in zip(gk, wk):
            if (a.gl, a.states, a.sol) != (b.gl, b.states, b.sol) or _bits(a.lb) != _bits(b.lb) or _bits(a.ub) != _bits(b.ub):
                bad.append(f"node {k}: cutset record differs: {a} vs {b}")
                break
    assert not bad, "\n".join(bad[:10])
