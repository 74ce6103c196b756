"""Fixture access and bit-exact comparison helpers for the parity tests."""
from __future__ import annotations

import gzip
import json
import os
import struct
from typing import List

from sgufp_solver_amd import pools

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden")


def manifest():
    with open(os.path.join(GOLDEN, "manifest.json")) as fh:
        return json.load(fh)


def case_dir(name: str) -> str:
    return os.path.join(GOLDEN, name)


_PLAIN = {}


def golden_file(d: str, fname: str) -> str:
    """Path of a plain-text fixture file of case directory d: the file itself, or -- for the
    large pools of the device-B&B cases, stored as <fname>.gz -- a decompressed copy."""
    path = os.path.join(d, fname)
    if os.path.exists(path):
        return path
    if path not in _PLAIN:
        import tempfile
        out = os.path.join(tempfile.mkdtemp(prefix="sgufp_golden_"), fname)
        with gzip.open(path + ".gz", "rb") as fi, open(out, "wb") as fo:
            fo.write(fi.read())
        _PLAIN[path] = out
    return _PLAIN[path]


def read_golden(name: str, fname: str) -> str:
    with gzip.open(os.path.join(case_dir(name), fname), "rb") as fh:
        return fh.read().decode()


def parse_results_text(text: str) -> List[pools.RelaxResult]:
    import tempfile
    with tempfile.NamedTemporaryFile("w", suffix=".txt", delete=False) as fh:
        fh.write(text)
        p = fh.name
    try:
        return pools.read_results(p)
    finally:
        os.remove(p)


def bits(x: float) -> int:
    return struct.unpack("<q", struct.pack("<d", x))[0]


def node_key(nd: pools.NodeRecord):
    return (nd.gl, bits(nd.lb), bits(nd.ub), tuple(nd.states), tuple(nd.sol))


def compare_results(got: List[pools.RelaxResult], want: List[pools.RelaxResult], check_stats: bool = True):
    """Bit-exact comparison; returns a list of human-readable mismatches (empty = parity)."""
    bad = []
    if len(got) != len(want):
        return [f"result count {len(got)} != {len(want)}"]
    for k, (g, w) in enumerate(zip(got, want)):
        if g.status != w.status:
            bad.append(f"node {k}: status {g.status} != {w.status}")
            continue
        if g.exact != w.exact:
            bad.append(f"node {k}: exact {g.exact} != {w.exact}")
        if bits(g.lb) != bits(w.lb) or bits(g.ub) != bits(w.ub):
            bad.append(f"node {k}: bounds ({g.lb!r},{g.ub!r}) != ({w.lb!r},{w.ub!r})")
        if g.path != w.path:
            bad.append(f"node {k}: path differs (len {len(g.path)} vs {len(w.path)})")
        if len(g.children) != len(w.children):
            bad.append(f"node {k}: {len(g.children)} children != {len(w.children)}")
        else:
            for c, (a, b) in enumerate(zip(g.children, w.children)):
                if node_key(a) != node_key(b):
                    bad.append(f"node {k} child {c}: {node_key(a)[:4]} != {node_key(b)[:4]}")
                    break
        if check_stats and (g.dd_nodes, g.dd_arcs, g.dd_layers) != (w.dd_nodes, w.dd_arcs, w.dd_layers):
            bad.append(f"node {k}: DD size {(g.dd_nodes, g.dd_arcs, g.dd_layers)} != {(w.dd_nodes, w.dd_arcs, w.dd_layers)}")
        if len(bad) > 20:
            break
    return bad


def refine_manifest():
    p = os.path.join(GOLDEN, "refine_manifest.json")
    if not os.path.exists(p):
        return {}
    with open(p) as fh:
        return json.load(fh)


# ---------------------------------------------------------------- restricted DD fixtures
RESTRICTED = os.path.join(GOLDEN, "restricted")


def restricted_manifest():
    with open(os.path.join(GOLDEN, "restricted_manifest.json")) as fh:
        return json.load(fh)


def restricted_dir(name: str) -> str:
    return os.path.join(RESTRICTED, name)


def read_restricted(name: str, fname: str) -> str:
    with gzip.open(os.path.join(restricted_dir(name), fname), "rb") as fh:
        return fh.read().decode()


def parse_restricted_text(text: str):
    """Per node: (status, exact, lb, path, children) from "Q status exact lb nchildren npath"
    blocks (oracle/ref_driver.cpp "restricted")."""
    lines = text.splitlines()
    out, k = [], 1
    while k < len(lines):
        q = lines[k].split()
        k += 1
        st, ex, lb, nc, np_ = int(q[1]), int(q[2]), float.fromhex(q[3]), int(q[4]), int(q[5])
        path = [int(x) for x in lines[k].split()] if np_ else []
        k += 1 if np_ else 0
        kids = []
        for _ in range(nc):
            t = lines[k].split()
            k += 1
            gl, ns = int(t[0]), int(t[3])
            states = [int(x) for x in t[4:4 + ns]]
            nsol = int(t[4 + ns])
            sol = [int(x) for x in t[5 + ns:5 + ns + nsol]]
            kids.append(pools.NodeRecord(gl, float.fromhex(t[1]), float.fromhex(t[2]), states, sol))
        out.append((st, ex, lb, path, kids))
    return out
