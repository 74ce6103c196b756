"""Seeded synthetic cut pools and the text exchange formats.

Cut recipe: the reference's own random-cut generator ``getActualCut``
(/root/reference/tests/tests2.cpp:259-286): for every DD layer (i, q) and every
head j of q's out-arcs, with probability 6/11 a coefficient U(-100, 100), else
an explicit 0.0 (dropped later by ``cutToCut``, Cut.h:406-421); RHS U(-100,100),
x10 for optimality cuts, |.|x7 for feasibility cuts.  The reference draws from
``std::random_device``; here numpy PCG64 with a fixed seed makes pools
reproducible.  Coefficients are enumerated per (i, q, j) key -- the layer order
of the recipe only decides which draw lands on which key.

Formats (shared with oracle/ref_driver.cpp and oracle/dd_oracle.cpp; doubles are
C99 hex floats so every bit survives the round trip):
    cuts  : "<ncuts>" then per cut "<type> <rhs> <nnz>" + nnz lines "<i> <q> <j> <v>"
            type 0 = optimality, 1 = feasibility; listed in insertion order.
    nodes : "<n>" then per node "<gl> <lb> <ub> <ns> s.. <nsol> d.."
"""
from __future__ import annotations

import dataclasses
from typing import List, Sequence, Tuple

import numpy as np

from .instance import Instance

DOUBLE_MIN = float(np.finfo(np.float64).min)
DOUBLE_MAX = float(np.finfo(np.float64).max)


@dataclasses.dataclass
class PoolCut:
    type: int                                   # 0 optimality, 1 feasibility
    rhs: float
    coeff: List[Tuple[int, int, int, float]]    # (i, q, j, value)


@dataclasses.dataclass
class NodeRecord:
    gl: int
    lb: float
    ub: float
    states: List[int]
    sol: List[int]


def vbar_keys(inst: Instance) -> List[Tuple[int, int, int]]:
    """All (i, q, j) triples a cut can carry: arc i->q into a V-bar node q, arc q->j out of it."""
    vb = set(inst.vbar)
    keys = []
    seen = set()
    for a in range(inst.m):
        q = int(inst.heads[a])
        if q not in vb:
            continue
        i = int(inst.tails[a])
        for b in range(inst.m):
            if int(inst.tails[b]) == q:
                k = (i, q, int(inst.heads[b]))
                if k not in seen:
                    seen.add(k)
                    keys.append(k)
    return keys


def synthetic_pool(inst: Instance, n_feas: int, n_opt: int, seed: int,
                   interleave: bool = True) -> List[PoolCut]:
    rng = np.random.Generator(np.random.PCG64(seed))
    keys = vbar_keys(inst)
    types = [1] * n_feas + [0] * n_opt
    if interleave:
        rng.shuffle(types)
    pool = []
    for t in types:
        keep = rng.integers(0, 11, size=len(keys)) % 2 == 0
        vals = rng.uniform(-100.0, 100.0, size=len(keys))
        coeff = [(i, q, j, float(v) if k else 0.0) for (i, q, j), v, k in zip(keys, vals, keep)]
        rhs = float(rng.uniform(-100.0, 100.0))
        rhs = rhs * 10.0 if t == 0 else abs(rhs) * 7.0
        pool.append(PoolCut(t, rhs, coeff))
    return pool


def write_pool(path: str, pool: Sequence[PoolCut]) -> None:
    lines = [str(len(pool))]
    for c in pool:
        lines.append(f"{c.type} {float(c.rhs).hex()} {len(c.coeff)}")
        for (i, q, j, v) in c.coeff:
            lines.append(f"{i} {q} {j} {float(v).hex()}")
    with open(path, "w") as fh:
        fh.write("\n".join(lines) + "\n")


def read_pool(path: str) -> List[PoolCut]:
    with open(path) as fh:
        tok = fh.read().split()
    pos = 0
    n = int(tok[pos]); pos += 1
    pool = []
    for _ in range(n):
        t = int(tok[pos]); rhs = float.fromhex(tok[pos + 1]); nnz = int(tok[pos + 2]); pos += 3
        coeff = []
        for _ in range(nnz):
            coeff.append((int(tok[pos]), int(tok[pos + 1]), int(tok[pos + 2]), float.fromhex(tok[pos + 3])))
            pos += 4
        pool.append(PoolCut(t, rhs, coeff))
    return pool


def _fmt(x: float) -> str:
    return float(x).hex()


def write_nodes(path: str, nodes: Sequence[NodeRecord]) -> None:
    lines = [str(len(nodes))]
    for nd in nodes:
        parts = [str(nd.gl), _fmt(nd.lb), _fmt(nd.ub), str(len(nd.states))]
        parts += [str(s) for s in nd.states]
        parts.append(str(len(nd.sol)))
        parts += [str(s) for s in nd.sol]
        lines.append(" ".join(parts))
    with open(path, "w") as fh:
        fh.write("\n".join(lines) + "\n")


def _parse_node(tok: List[str], pos: int) -> Tuple[NodeRecord, int]:
    gl = int(tok[pos]); lb = float.fromhex(tok[pos + 1]); ub = float.fromhex(tok[pos + 2])
    ns = int(tok[pos + 3]); pos += 4
    states = [int(x) for x in tok[pos:pos + ns]]; pos += ns
    nsol = int(tok[pos]); pos += 1
    sol = [int(x) for x in tok[pos:pos + nsol]]; pos += nsol
    return NodeRecord(gl, lb, ub, states, sol), pos


def read_nodes(path: str) -> List[NodeRecord]:
    with open(path) as fh:
        tok = fh.read().split()
    n = int(tok[0]); pos = 1
    out = []
    for _ in range(n):
        nd, pos = _parse_node(tok, pos)
        out.append(nd)
    return out


@dataclasses.dataclass
class RelaxResult:
    status: int      # 0 SUCCESS, 1 PRUNED_F, 2 PRUNED_O, 3 NEEDS_LP (exact tree)
    exact: int
    lb: float
    ub: float
    children: List[NodeRecord]
    path: List[int]
    dd_nodes: int
    dd_arcs: int
    dd_layers: int


def read_results(path: str) -> List[RelaxResult]:
    with open(path) as fh:
        tok = fh.read().split()
    n = int(tok[0]); pos = 1
    out = []
    for _ in range(n):
        assert tok[pos] == "R"
        status, exact = int(tok[pos + 1]), int(tok[pos + 2])
        lb, ub = float.fromhex(tok[pos + 3]), float.fromhex(tok[pos + 4])
        nch, npath = int(tok[pos + 5]), int(tok[pos + 6])
        ddn, dda, ddl = int(tok[pos + 7]), int(tok[pos + 8]), int(tok[pos + 9])
        pos += 10
        path = [int(x) for x in tok[pos:pos + npath]]; pos += npath
        ch = []
        for _ in range(nch):
            nd, pos = _parse_node(tok, pos)
            ch.append(nd)
        out.append(RelaxResult(status, exact, lb, ub, ch, path, ddn, dda, ddl))
    return out
