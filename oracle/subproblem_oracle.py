"""CPU oracle for the scenario subproblem (TEST INFRASTRUCTURE ONLY).

Restates the reference's per-scenario dual LP of ``GuroSolver`` -- variables
(grb.cpp:8-40), constraints 7b-7i (grb.cpp:42-136), objective for a path y-bar
(grb.cpp:166-227) -- and solves it with scipy's HiGHS instead of Gurobi 11.0.3
(absent here).  Also solves the primal it is the dual of, so that
the two objectives can be compared, and evaluates Q_s(y) for arbitrary matchings
(validity checks of generated cuts).

Parity at the Gurobi boundary is UNPINNED: the reference has no fixture for it, and
optimal duals / unbounded rays are not unique, so tests compare objective values
(1e-9 relative, integral data), infeasibility status, and tightness/validity of the
cuts the HIP kernel builds -- never the coefficients themselves.

Only ``tests/`` may import this module.
"""
from __future__ import annotations

import dataclasses
from typing import Dict, List, Sequence, Tuple

import numpy as np
from scipy.optimize import linprog
from scipy.sparse import coo_matrix


@dataclasses.dataclass
class SubNet:
    n: int
    tails: np.ndarray          # [m]
    heads: np.ndarray          # [m]
    lb: np.ndarray             # [m, S] int
    ub: np.ndarray             # [m, S] int
    reward: np.ndarray         # [m, S] int
    vbar: Sequence[int]
    layer_arcs: Sequence[int]  # processingOrder[l].second

    @property
    def m(self) -> int:
        return int(self.tails.shape[0])

    @property
    def S(self) -> int:
        return int(self.lb.shape[1])

    def out_arcs(self, v: int) -> List[int]:
        return [a for a in range(self.m) if int(self.tails[a]) == v]

    def in_arcs(self, v: int) -> List[int]:
        return [a for a in range(self.m) if int(self.heads[a]) == v]


def from_instance(inst, layer_arcs) -> SubNet:
    return SubNet(inst.n, np.asarray(inst.tails), np.asarray(inst.heads), np.asarray(inst.lb),
                  np.asarray(inst.ub), np.asarray(inst.reward), list(inst.vbar), list(layer_arcs))


def ybar_of_path(net: SubNet, path: Sequence[int]) -> Dict[Tuple[int, int, int], int]:
    """y-bar of GuroSolver::solveSubProblem(path) (grb.cpp:139-150)."""
    y = {}
    for a, d in enumerate(path):
        if d == -1:
            continue
        arc = net.layer_arcs[a]
        q, i = int(net.heads[arc]), int(net.tails[arc])
        j = int(net.heads[d])
        y[(i, q, j)] = 1
    return y


class _Index:
    def __init__(self):
        self.n = 0
        self.names = []

    def add(self, name):
        self.names.append(name)
        self.n += 1
        return self.n - 1


def dual_lp(net: SubNet, y: Dict[Tuple[int, int, int], int], s: int):
    """min-form dual of grb.cpp for scenario s.  Returns (status, objective, solution dict).

    status: 'optimal' | 'infeasible' (dual unbounded = primal infeasible) | 'other'."""
    n, m = net.n, net.m
    T, H = net.tails, net.heads
    vb = set(int(v) for v in net.vbar)
    ins = [[] for _ in range(n)]
    outs = [[] for _ in range(n)]
    for a in range(m):
        outs[int(T[a])].append(a)
        ins[int(H[a])].append(a)
    idx = _Index()
    alpha = {v: idx.add(("alpha", v)) for v in range(n)}
    beta = {a: idx.add(("beta", a)) for a in range(m)}
    gamma = {a: idx.add(("gamma", a)) for a in range(m)}
    lam, mu, sig, phi = {}, {}, {}, {}
    for q in net.vbar:
        q = int(q)
        for ai in ins[q]:
            i = int(T[ai])
            sig[(i, q)] = idx.add(("sigma", i, q))
            for bo in outs[q]:
                j = int(H[bo])
                lam[(i, q, j)] = idx.add(("lambda", i, q, j))
                mu[(i, q, j)] = idx.add(("mu", i, q, j))
        for bo in outs[q]:
            phi[(q, int(H[bo]))] = idx.add(("phi", q, int(H[bo])))
    nv = idx.n
    rows, cols, vals, rhs = [], [], [], []

    def con(terms, r):                      # sum(terms) >= r  ->  -sum <= -r
        k = len(rhs)
        for c, v in terms:
            rows.append(k)
            cols.append(c)
            vals.append(-v)
        rhs.append(-r)

    for a in range(m):
        i, j = int(T[a]), int(H[a])
        r = float(net.reward[a, 0])        # scenario-0 rewards (grb.cpp:53,71,89)
        src = len(ins[i]) == 0
        snk = len(outs[j]) == 0
        if src and snk:
            continue                          # A4 is emptied (Network.cpp:80)
        terms = [(beta[a], -1.0), (gamma[a], 1.0)]
        if src:                               # A1: alpha[q] ...
            terms.append((alpha[j], 1.0))
            if j in vb:
                for bo in outs[j]:
                    k = int(H[bo])
                    terms += [(lam[(i, j, k)], 1.0), (mu[(i, j, k)], -1.0)]
                terms.append((sig[(i, j)], 1.0))
        elif snk:                             # A2: -alpha[q] ...
            terms.append((alpha[i], -1.0))
            if i in vb:
                for ai in ins[i]:
                    k = int(T[ai])
                    terms += [(lam[(k, i, j)], -1.0), (mu[(k, i, j)], 1.0)]
                terms.append((phi[(i, j)], 1.0))
        else:                                 # A3
            terms += [(alpha[i], -1.0), (alpha[j], 1.0)]
            if i in vb:
                for ai in ins[i]:
                    k = int(T[ai])
                    terms += [(mu[(k, i, j)], 1.0), (lam[(k, i, j)], -1.0)]
                terms.append((phi[(i, j)], 1.0))
            if j in vb:
                for bo in outs[j]:
                    k = int(H[bo])
                    terms += [(lam[(i, j, k)], 1.0), (mu[(i, j, k)], -1.0)]
                terms.append((sig[(i, j)], 1.0))
        con(terms, r)
    c = np.zeros(nv)
    for a in range(m):
        c[gamma[a]] += float(net.ub[a, s])
        c[beta[a]] -= float(net.lb[a, s])
    for (i, q, j), k in lam.items():
        yv = y.get((i, q, j), 0)
        ai = next(x for x in ins[q] if int(T[x]) == i)
        bo = next(x for x in outs[q] if int(H[x]) == j)
        c[k] += float(net.ub[ai, s]) * (1 - yv)
        c[mu[(i, q, j)]] += float(net.ub[bo, s]) * (1 - yv)
    for (i, q), k in sig.items():
        ai = next(x for x in ins[q] if int(T[x]) == i)
        c[k] += float(net.ub[ai, s]) * sum(y.get((i, q, int(H[bo])), 0) for bo in outs[q])
    for (q, j), k in phi.items():
        bo = next(x for x in outs[q] if int(H[x]) == j)
        c[k] += float(net.ub[bo, s]) * sum(y.get((int(T[ai]), q, j), 0) for ai in ins[q])
    bounds = [(None, None) if idx.names[k][0] == "alpha" else (0, None) for k in range(nv)]
    for v in (0, n - 1):                      # alpha[0] == alpha[n-1] == 0 (grb.cpp:131-132)
        bounds[alpha[v]] = (0, 0)
    A = coo_matrix((vals, (rows, cols)), shape=(len(rhs), nv)).tocsr()
    res = linprog(c, A_ub=A, b_ub=np.array(rhs), bounds=bounds, method="highs")
    if res.status == 0:
        return "optimal", float(res.fun), dict(zip(idx.names, res.x))
    if res.status in (2, 3):                  # dual unbounded (or infeasible) -> primal infeasible
        return "infeasible", None, None
    return "other", None, None


def primal_lp(net: SubNet, y: Dict[Tuple[int, int, int], int], s: int):
    """The primal the dual above belongs to: max sum r x, conservation at nodes with in- and
    out-arcs, l <= x <= u, and the V-bar coupling rows (lambda, mu, sigma, phi)."""
    n, m = net.n, net.m
    T, H = net.tails, net.heads
    vb = set(int(v) for v in net.vbar)
    ins = [[] for _ in range(n)]
    outs = [[] for _ in range(n)]
    for a in range(m):
        outs[int(T[a])].append(a)
        ins[int(H[a])].append(a)
    Aeq, beq = [], []
    for v in range(n):
        if ins[v] and outs[v]:
            row = np.zeros(m)
            row[ins[v]] = 1.0
            row[outs[v]] = -1.0
            Aeq.append(row)
            beq.append(0.0)
    Aub, bub = [], []
    for q in vb:
        for ai in ins[q]:
            i = int(T[ai])
            tot = 0
            for bo in outs[q]:
                j = int(H[bo])
                yv = y.get((i, q, j), 0)
                tot += yv
                r1 = np.zeros(m); r1[ai] = 1.0; r1[bo] = -1.0
                Aub.append(r1); bub.append(float(net.ub[ai, s]) * (1 - yv))
                r2 = np.zeros(m); r2[bo] = 1.0; r2[ai] = -1.0
                Aub.append(r2); bub.append(float(net.ub[bo, s]) * (1 - yv))
            r3 = np.zeros(m); r3[ai] = 1.0
            Aub.append(r3); bub.append(float(net.ub[ai, s]) * tot)
        for bo in outs[q]:
            j = int(H[bo])
            tot = sum(y.get((int(T[ai]), q, j), 0) for ai in ins[q])
            r4 = np.zeros(m); r4[bo] = 1.0
            Aub.append(r4); bub.append(float(net.ub[bo, s]) * tot)
    c = -np.array([float(net.reward[a, 0]) for a in range(m)])
    bounds = [(float(net.lb[a, s]), float(net.ub[a, s])) for a in range(m)]
    res = linprog(c, A_ub=np.array(Aub) if Aub else None, b_ub=np.array(bub) if bub else None,
                  A_eq=np.array(Aeq) if Aeq else None, b_eq=np.array(beq) if beq else None,
                  bounds=bounds, method="highs")
    if res.status == 0:
        return "optimal", float(-res.fun)
    if res.status == 2:
        return "infeasible", None
    return "other", None


def evaluate(net: SubNet, path: Sequence[int]):
    """Per-scenario (status, objective) of the reference subproblem for a path, via the dual."""
    y = ybar_of_path(net, path)
    return [dual_lp(net, y, s)[:2] for s in range(net.S)]


def random_matching(net: SubNet, rng) -> Dict[Tuple[int, int, int], int]:
    """A random y: at every V-bar node each in-arc picks a distinct out-arc or nothing."""
    T, H = net.tails, net.heads
    y = {}
    for q in net.vbar:
        q = int(q)
        ins = [a for a in range(net.m) if int(H[a]) == q]
        outs = [int(H[b]) for b in range(net.m) if int(T[b]) == q]
        free = list(outs)
        for ai in ins:
            if free and rng.random() < 0.7:
                j = free.pop(int(rng.integers(0, len(free))))
                y[(int(T[ai]), q, j)] = 1
    return y


def cut_value(rhs: float, coef: Dict[Tuple[int, int, int], float], y) -> float:
    """RHS + sum coef * y, accumulated in key order."""
    v = rhs
    for k in sorted(coef):
        if y.get(k, 0):
            v += coef[k]
    return v
