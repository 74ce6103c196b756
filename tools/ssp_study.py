"""Study tool (not product, not test): how many shortest-path phases the scenario
subproblem's max-reward flow needs under different augmentation rules, on the contracted
network of random full matchings of a generated instance.

    python tools/ssp_study.py C3 1 8

Counts per (matching, scenario): SSP augmentations (one path per shortest-path
computation), Dinic-style phases (blocking flow over the (cost, hops)-tight arcs) and
primal-dual phases (max flow over the cost-tight arcs).
"""
import sys
from collections import deque

import numpy as np

sys.path.insert(0, ".")
from sgufp_solver_amd import instance  # noqa: E402

INF = float("inf")


def contracted(inst, y_dec, s):
    """y_dec[a] = chosen out-arc at head(a) (V-bar heads), -1 none.  Returns arcs
    (t, h, L, U, R) of complete chains and the node count."""
    n, m = inst.n, len(inst.tails)
    vb = np.zeros(n, bool)
    vb[list(inst.vbar)] = True
    chosen = -np.ones(m, int)
    for a in range(m):
        d = y_dec[a]
        if d >= 0:
            chosen[d] = a
    arcs = []
    for a0 in range(m):
        if vb[inst.tails[a0]] and chosen[a0] >= 0:
            continue
        a = a0
        L, U, R = inst.lb[a, s], inst.ub[a, s], inst.reward[a, s]
        h = -1
        while True:
            q = inst.heads[a]
            if not vb[q]:
                h = q
                break
            d = y_dec[a]
            if d < 0:
                break
            a = d
            L, U, R = max(L, inst.lb[a, s]), min(U, inst.ub[a, s]), R + inst.reward[a, s]
        t = -1 if vb[inst.tails[a0]] else inst.tails[a0]
        if t >= 0 and h >= 0:
            arcs.append([int(t), int(h), int(L), int(U), int(R)])
    return arcs


def residual(arcs, x, n, src, snk):
    """(u, v, cost, cap, arc index, dir)"""
    out = []
    for k, (t, h, L, U, R) in enumerate(arcs):
        if x[k] < U:
            out.append((t, h, -R, U - x[k], k, 1))
        if x[k] > 0:
            out.append((h, t, R, x[k], k, -1))
    for v in src:
        out.append((n, v, 0, 10**9, -1, 0))
    for v in snk:
        out.append((v, n + 1, 0, 10**9, -1, 0))
    return out


def bf(res, nn, start):
    d = [INF] * nn
    hops = [INF] * nn
    d[start] = 0
    hops[start] = 0
    for _ in range(nn + 2):
        ch = False
        for u, v, c, cap, k, dr in res:
            if d[u] == INF:
                continue
            cand = (d[u] + c, hops[u] + 1)
            if cand < (d[v], hops[v]):
                d[v], hops[v] = cand
                ch = True
        if not ch:
            break
    return d, hops


def apply(path, x, delta):
    for (u, v, c, cap, k, dr) in path:
        if k >= 0:
            x[k] += dr * delta


def blocking(res, n, tight, x):
    """repeated DFS augmentations over tight residual arcs with dead-end removal; returns #paths"""
    nn = n + 2
    adj = [[] for _ in range(nn)]
    for e in res:
        if tight(e):
            adj[e[0]].append(list(e))
    ptr = [0] * nn
    paths = 0
    while True:
        stack, v = [], n
        seen = {n}
        while v != n + 1:
            moved = False
            while ptr[v] < len(adj[v]):
                e = adj[v][ptr[v]]
                if e[3] > 0 and e[1] not in seen:
                    stack.append(e)
                    seen.add(e[1])
                    v = e[1]
                    moved = True
                    break
                ptr[v] += 1
            if not moved:
                if not stack:
                    return paths
                e = stack.pop()
                seen.discard(v)
                v = e[0]
                ptr[v] += 1
        delta = min(e[3] for e in stack)
        for e in stack:
            e[3] -= delta
            if e[4] >= 0:
                x[e[4]] += e[5] * delta
        paths += 1


def run(arcs, n, src, snk, mode):
    x = [0] * len(arcs)
    phases = paths = 0
    while True:
        res = residual(arcs, x, n, src, snk)
        d, hp = bf(res, n + 2, n)
        if d[n + 1] == INF or d[n + 1] >= 0:
            break
        phases += 1
        if mode == "ssp":
            # one path: tight (cost, hops) predecessor walk
            pred = {}
            for e in res:
                u, v = e[0], e[1]
                if d[u] < INF and (d[u] + e[2], hp[u] + 1) == (d[v], hp[v]) and v not in pred:
                    pred[v] = e
            v, path = n + 1, []
            while v != n:
                e = pred[v]
                path.append(e)
                v = e[0]
            delta = min(e[3] for e in path)
            apply(path, x, delta)
            paths += 1
        elif mode == "dinic":
            paths += blocking(res, n, lambda e: d[e[0]] < INF and (d[e[0]] + e[2], hp[e[0]] + 1) == (d[e[1]], hp[e[1]]), x)
        else:
            paths += blocking(res, n, lambda e: d[e[0]] < INF and d[e[0]] + e[2] == d[e[1]], x)
            # max flow on the cost-tight graph: repeat until no tight path
            while True:
                res2 = residual(arcs, x, n, src, snk)
                p = blocking(res2, n, lambda e: d[e[0]] < INF and d[e[1]] < INF and d[e[0]] + e[2] == d[e[1]], x)
                if p == 0:
                    break
                paths += p
    obj = sum(a[4] * xi for a, xi in zip(arcs, x))
    return phases, paths, obj


def main():
    cfg, seed, trials = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    inst = instance.generate(instance.CONFIGS[cfg], seed, scenarios=4)
    inst.lb[:] = 0
    n, m = inst.n, len(inst.tails)
    rng = np.random.default_rng(seed)
    vb = set(int(v) for v in inst.vbar)
    indeg = np.bincount(inst.heads, minlength=n)
    outdeg = np.bincount(inst.tails, minlength=n)
    for t in range(trials):
        y = -np.ones(m, int)
        for q in vb:
            ins = [a for a in range(m) if inst.heads[a] == q]
            outs = [b for b in range(m) if inst.tails[b] == q]
            rng.shuffle(ins)
            rng.shuffle(outs)
            for a, b in zip(ins, outs):
                y[a] = b
        arcs = contracted(inst, y, 0)
        src = [v for v in range(n) if indeg[v] == 0 and outdeg[v] > 0]
        snk = [v for v in range(n) if outdeg[v] == 0 and indeg[v] > 0]
        r = {md: run(arcs, n, src, snk, md) for md in ("ssp", "dinic", "pd")}
        print(t, len(arcs), {k: v[:2] for k, v in r.items()}, [v[2] for v in r.values()])


if __name__ == "__main__":
    main()
