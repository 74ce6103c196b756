"""Seeded synthetic SGUFP instances in the reference's text format.

The reference reads instances with ``Network::Network(const std::string&)``
(/root/reference/Network.cpp:10-129):

    n m S
    tail head  lb_0 ub_0 r_0  lb_1 ub_1 r_1 ...      (m lines, S triples each)
    Vbar
    id id id ...

The generator follows SURVEY.md §8(d): a layered DAG with source 0, sink n-1
and K middle layers of width W.  Every middle node gets ``d`` distinct random
out-arcs into the next layer, uncovered next-layer nodes get one in-arc, layer 0
is fed from the source and the last layer drains into the sink.  Random extra
inter-layer arcs are added (or removable ones trimmed) until |E| matches.
Each middle node is in V-bar with probability ``f``.  Per scenario
ub ~ U{5..50}, lb = 0 except sink arcs (lb ~ U{1..3} w.p. 0.3); the reward
r ~ U{-5..30} is the same for every scenario (the reference subproblem uses
scenario-0 rewards, grb.cpp:53,71,89, while the extensive form uses per-scenario
rewards, StochasticModel.h:57-58 -- scenario-invariant rewards make both agree).

Parallel arcs are never generated: the dual LP indexes beta/gamma by node pair
(grb.cpp:8-39), so parallel arcs would alias there.
"""
from __future__ import annotations

import dataclasses
from typing import List, Tuple

import numpy as np


@dataclasses.dataclass(frozen=True)
class InstanceConfig:
    name: str
    n_arcs: int
    layers: int        # K middle layers
    width: int         # W nodes per middle layer
    out_degree: int    # d distinct out-arcs per middle node
    vbar_prob: float   # f
    scenarios: int     # S


# SURVEY.md §8(d) configurations, plus T1/T2: tiny networks whose whole B&B tree is
# small enough for the end-to-end optimum check against the extensive form (main.cpp:66-76).
CONFIGS = {
    "T0": InstanceConfig("T0", 8, 2, 2, 2, 1.0, 1),
    "T1": InstanceConfig("T1", 12, 2, 3, 2, 1.0, 1),
    "T2": InstanceConfig("T2", 24, 3, 4, 2, 0.6, 1),
    "T3": InstanceConfig("T3", 30, 3, 5, 2, 0.6, 1),
    "T4": InstanceConfig("T4", 40, 4, 5, 2, 0.4, 1),
    # M1 / M2: the largest networks whose whole B&B tree and whose 64-scenario extensive form
    # (HiGHS) both close in minutes -- the end-to-end optimum check of BASELINE configs[2]
    # (64 scenarios) at a size that finishes; C3 itself closes neither
    "M1": InstanceConfig("M1", 60, 4, 6, 2, 0.5, 64),
    "M2": InstanceConfig("M2", 100, 5, 8, 2, 0.4, 64),
    # P1 / P3: between T4 and M1, generated lower bounds kept -- 64-scenario instances whose
    # extensive form (HiGHS) and device B&B both close (tools/closure_study.py)
    "P1": InstanceConfig("P1", 48, 4, 6, 2, 0.45, 64),
    "P3": InstanceConfig("P3", 52, 4, 6, 2, 0.5, 64),
    "C1": InstanceConfig("C1", 40, 3, 6, 2, 1.0, 1),
    "C2": InstanceConfig("C2", 200, 6, 12, 3, 0.5, 1),
    "C3": InstanceConfig("C3", 1000, 12, 30, 3, 0.3, 64),
    "C4": InstanceConfig("C4", 1000, 12, 30, 3, 0.3, 256),
    "C5": InstanceConfig("C5", 5000, 10, 165, 3, 0.08, 512),
}


@dataclasses.dataclass
class Instance:
    n: int
    tails: np.ndarray      # int32 [m]
    heads: np.ndarray      # int32 [m]
    lb: np.ndarray         # int32 [m, S]
    ub: np.ndarray         # int32 [m, S]
    reward: np.ndarray     # int32 [m, S]
    vbar: List[int]

    @property
    def m(self) -> int:
        return int(self.tails.shape[0])

    @property
    def scenarios(self) -> int:
        return int(self.lb.shape[1])

    def to_text(self) -> str:
        out = [f"{self.n} {self.m} {self.scenarios}"]
        for a in range(self.m):
            parts = [str(int(self.tails[a])), str(int(self.heads[a]))]
            for s in range(self.scenarios):
                parts += [str(int(self.lb[a, s])), str(int(self.ub[a, s])),
                          str(int(self.reward[a, s]))]
            out.append(" ".join(parts))
        out.append("Vbar")
        out.append(" ".join(str(v) for v in self.vbar))
        return "\n".join(out) + "\n"

    def write(self, path: str) -> None:
        with open(path, "w") as fh:
            fh.write(self.to_text())


def generate(cfg: InstanceConfig, seed: int, scenarios: int | None = None) -> Instance:
    """Deterministic (numpy PCG64) instance for ``cfg`` and ``seed``."""
    rng = np.random.Generator(np.random.PCG64(seed))
    S = cfg.scenarios if scenarios is None else scenarios
    K, W, d = cfg.layers, cfg.width, cfg.out_degree
    n = 2 + K * W
    sink = n - 1

    def node(layer: int, k: int) -> int:
        return 1 + layer * W + k

    arcs: List[Tuple[int, int]] = []
    arcset = set()

    def add(t: int, h: int) -> bool:
        if (t, h) in arcset:
            return False
        arcset.add((t, h))
        arcs.append((t, h))
        return True

    for k in range(W):
        add(0, node(0, k))
    for layer in range(K - 1):
        covered = np.zeros(W, dtype=bool)
        for k in range(W):
            heads = rng.choice(W, size=min(d, W), replace=False)
            for h in sorted(int(x) for x in heads):
                add(node(layer, k), node(layer + 1, h))
                covered[h] = True
        for h in range(W):
            if not covered[h]:
                add(node(layer, int(rng.integers(0, W))), node(layer + 1, h))
    for k in range(W):
        add(node(K - 1, k), sink)

    # top up / trim inter-layer arcs to hit |E| exactly
    target = cfg.n_arcs
    guard = 0
    while len(arcs) < target and guard < 100000:
        guard += 1
        layer = int(rng.integers(0, K - 1))
        add(node(layer, int(rng.integers(0, W))), node(layer + 1, int(rng.integers(0, W))))
    guard = 0
    while len(arcs) > target and guard < 100000:
        guard += 1
        idx = int(rng.integers(0, len(arcs)))
        t, h = arcs[idx]
        if t == 0 or h == sink:
            continue
        outdeg = sum(1 for (a, _) in arcs if a == t)
        indeg = sum(1 for (_, b) in arcs if b == h)
        if outdeg > 1 and indeg > 1:
            arcs.pop(idx)
            arcset.discard((t, h))
    if len(arcs) != target:
        raise ValueError(f"could not reach {target} arcs (got {len(arcs)})")

    # file order: shuffle so that incoming-arc lists are not trivially sorted
    order = rng.permutation(len(arcs))
    arcs = [arcs[i] for i in order]
    m = len(arcs)
    tails = np.array([a[0] for a in arcs], dtype=np.int32)
    heads = np.array([a[1] for a in arcs], dtype=np.int32)

    # V-bar is drawn before any scenario data so that the network structure (and the DD
    # built on it) is the same for every scenario count: C3 and C4 differ only in S.
    vbar = [v for v in range(1, n - 1) if rng.random() < cfg.vbar_prob]
    if not vbar:
        vbar = [node(K - 1, 0)]

    ub = rng.integers(5, 51, size=(m, S)).astype(np.int32)
    lb = np.zeros((m, S), dtype=np.int32)
    sink_arcs = heads == sink
    lbv = rng.integers(1, 4, size=(m, S)).astype(np.int32)
    lbmask = rng.random(size=(m, S)) < 0.3
    lb[sink_arcs] = np.where(lbmask[sink_arcs], lbv[sink_arcs], 0)
    r = rng.integers(-5, 31, size=m).astype(np.int32)
    reward = np.repeat(r[:, None], S, axis=1)

    return Instance(n=n, tails=tails, heads=heads, lb=lb, ub=ub, reward=reward, vbar=vbar)


def generate_text(name: str, seed: int, scenarios: int | None = None) -> str:
    return generate(CONFIGS[name], seed, scenarios).to_text()


def random_matching_path(inst: Instance, layer_arcs, rng) -> list:
    """DD decision vector (one entry per layer, GuroSolver::solveSubProblem's input,
    grb.cpp:139-150) of a random full matching at every V-bar node: each incoming arc
    of q is matched to a distinct out-arc of q while both last.  Layer l decides the
    in-arc processingOrder[l] (layer_arcs[l]); the decision is the chosen out-arc's id
    or -1.  Synthetic exact-leaf paths for subproblem throughput runs."""
    m = len(inst.tails)
    outs = {}
    for b in range(m):
        outs.setdefault(int(inst.tails[b]), []).append(b)
    vb = set(int(v) for v in inst.vbar)
    choice = {}
    for q in sorted(vb):
        ins = [a for a in range(m) if int(inst.heads[a]) == q]
        free = list(outs.get(q, []))
        rng.shuffle(ins)
        rng.shuffle(free)
        for a in ins:
            if free:
                choice[a] = free.pop()
    return [int(choice.get(int(a), -1)) for a in layer_arcs]

