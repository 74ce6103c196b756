"""Open-node frontiers for benches and the batched solver driver.

bfs_frontier follows the survey probe: start from the root record
(DDSolver::startSolver builds the root with Node{}, DDSolver.cpp:788-791) and expand
cutset children breadth-first on the device until ``n`` records exist.
"""
from __future__ import annotations

import numpy as np

from . import engine as E
from .pools import DOUBLE_MAX, DOUBLE_MIN, NodeRecord


def root_batch() -> E.BatchArrays:
    return E.BatchArrays([NodeRecord(0, DOUBLE_MIN, DOUBLE_MAX, [], [])])


def bfs_frontier(eng: E.Engine, n: int, incumbent: float = DOUBLE_MIN) -> E.BatchArrays:
    """First ``n`` records of a BFS over cutset children (relaxed with the engine's pool)."""
    level = root_batch()
    done = []
    count = 0
    queue = [level]
    while queue and count < n:
        cur = queue.pop(0)
        if cur.n == 0:
            continue
        nxt_parts = []
        got = 0
        for s in range(0, cur.n, eng.info.max_batch):
            part = E.batch_slice(cur, np.arange(s, min(cur.n, s + eng.info.max_batch)))
            eng.upload(part)
            eng.relax_async(incumbent)
            eng.sync()
            nxt_parts.append(eng.children_batch())
            got += nxt_parts[-1].n
            if count + got >= n:
                break   # the first n records of BFS order are complete: stop relaxing this level
        nxt = E.batch_concat(nxt_parts)
        take = min(n - count, nxt.n)
        done.append(E.batch_slice(nxt, np.arange(take)))
        count += take
        queue.append(nxt)
    return E.batch_concat(done) if done else root_batch()
