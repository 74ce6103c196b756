"""Restricted-DD primal heuristic: the restricted half of Inavap::NodeExplorer::processX3
(/root/reference/NodeExplorer.cpp:605-796) on the device.

For each record a restricted DD of at most ``width`` nodes per layer
(Inavap::RestrictedDDNew, DD.cpp:3090-3505; k_restrict) is swept with the pool, then the
refinement loop of processX3 runs: the max path (getSolution) goes to the scenario
subproblem (GuroSolver::solveSubProblem; k_sub_scenario), the new cut joins the pool
(Container::add) and is applied, until the path repeats with an unchanged bound
(NodeExplorer.cpp:650-664 / 736-748).  A record that converges returns
{lowerBound, ...}: the value of a feasible routing, which raises the incumbent
(DDSolver.cpp:723-731).  A false feasibility sweep or a bound <= optimalLB ends the record
(INVALID_OBJECT).  What is reproduced is the value of the exact-tree refinement only: in
processX3's non-exact branch (NodeExplorer.cpp:698-793) a restricted infeasibility or a
bound <= optimalLB still returns SUCCESS with the cutset and the relaxed DD decides the
pruning; the heuristic here drops such records instead (it only seeds the incumbent).
A record the device cannot represent (status 16) raises.  The restricted DD is re-swept from scratch with the grown pool each
iteration; the outcome equals applying only the new cut (removals are a union, terminal
weights a running minimum).
"""
from __future__ import annotations

from typing import List, Sequence

from .pools import DOUBLE_MIN, NodeRecord


class RestrictedResult:
    __slots__ = ("status", "lb", "path", "iterations", "converged")

    def __init__(self, status, lb, path, iterations, converged):
        self.status, self.lb, self.path, self.iterations, self.converged = status, lb, path, iterations, converged


class RestrictedExplorer:
    def __init__(self, engine, width: int = 128, max_iters: int = 500):
        self.eng = engine
        self.width = width
        self.max_iters = max_iters
        self.subproblems = 0

    def explore(self, records: Sequence[NodeRecord], optimal_lb: float) -> List[RestrictedResult]:
        eng = self.eng
        n = len(records)
        out: List[RestrictedResult] = [None] * n
        prev_path = [None] * n
        prev_lb = [None] * n
        active = list(range(n))
        it = 0
        while active:
            res = eng.restricted([records[k] for k in active], optimal_lb, self.width)
            nxt, paths = [], []
            for k, (st, ex, lb, path, kids) in zip(active, res):
                if st >= 16:
                    raise RuntimeError(f"restricted heuristic: record {k} failed on the device (status {st})")
                if st != 0:
                    out[k] = RestrictedResult(st, lb, path, it, False)       # INVALID_OBJECT
                    continue
                if prev_path[k] == path:
                    if prev_lb[k] == lb:
                        out[k] = RestrictedResult(0, lb, path, it, True)     # {lowerBound, ...}
                        continue
                    prev_lb[k] = lb
                else:
                    prev_path[k] = path
                    prev_lb[k] = lb
                nxt.append(k)
                paths.append(path)
            if not nxt:
                break
            if it >= self.max_iters:
                for k in nxt:
                    out[k] = RestrictedResult(0, prev_lb[k], prev_path[k], it, False)
                break
            typ, rhs, rows, _ = eng.subproblem(paths)
            self.subproblems += len(paths)
            keep = []
            for j, k in enumerate(nxt):
                if typ[j] < 0:
                    raise RuntimeError(f"restricted heuristic: subproblem failed for record {k}")
                eng.add_cut_rows(int(typ[j]), rhs[j:j + 1], rows[j:j + 1])
                keep.append(k)
            active = keep
            it += 1
        return out

    def incumbent(self, records: Sequence[NodeRecord], optimal_lb: float = DOUBLE_MIN) -> float:
        """The best converged bound of the records (optimal_lb when none converges)."""
        best = optimal_lb
        for r in self.explore(records, optimal_lb):
            if r.converged and r.lb > best:
                best = r.lb
        return best
