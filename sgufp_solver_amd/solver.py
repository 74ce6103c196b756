"""Inavap::DDSolver on MI355X: batched B&B rounds over a device-resident frontier.

Mirrors the reference's solver surface (/root/reference/DDSolver.h:431-439):

    DDSolver(network, n_workers)           -> DDSolver(network_path, n_workers=..., ...)
    std::pair<double,double> start(double) -> start(known_opt) -> (solution, seconds)
    double startSolver(double)             -> start_solver(known_opt)

and its final report line (DDSolver.cpp:863-865).  The work of one round is native
(``sgufp_bnb_step``, sgufp_solver_amd/csrc/bnb.cpp): pop a batch from the frontier stack
in HBM, relax it, run the exact-leaf refinement loops with the device subproblem, raise
the incumbent, push the children.  This module only sequences rounds and, with more
than one rank (one process per GPU, ``torch.distributed``; the "nccl" backend is RCCL
over xGMI), does the exchanges the reference does through shared memory:

* incumbent: all-reduce(MAX) of one double per round -- the CAS-max on
  ``DDSolver::optimal`` (DDSolver.cpp:723-731);
* cut pool: the rows each rank appended in the round are all-gathered and appended on
  every other rank -- the global ``feasCutsGlobal`` / ``optCutsGlobal`` Containers
  (DDSolver.h:415-416) every worker reads;
* load balance: frontier sizes are all-gathered; when a rank runs dry the largest
  shard gives away a share of its oldest records (the bottom of its stack) -- the
  master's half-split and 40 % steal (DDSolver.cpp:603-621, 642-652);
* termination: every shard empty (DDSolver.cpp:630-640).

``engine`` may be any object with the Engine's frontier / bnb_step / cut-row methods;
the product path passes ``sgufp_solver_amd.engine.Engine`` (HIP), the CPU multi-process
tests pass a toy engine to exercise the protocol.
"""
from __future__ import annotations

import time
from typing import Optional

import numpy as np

from .pools import DOUBLE_MAX, DOUBLE_MIN, NodeRecord


class DDSolver:
    def __init__(self, network_path: Optional[str] = None, n_workers: int = 1, device: int = 0,
                 max_batch: int = 4096, batch_nodes: int = 0, engine=None, group=None, verbose: bool = True,
                 progress: float = 0.0, max_rounds: int = 0, dive_batch: int = 64, time_budget: float = 0.0,
                 restricted_width: int = 0, round_seconds: float = 0.0, round_iters: int = 0,
                 native_world: int = 0, comm=None, stop_rounds: int = 0):
        """n_workers is accepted for API compatibility with the reference (threads there);
        the parallelism here is the batch of ``batch_nodes`` (<= max_batch) records per
        round and one rank per GPU."""
        self.n_workers = n_workers
        if engine is None:
            from .engine import Engine
            engine = Engine(network_path, device, max_batch)
        self.eng = engine
        self.batch_nodes = batch_nodes
        self.group = group
        self.verbose = verbose
        self.progress = progress        # seconds between progress lines on stderr (0: none)
        self.max_rounds = max_rounds    # safety cap for tests (0: none); hitting it raises
        # stop after this many rounds (0: none) with complete = False, like the C++
        # Inavap::DDSolver::maxRounds (the same rounds for a deterministic comparison)
        self.stop_rounds = stop_rounds
        # Until the first exact leaf is reached there is no cut to prune with (and at most
        # the seeded incumbent):
        # rounds of dive_batch records from the top of the stack go depth-first to the
        # exact leaves (like the reference's LIFO workers) instead of relaxing wide layers
        # of siblings that nothing can prune yet.
        self.dive_batch = dive_batch
        # stop after this many seconds (0: none) with complete = False -- for throughput
        # measurements of searches that would run for hours
        self.time_budget = time_budget
        # primal heuristic (0: off): before the search, the restricted-DD half of
        # NodeExplorer::processX3 (NodeExplorer.cpp:605-796) on the root record seeds the
        # incumbent with the value of the routing its refinement loop converges to
        self.restricted_width = restricted_width
        # > 0: the engine's context is one shard of an RCCL communicator of that many ranks
        # (Engine.comm_init done by the caller) and the round's exchanges are the library's own
        # (sgufp_incumbent_allreduce / _cuts_exchange / _frontier_sizes / _frontier_balance,
        # shard.cpp: device buffers, no host staging); 0: torch.distributed (shards.py)
        self.native_world = native_world
        # an explicit exchange object (shards.LocalComm: several shards as threads of one
        # process, e.g. on one GPU); None: torch.distributed when initialised with > 1 rank
        self.comm = comm
        # bound of one round's exact-leaf refinement loops (0: none; see Engine.bnb_set_limits)
        self.round_seconds = round_seconds
        self.round_iters = round_iters
        self.heuristic_incumbent = None
        self.complete = False
        self.counters = {}
        self.rounds = 0
        self.seconds = 0.0
        self.shard_comm = None
        self.received = 0

    # -- collectives ---------------------------------------------------------------
    def _comm(self):
        """ShardComm over the group (None with one rank)."""
        import torch.distributed as dist
        if not dist.is_available() or not dist.is_initialized():
            return None
        if dist.get_world_size(self.group) == 1:
            return None
        from .shards import ShardComm
        return ShardComm(self.group)

    # -- the solver -------------------------------------------------------------------
    def start_solver(self, known_optimal: float) -> float:
        """DDSolver::startSolver (DDSolver.cpp:782-846): incumbent := known_optimal, the root
        record Node{} on the frontier (rank 0), rounds until every shard is empty."""
        comm = None if self.native_world else (self.comm if self.comm is not None else self._comm())
        self.shard_comm = comm
        rank = comm.rank if comm else 0
        eng = self.eng
        if self.native_world:
            import ctypes
            w, r = ctypes.c_int(0), ctypes.c_int(0)
            eng._check(eng.lib.sgufp_comm_info(eng.ctx, ctypes.byref(w), ctypes.byref(r)))
            rank = r.value
        eng.frontier_clear()
        if rank == 0:
            eng.frontier_push([NodeRecord(0, DOUBLE_MIN, DOUBLE_MAX, [], [])])
        z = float(known_optimal)
        # rows already shared: the heuristic's cuts below are new, so the first exchange
        # sends them to every shard (the global pool, DDSolver.h:415-416)
        marks = {1: eng.cuts_count(1), 0: eng.cuts_count(0)}
        if self.restricted_width > 0 and rank == 0:
            from .restricted import RestrictedExplorer
            h = RestrictedExplorer(eng, self.restricted_width).incumbent([NodeRecord(0, DOUBLE_MIN, DOUBLE_MAX, [], [])], z)
            self.heuristic_incumbent = h
            z = max(z, h)
        keys = ("popped", "relaxed", "pruned_bound", "pruned_feasibility", "pruned_optimality", "exact",
                "exact_closed", "subproblems", "new_feasibility_cuts", "new_optimality_cuts", "children", "pushed",
                "deferred", "resumed")
        self.counters = {k: 0 for k in keys}
        self.received = 0     # records received from other shards (work sharing)
        self.rounds = 0
        t_last = time.perf_counter()
        diving = self.dive_batch > 0
        self.complete = False
        t_start = time.perf_counter()
        limits = hasattr(eng, "bnb_set_limits")
        while True:
            batch = self.batch_nodes
            if diving:
                batch = self.dive_batch if not batch else min(batch, self.dive_batch)
            if limits:
                # a round's refinement loops stop at the budget (or round_seconds); the
                # unfinished exact records go back on top of the frontier
                left = self.time_budget - (time.perf_counter() - t_start) if self.time_budget > 0 else 0.0
                secs = self.round_seconds
                if self.time_budget > 0:
                    secs = max(1e-3, min(left, secs) if secs > 0 else left)
                eng.bnb_set_limits(self.round_iters, secs)
            z, st = eng.bnb_step(z, batch)
            if diving and int(getattr(st, "exact", 0) if not isinstance(st, dict) else st["exact"]) > 0:
                diving = False   # the dive reached exact leaves: cuts exist from here on
            self.rounds += 1
            if self.progress and time.perf_counter() - t_last > self.progress:
                t_last = time.perf_counter()
                import sys
                print(f"[DDSolver r{rank}] round {self.rounds} z={z!r} frontier={eng.frontier_size()} "
                      f"{self.counters}", file=sys.stderr, flush=True)
            if self.max_rounds and self.rounds >= self.max_rounds:
                raise RuntimeError(f"DDSolver: no termination within {self.max_rounds} rounds (z={z!r})")
            for k in keys:
                self.counters[k] += int(getattr(st, k, 0) if not isinstance(st, dict) else st.get(k, 0))
            over = (self.time_budget > 0 and time.perf_counter() - t_start > self.time_budget) or \
                (self.stop_rounds > 0 and self.rounds >= self.stop_rounds)
            if self.native_world:
                z = eng.incumbent_allreduce(z)
                eng.cuts_exchange()
                sizes = eng.frontier_sizes(self.native_world)
                if sum(sizes) == 0:
                    self.complete = True
                    break
                if eng.incumbent_allreduce(1.0 if over else 0.0) > 0.0:
                    break
                self.received += eng.frontier_balance()
                continue
            if comm is None:
                if eng.frontier_size() == 0:
                    self.complete = True
                    break
                if over:
                    break
                continue
            z = comm.allreduce_max(z)
            comm.exchange_cuts(eng, marks)
            g = comm.allgather_i64([eng.frontier_size(), 1 if over else 0])
            sizes = [int(x) for x in g[:, 0]]
            if sum(sizes) == 0:
                self.complete = True
                break
            if g[:, 1].any():
                break
            self.received += comm.rebalance(eng, sizes)
        return z

    def start(self, known_opt: float, solver_counters: bool = False):
        """DDSolver::start (DDSolver.cpp:848-867): solve, time, print the reference's line
        (and, with solver_counters -- the reference's SOLVER_COUNTERS build -- its
        printWorkerStats report first, one worker per rank)."""
        t0 = time.perf_counter()
        solution = self.start_solver(known_opt)
        self.seconds = time.perf_counter() - t0
        # "Explored N nodes" = sum of nQueue = children produced (DDSolver.cpp:742, 856-865)
        explored = self.counters.get("children", 0)
        comm = self.shard_comm
        per_rank = [dict(self.counters)]
        keys = sorted(self.counters)
        first = True
        if comm is not None:
            g = comm.allgather_i64([int(self.counters[k]) for k in keys])
            per_rank = [{k: int(v) for k, v in zip(keys, row)} for row in g]
            explored = sum(c.get("children", 0) for c in per_rank)
            first = comm.rank == 0
        elif self.native_world > 1:
            # the library's own communicator (shard.cpp): counters gathered four at a time
            import ctypes
            w, r = ctypes.c_int(0), ctypes.c_int(0)
            self.eng._check(self.eng.lib.sgufp_comm_info(self.eng.ctx, ctypes.byref(w), ctypes.byref(r)))
            cols = []
            for i in range(0, len(keys), 4):
                cols.append(self.eng.comm_allgather_i64([int(self.counters[k]) for k in keys[i:i + 4]], w.value))
            g = np.concatenate(cols, axis=1)
            per_rank = [{k: int(v) for k, v in zip(keys, row)} for row in g]
            explored = sum(c.get("children", 0) for c in per_rank)
            first = r.value == 0
        if self.verbose and solver_counters and first:
            print(worker_stats_text(per_rank, self.eng.cuts_count(1), self.eng.cuts_count(0)), end="")
        if self.verbose and first:
            print(f"Optimal solution: {solution}. Explored {explored} nodes (entire search space) in "
                  f"{self.seconds} seconds.")
        return solution, self.seconds


def worker_stats_text(per_worker, n_feas_cuts: int, n_opt_cuts: int) -> str:
    """DDSolver::printWorkerStats (DDSolver.h:441-501) for per-worker counter dicts (one per
    rank here): processed counts with total / mean / absolute deviation / min / max, the
    global cut counts, per-worker (feasibility, optimality, bound) prunes, waiting times
    (none: ranks do not sleep).  The dash line is 72 wide as in the reference (its length
    is computed before the list fills)."""
    dash = "-" * 72
    processed = [float(c.get("relaxed", 0)) for c in per_worker]
    mean = sum(processed) / len(processed) if processed else 0.0
    absdev = 0.0      # the reference's stats_absdev is a stub returning 0 (statistics.h:31-33)
    lines = [dash, "Processed: " + "".join(f"{int(p)}  " for p in processed),
             f"Total: {_g(sum(processed))}\t Mean: {_g(mean)}\t Deviation: {_g(absdev)}\t "
             f"Min: {_g(min(processed) if processed else 0.0)}\t Max: {_g(max(processed) if processed else 0.0)}",
             dash, "", f"Cuts (feasibility, optimality): {n_feas_cuts} , {n_opt_cuts}", dash,
             "Nodes pruned (feasibility, optimality, bound): ",
             "".join(f"({c.get('pruned_feasibility', 0)}, {c.get('pruned_optimality', 0)}, {c.get('pruned_bound', 0)})  "
                     for c in per_worker),
             dash, "Waiting Time (seconds): " + "".join("0   " for _ in per_worker), dash, ""]
    return "\n".join(lines) + "\n"


def _g(x: float) -> str:
    """std::cout's default formatting of a double (%g with 6 significant digits)."""
    return f"{x:g}"

