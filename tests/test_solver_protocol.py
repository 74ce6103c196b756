"""Multi-rank DDSolver protocol on CPU (gloo, world size 2 and 3).

sgufp_solver_amd/solver.py sequences B&B rounds and does the reference's shared-memory
exchanges with collectives: incumbent all-reduce(MAX) (DDSolver.cpp:723-731), all-gather
of new cut rows (global Containers, DDSolver.h:415-416), frontier rebalancing (master
half-split / 40 % steal, DDSolver.cpp:603-652) and termination (:630-640).  The engine is
a toy knapsack B&B with the Engine's frontier / bnb_step / cut-row surface (test
infrastructure), so the protocol is checked without a GPU: every rank ends with the
brute-force optimum and identical cut pools, and every leaf is closed exactly once.
"""
import itertools
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from sgufp_solver_amd.engine import BatchArrays, batch_concat, batch_slice
from sgufp_solver_amd.pools import NodeRecord
from sgufp_solver_amd.solver import DDSolver

D = 12
RNG = np.random.default_rng(7)
W = RNG.integers(1, 20, size=D).astype(float)
A = RNG.integers(1, 10, size=D).astype(float)
CAP = float(A.sum() * 0.45)


def brute():
    best = 0.0
    for x in itertools.product([0, 1], repeat=D):
        if np.dot(A, x) <= CAP:
            best = max(best, float(np.dot(W, x)))
    return best


class ToyEngine:
    """Knapsack B&B with the frontier / round / cut-row interface of engine.Engine."""

    def __init__(self):
        self.stack = []          # NodeRecord, top = end
        self.cuts = {0: [], 1: []}
        self.closed = []         # leaves closed on this rank

    def _ub(self, sol):
        d = len(sol)
        v = float(np.dot(W[:d], sol))
        return v + float(W[d:].sum())

    def frontier_clear(self):
        self.stack = []

    def frontier_size(self):
        return len(self.stack)

    def frontier_push(self, recs):
        if isinstance(recs, BatchArrays):
            recs = [NodeRecord(int(recs.gl[k]), float(recs.lb[k]), float(recs.ub[k]),
                               [int(s) for s in recs.states[recs.states_off[k]:recs.states_off[k + 1]]],
                               [int(s) for s in recs.sol[recs.sol_off[k]:recs.sol_off[k + 1]]])
                    for k in range(recs.n)]
        self.stack.extend(recs)

    def frontier_take(self, n, from_bottom=True):
        if from_bottom:
            out, self.stack = self.stack[:n], self.stack[n:]
        else:
            out, self.stack = self.stack[len(self.stack) - n:], self.stack[:len(self.stack) - n]
        return BatchArrays(out)

    def cuts_count(self, t):
        return len(self.cuts[t])

    def cut_rows(self, t, first=0, count=None):
        rows = self.cuts[t][first:first + (len(self.cuts[t]) - first if count is None else count)]
        return np.array([r[0] for r in rows]), np.array([r[1] for r in rows]).reshape(len(rows), 2)

    def add_cut_rows(self, t, rhs, rows):
        for h, r in zip(rhs, rows):
            self.cuts[t].append((float(h), tuple(float(x) for x in r)))

    def bnb_step(self, z, max_nodes=0):
        b = min(len(self.stack), max_nodes or 4)
        batch = self.stack[len(self.stack) - b:]
        del self.stack[len(self.stack) - b:]
        st = {k: 0 for k in ("popped", "relaxed", "pruned_bound", "pruned_feasibility", "pruned_optimality", "exact",
                             "exact_closed", "subproblems", "new_feasibility_cuts", "new_optimality_cuts",
                             "children", "pushed")}
        st["popped"] = b
        best = z
        kids = []
        for nd in batch:
            if nd.ub <= z:
                st["pruned_bound"] += 1
                continue
            st["relaxed"] += 1
            sol = nd.sol
            if float(np.dot(A[:len(sol)], sol)) > CAP:
                st["pruned_feasibility"] += 1
                self.cuts[1].append((-1.0, (float(len(sol)), float(sum(sol)))))
                st["new_feasibility_cuts"] += 1
                continue
            if len(sol) == D:
                st["exact"] += 1
                st["exact_closed"] += 1
                v = float(np.dot(W, sol))
                self.closed.append(tuple(sol))
                self.cuts[0].append((v, (float(D), float(sum(sol)))))
                st["new_optimality_cuts"] += 1
                best = max(best, v)
                continue
            for x in (0, 1):
                s2 = list(sol) + [x]
                kids.append((nd, NodeRecord(len(s2), -1e300, self._ub(s2), [], s2)))
            st["children"] += 2
        for parent, c in kids:
            if parent.ub > best:
                self.stack.append(c)
                st["pushed"] += 1
        return best, st


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    eng = ToyEngine()
    solver = DDSolver(engine=eng, batch_nodes=3, verbose=False)
    z = solver.start_solver(-1.0)
    q.put((rank, z, sorted(eng.cuts[0]), sorted(eng.cuts[1]), eng.closed, solver.counters, solver.rounds,
           solver.received))
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world", [2, 3])
def test_multi_rank_solver_protocol(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    opt = brute()
    res.sort()
    for rank, z, c0, c1, closed, counters, rounds, received in res:
        assert z == opt, (rank, z, opt)
    # identical global pools on every rank (all-gathered rows)
    assert all(r[2] == res[0][2] and r[3] == res[0][3] for r in res)
    # every closed leaf closed by exactly one rank, and the work was shared
    leaves = [t for r in res for t in r[4]]
    assert len(leaves) == len(set(leaves))
    assert sum(1 for r in res if r[5]["relaxed"] > 0) == world


def test_work_sharing_balances_shards():
    """World 3, every record starts on rank 0: ranks 1 and 2 run dry and are fed from every
    busy shard (40 % of a stack of >= 32 from its bottom, m_pop; half of a smaller one), so
    both receive records and the relaxed counts end up within 1.5x of each other."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    world = 3
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    relaxed = [r[5]["relaxed"] for r in res]
    received = [r[7] for r in res]
    assert received[1] > 0 and received[2] > 0, received
    assert max(relaxed) <= 1.5 * min(relaxed), relaxed


def test_work_sharing_plan():
    """give counts follow m_pop(0.4) from 32 records up, the half split below; idle ranks
    are the empty ones; nothing moves while no shard is idle."""
    from sgufp_solver_amd.shards import give_count, plan
    assert give_count(100) == 100 - int(100 * 0.6) == 40
    assert give_count(32) == 32 - int(32 * 0.6) == 13
    assert give_count(31) == 15 and give_count(2) == 1 and give_count(1) == 0
    assert plan([5, 7]) == ([], [])
    assert plan([0, 100, 3, 0]) == ([(1, 40), (2, 1)], [0, 3])


def test_native_balance_plan_matches_shards_plan():
    """The C ABI's work-sharing plan (shard.cpp balance_plan / chunk_of, behind
    sgufp_frontier_balance's RCCL sends) == shards.plan and ShardComm.rebalance's chunking on
    random stack-size vectors (host only: no device is touched)."""
    from sgufp_solver_amd.engine import balance_plan
    from sgufp_solver_amd.shards import plan
    rng = np.random.default_rng(7)
    cases = [[0], [5], [0, 0], [1, 0], [0, 100, 3, 0], [5, 7], [31, 0, 32, 0, 0, 1]]
    for _ in range(300):
        w = int(rng.integers(1, 9))
        sizes = [int(x) if rng.random() > 0.35 else 0 for x in rng.integers(0, 5000, size=w)]
        if rng.random() < 0.3:
            sizes = [int(x) for x in rng.integers(0, 40, size=w)]
        cases.append(sizes)
    for sizes in cases:
        give, idle, lo, hi = balance_plan(sizes)
        donors, idle_py = plan(sizes)
        assert idle == (idle_py if donors else []), sizes
        assert {r: int(g) for r, g in enumerate(give) if g > 0} == dict(donors), sizes
        for r, g in donors:
            for j in range(len(idle)):
                assert (lo[r, j], hi[r, j]) == (g * j // len(idle), g * (j + 1) // len(idle)), (sizes, r, j)
            assert hi[r, len(idle) - 1] == g          # the chunks cover the donor's records


def test_record_pack_roundtrip():
    from sgufp_solver_amd.shards import pack_batch, unpack_batch
    recs = [NodeRecord(3, -1.5, 7.25, [1, 4], [2, -1, 5]), NodeRecord(0, -1e300, 1e300, [], []),
            NodeRecord(9, 0.0, 2.0, [-1, 3, 8], [1] * 9)]
    b = unpack_batch(pack_batch(BatchArrays(recs)))
    assert b.n == 3
    for k, r in enumerate(recs):
        assert int(b.gl[k]) == r.gl and b.lb[k] == r.lb and b.ub[k] == r.ub
        assert list(b.states[b.states_off[k]:b.states_off[k + 1]]) == r.states
        assert list(b.sol[b.sol_off[k]:b.sol_off[k + 1]]) == r.sol


def test_single_rank_toy_matches_brute_force():
    eng = ToyEngine()
    z = DDSolver(engine=eng, batch_nodes=5, verbose=False).start_solver(-1.0)
    assert z == brute()


def test_toy_frontier_order_is_a_stack():
    eng = ToyEngine()
    recs = [NodeRecord(1, 0.0, float(k), [], [k % 2]) for k in range(6)]
    eng.frontier_push(recs)
    top = eng.frontier_take(2, from_bottom=False)
    assert list(top.ub) == [4.0, 5.0]
    bot = eng.frontier_take(2, from_bottom=True)
    assert list(bot.ub) == [0.0, 1.0]
    assert batch_concat([bot, top]).n == 4 and batch_slice(bot, np.array([1])).ub[0] == 1.0


def test_worker_stats_format():
    """printWorkerStats (DDSolver.h:441-501): 72-wide dash lines, processed counts with
    total / mean / absolute deviation / min / max, cut counts, per-worker prunes."""
    from sgufp_solver_amd.solver import worker_stats_text
    txt = worker_stats_text([{"relaxed": 10, "pruned_optimality": 3, "pruned_feasibility": 1},
                             {"relaxed": 14, "pruned_bound": 2}], 1, 5)
    lines = txt.split("\n")
    assert lines[0] == "-" * 72
    assert lines[1] == "Processed: 10  14  "
    assert lines[2] == "Total: 24\t Mean: 12\t Deviation: 0\t Min: 10\t Max: 14"   # statistics.h:31-33 stub
    assert "Cuts (feasibility, optimality): 1 , 5" in lines
    assert "(1, 3, 0)  (0, 0, 2)  " in lines
    assert lines[-3] == "-" * 72 and lines[-2] == "" and lines[-1] == ""   # dash, endl, endl


@pytest.mark.parametrize("world", [2, 3])
def test_in_process_shards_protocol(world):
    """Several frontier shards as threads of one process (shards.LocalComm: one device context
    each, e.g. on one GPU) run the same exchanges: every shard ends with the brute-force
    optimum and the same global cut pool, every leaf is closed once, and every shard works."""
    from sgufp_solver_amd.shards import LocalComm, LocalGroup, run_local_shards
    group = LocalGroup(world)
    engines = [ToyEngine() for _ in range(world)]
    solvers = [DDSolver(engine=engines[r], batch_nodes=3, verbose=False, comm=LocalComm(group, r))
               for r in range(world)]
    zs = run_local_shards(solvers, lambda s: s.start_solver(-1.0))
    opt = brute()
    assert all(z == opt for z in zs), (zs, opt)
    assert all(sorted(e.cuts[0]) == sorted(engines[0].cuts[0]) and sorted(e.cuts[1]) == sorted(engines[0].cuts[1])
               for e in engines)
    leaves = [t for e in engines for t in e.closed]
    assert len(leaves) == len(set(leaves))
    assert all(s.counters["relaxed"] > 0 for s in solvers)
    assert all(s.complete for s in solvers)
