"""The library's own multi-shard exchanges (shard.cpp) with W > 1 shards on ONE GPU.

RCCL refuses two ranks on one device, so the native path of the 8-GPU run is exercised here
through the in-process loopback transport (sgufp_comm_init_loopback): the same code -- balance
plan, chunk spans, field-by-field send / receive, solution-offset rebase, drop-bottom, row
gather / append -- with device-to-device copies between W contexts driven by W threads.
Checked bit for bit against the torch.distributed driver's protocol (shards.py, LocalComm:
plan, packed records, frontier_take / frontier_push), and end to end: a W = 3 search reaches
the extensive-form optimum.  Replaces DDSolver.cpp:603-652,723-731 (work sharing, incumbent
CAS), lock_free_queue.h:125-164 (m_pop) and the global Containers of DDSolver.h:415-416.
"""
import os
import tempfile
import threading

import numpy as np
import pytest

from sgufp_solver_amd import engine as E
from sgufp_solver_amd import instance, pools
from sgufp_solver_amd.pools import DOUBLE_MIN
from tests import golden_io

pytestmark = pytest.mark.gpu
os.environ.setdefault("SGUFP_LOOPBACK_TIMEOUT", "60")


def run_threads(fns):
    out = [None] * len(fns)
    err = []

    def body(k):
        try:
            out[k] = fns[k]()
        except BaseException as e:   # noqa: BLE001
            err.append(e)
    ts = [threading.Thread(target=body, args=(k,)) for k in range(len(fns))]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    if err:
        raise err[0]
    return out


def frontier_records(eng):
    n = eng.frontier_size()
    return E.batch_to_records(eng.frontier_peek(0, n)) if n else []


def same_records(a, b):
    if len(a) != len(b):
        return False
    for x, y in zip(a, b):
        if (x.gl, x.states, x.sol) != (y.gl, y.states, y.sol):
            return False
        if golden_io.bits(x.lb) != golden_io.bits(y.lb) or golden_io.bits(x.ub) != golden_io.bits(y.ub):
            return False
    return True


SPLITS = {2: [100, 0], 3: [70, 0, 25], 4: [0, 60, 0, 5]}


@pytest.mark.parametrize("world", [2, 3, 4])
def test_loopback_balance_matches_shards_protocol(native_lib, world):
    from sgufp_solver_amd.shards import LocalComm, LocalGroup
    d = golden_io.case_dir("c2_s2_dfs")
    net = os.path.join(d, "net.txt")
    recs = pools.read_nodes(os.path.join(d, "nodes.txt"))
    parts, o = [], 0
    for sz in SPLITS[world]:
        parts.append(recs[o:o + sz])
        o += sz
    # native: loopback transport, sgufp_frontier_balance
    grp = E.LoopbackGroup(world)
    nat = [E.Engine(net, 0, 64) for _ in range(world)]
    for r, e in enumerate(nat):
        e.comm_init_loopback(grp, r)
        e.frontier_clear()
        if parts[r]:
            e.frontier_push(parts[r])
    got = run_threads([lambda e=e: e.frontier_balance() for e in nat])
    # shards.py protocol on separate contexts
    lg = LocalGroup(world)
    py = [E.Engine(net, 0, 64) for _ in range(world)]
    for r, e in enumerate(py):
        e.frontier_clear()
        if parts[r]:
            e.frontier_push(parts[r])
    sizes = [len(p) for p in parts]
    want = run_threads([lambda e=e, r=r: LocalComm(lg, r).rebalance(e, sizes) for r, e in enumerate(py)])
    try:
        assert got == want, (got, want)
        assert sum(got) > 0
        for r in range(world):
            assert same_records(frontier_records(nat[r]), frontier_records(py[r])), f"rank {r}"
        total = sum(len(frontier_records(e)) for e in nat)
        assert total == sum(sizes)
    finally:
        for e in nat + py:
            e.close()
        grp.close()


@pytest.mark.parametrize("world", [2, 3, 4])
def test_loopback_cuts_exchange_matches_shards_protocol(native_lib, world):
    from sgufp_solver_amd.shards import LocalComm, LocalGroup
    d = golden_io.case_dir("c2_s2_dfs")
    net = os.path.join(d, "net.txt")
    inst = instance.generate(instance.CONFIGS["C2"], 2, scenarios=1)
    mine = [pools.synthetic_pool(inst, (r * 3) % 4, (r * 5) % 7, 100 + r) for r in range(world)]
    grp = E.LoopbackGroup(world)
    nat = [E.Engine(net, 0, 16) for _ in range(world)]
    py = [E.Engine(net, 0, 16) for _ in range(world)]
    for r in range(world):
        nat[r].comm_init_loopback(grp, r)
        for e in (nat[r], py[r]):
            if mine[r]:
                e.add_cuts(mine[r])
    got = run_threads([lambda e=e: e.cuts_exchange() for e in nat])
    lg = LocalGroup(world)
    want = run_threads([lambda e=e, r=r: LocalComm(lg, r).exchange_cuts(e, {1: 0, 0: 0}) for r, e in enumerate(py)])
    try:
        assert got == want, (got, want)
        for r in range(world):
            for t in (1, 0):
                a, b = nat[r].cut_rows(t), py[r].cut_rows(t)
                assert a[0].tobytes() == b[0].tobytes() and a[1].tobytes() == b[1].tobytes(), (r, t)
        # every shard holds the same global pool (rows in a shard-dependent order: own rows first)
        for t in (1, 0):
            ref = sorted(map(bytes, [np.concatenate([[x], y]).tobytes() for x, y in zip(*nat[0].cut_rows(t))]))
            for r in range(1, world):
                cur = sorted(map(bytes, [np.concatenate([[x], y]).tobytes() for x, y in zip(*nat[r].cut_rows(t))]))
                assert cur == ref
        # the incumbent CAS: all-reduce(MAX)
        zs = run_threads([lambda e=e, r=r: e.incumbent_allreduce(float(r) * 7.5 - 3.0) for r, e in enumerate(nat)])
        assert zs == [float(world - 1) * 7.5 - 3.0] * world
    finally:
        for e in nat + py:
            e.close()
        grp.close()


T4_64 = float.fromhex("0x1.b664400000000p+12")   # tests/test_bnb.py: HiGHS extensive form of T4-1-64z


def test_loopback_three_shard_search_reaches_the_optimum(native_lib):
    from sgufp_solver_amd.solver import DDSolver
    inst = instance.generate(instance.CONFIGS["T4"], 1, scenarios=64)
    inst.lb[:] = 0
    path = os.path.join(tempfile.mkdtemp(prefix="sgufp_nat_"), "net.txt")
    inst.write(path)
    world = 3
    grp = E.LoopbackGroup(world)
    engs = [E.Engine(path, 0, 256) for _ in range(world)]
    for r, e in enumerate(engs):
        e.comm_init_loopback(grp, r)
    solvers = [DDSolver(engine=engs[r], batch_nodes=16, verbose=False, native_world=world, max_rounds=20000)
               for r in range(world)]
    try:
        zs = run_threads([lambda s=s: s.start_solver(DOUBLE_MIN) for s in solvers])
        assert all(abs(z - T4_64) <= 1e-5 * abs(T4_64) for z in zs), zs
        assert all(s.complete for s in solvers)
        assert sum(s.received for s in solvers) > 0          # work sharing moved records
        assert sum(s.counters["relaxed"] > 0 for s in solvers) >= 2
    finally:
        for e in engs:
            e.close()
        grp.close()
