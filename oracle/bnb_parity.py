"""B&B parity under real Benders pools (TEST INFRASTRUCTURE ONLY).

The device B&B (sgufp_bnb_step) applies only cuts its own scenario subproblem produced
(NodeExplorer.cpp:957-969 -> grb.cpp:236-281): rows with integral or dyadic coefficients,
where equal state values and signed zeros are common -- exactly where the reference's
strict-`>` argmax (DD.cpp:3834), first-match back-tracking (DD.cpp:3808) and std::max /
std::min tie behaviour decide the result.  This module reads such a pool and the next
frontier batch back from a running search and hands them to the reference's own
RelaxedDDNew (oracle/_ref/ref_dd, built from /root/reference by oracle/Makefile):

* ``pool_of``       the context's F and O lists (insertion order) as (i, q, j, v) cuts --
                    cutToCut's form (Cut.h:406-421: zero coefficients dropped);
* ``snapshot_top``  the next b frontier records (the batch the next round pops), left on
                    the frontier;
* ``ref_relax``     ``ref_dd relaxp`` over records / pool / incumbent (NodeExplorer::process
                    up to the first subproblem call);
* ``ref_refine``    ``ref_dd refine``: process(), then a refinement loop fed with given cuts;
* ``refine_replay`` the device refinement loop of one exact record, step by step
                    (sgufp_batch_refine with the subproblem's cuts), for ref_refine.

Only tests/ and bench.py's parity legs import this module; nothing in the product does.
"""
from __future__ import annotations

import os
import subprocess
import sys
import tempfile
from typing import List, Sequence

import numpy as np

from sgufp_solver_amd import engine as E
from sgufp_solver_amd import pools
from sgufp_solver_amd.pools import PoolCut

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_BIN = os.path.join(ROOT, "oracle", "_ref", "ref_dd")


def decode_key(key: int):
    """(i, q, j) of Inavap::getKey(q, i, j) = q | i << 16 | j << 32 (Cut.h:342-344)."""
    return (key >> 16) & 0xFFFF, key & 0xFFFF, (key >> 32) & 0xFFFF


def rows_to_cuts(keys: np.ndarray, typ: int, rhs: np.ndarray, rows: np.ndarray) -> List[PoolCut]:
    """Dense rows (slot order, sgufp_slot_keys) -> the reference's cut form: one (i, q, j)
    entry per non-zero slot (cutToCut drops v == 0, so +0.0 and -0.0 alike)."""
    ijk = [decode_key(int(k)) for k in keys]
    if len(set(ijk)) != len(ijk):
        raise ValueError("duplicate slot keys: the dense row has no unique (i, q, j) form")
    out = []
    for c in range(len(rhs)):
        row = rows[c]
        coeff = [(i, q, j, float(row[s])) for s, (i, q, j) in enumerate(ijk) if row[s] != 0.0]
        out.append(PoolCut(typ, float(rhs[c]), coeff))
    return out


def pool_of(eng: E.Engine) -> List[PoolCut]:
    """The context's global pool: feasibility list then optimality list, each in insertion
    order (ref_dd applies each list newest first, as the Containers are read)."""
    keys = eng.slot_keys()
    out: List[PoolCut] = []
    for t in (1, 0):
        if eng.cuts_count(t):
            rhs, rows = eng.cut_rows(t)
            out += rows_to_cuts(keys, t, rhs, rows)
    return out


def snapshot_top(eng: E.Engine, b: int) -> E.BatchArrays:
    """The top min(b, frontier) records in stack order (what the next round pops), left in place."""
    total = eng.frontier_size()
    n = min(b, total)
    if n == 0:
        return E.BatchArrays([])
    return eng.frontier_peek(total - n, n)


def _threads() -> int:
    try:
        return max(1, min(16, len(os.sched_getaffinity(0))))
    except AttributeError:
        return max(1, min(16, os.cpu_count() or 1))


def ref_relax(net: str, pool: Sequence[PoolCut], records: Sequence[pools.NodeRecord], z: float,
              work: str = None, threads: int = 0) -> List[pools.RelaxResult]:
    work = work or tempfile.mkdtemp(prefix="sgufp_bnbpar_")
    cuts, nodes, out = (os.path.join(work, f) for f in ("cuts.txt", "nodes.txt", "ref.txt"))
    pools.write_pool(cuts, pool)
    pools.write_nodes(nodes, records)
    subprocess.run([REF_BIN, "relaxp", net, cuts, nodes, z.hex(), str(threads or _threads()), out], check=True,
                   capture_output=True, timeout=900)
    return pools.read_results(out)


def ref_refine(net: str, pool: Sequence[PoolCut], records: Sequence[pools.NodeRecord], z: float,
               extra: Sequence[PoolCut], work: str = None) -> List[pools.RelaxResult]:
    work = work or tempfile.mkdtemp(prefix="sgufp_bnbpar_")
    cuts, nodes, xc, out = (os.path.join(work, f) for f in ("cuts.txt", "nodes.txt", "extra.txt", "ref.txt"))
    pools.write_pool(cuts, pool)
    pools.write_nodes(nodes, records)
    pools.write_pool(xc, extra)
    subprocess.run([REF_BIN, "refine", net, cuts, nodes, z.hex(), xc, out], check=True, capture_output=True,
                   timeout=900)
    return pools.read_results(out)


def load_pool(eng: E.Engine, pool: Sequence[PoolCut]):
    eng.add_cuts(list(pool))


def refine_replay(eng: E.Engine, record: pools.NodeRecord, z: float, max_iters: int = 64):
    """NodeExplorer::process's refinement loop (NodeExplorer.cpp:946-969) for one exact
    record on the device, one step at a time: relax (status 3 = needs the subproblem), then
    until the argmax path repeats: subproblem on the path -> append the cut to the pool
    (sgufp_cuts_append_rows) -> apply it in place (sgufp_batch_refine).  ``eng`` holds the
    round's pool.  Returns (the cuts appended in order, per step the device state after it:
    (status, ub, path)); the loop's own end state is the last entry."""
    keys = eng.slot_keys()
    eng.upload([record])
    eng.relax_async(z)
    eng.sync()
    res = eng._collect()[0]
    states = [(res.status, res.ub, list(res.path))]
    extra: List[PoolCut] = []
    seen = []
    while res.status == E.NEEDS_SUBPROBLEM and len(extra) < max_iters:
        path = list(res.path)
        if path in seen:
            break
        seen.append(path)
        typ, rhs, rows, _ = eng.subproblem([path])
        if int(typ[0]) < 0:
            raise RuntimeError("subproblem failed on a replayed path")
        t = int(typ[0])
        eng.add_cut_rows(t, rhs[:1], rows[:1])
        extra += rows_to_cuts(keys, t, rhs[:1], rows[:1])
        idx = eng.cuts_count(t) - 1
        eng.refine([0], [t], [idx], z)
        res = eng._collect()[0]
        states.append((res.status, res.ub, list(res.path)))
    return extra, states


# ---------------------------------------------------------------- round-by-round search check
TOL = 1e-9


def _bits(x: float) -> int:
    import struct
    return struct.unpack("<q", struct.pack("<d", x))[0]


def _node_key(nd):
    return (nd.gl, _bits(nd.lb), _bits(nd.ub), tuple(nd.states), tuple(nd.sol))


def compare(got, want) -> List[str]:
    """Bit-exact NodeExplorer::process outcomes: status, exact flag, lb / ub bits, argmax path,
    cutset children (the branching indices), DD sizes."""
    bad = []
    if len(got) != len(want):
        return [f"result count {len(got)} != {len(want)}"]
    for k, (g, w) in enumerate(zip(got, want)):
        why = None
        if (g.status, g.exact) != (w.status, w.exact):
            why = f"status/exact {(g.status, g.exact)} != {(w.status, w.exact)}"
        elif _bits(g.lb) != _bits(w.lb) or _bits(g.ub) != _bits(w.ub):
            why = f"bounds {(g.lb, g.ub)} != {(w.lb, w.ub)}"
        elif g.path != w.path:
            why = "argmax path differs"
        elif [_node_key(c) for c in g.children] != [_node_key(c) for c in w.children]:
            why = f"children differ ({len(g.children)} vs {len(w.children)})"
        elif (g.dd_nodes, g.dd_arcs, g.dd_layers) != (w.dd_nodes, w.dd_arcs, w.dd_layers):
            why = "DD size differs"
        if why:
            bad.append(f"record {k}: {why}")
    return bad


def _cut_at(rhs: float, row, ijk, y) -> float:
    """RHS + coef . y-bar over a dense row (slot order; the DD's layer order differs, so the
    comparison below is to TOL)."""
    v = rhs
    for s, t in enumerate(ijk):
        if row[s] != 0.0 and y.get(t, 0):
            v += row[s]
    return v


def check_search(cfg: str, seed: int, width: int, rounds: int, batch: int, sample: int, round_seconds: float = 5.0,
                 replay: bool = True, highs: bool = True, device: int = 0, min_subproblems: int = 0,
                 rounds_after: int = 3, min_closed: int = 0, round_iters: int = 0, keep_lb: bool = False,
                 min_feas_cuts: int = 0):
    """Run the device B&B (sgufp_bnb_step, traced) on a seeded instance of ``cfg`` (lower
    bounds 0; keep_lb: the generator's sink-arc lower bounds, so that scenarios are infeasible
    and the loop generates feasibility cuts, grb.cpp:284-351, applied with their cascade,
    DD.cpp:3842-3930, 4025-4177) -- the incumbent seeded by the restricted-DD heuristic of
    ``width`` (0: none) --
    and check every round against the reference.  The search dives (LIFO batches of ``batch``
    records) until at least ``min_subproblems`` subproblems and ``min_closed`` closed loops
    were seen, then runs ``rounds_after`` more rounds; ``rounds`` caps the total.  ``round_iters``
    bounds each round's refinement loops (sgufp_bnb_set_limits; 0: none) -- one C3 round of 64
    exact records otherwise appends ~17k cuts, which the reference then sweeps for minutes per
    record.  Returns a report whose "failures" list is empty on parity:

    * the records the round pops (``sample`` of them), relaxed under the round's pool and
      incumbent, == ``ref_dd relaxp`` bit for bit, and the round's own k_relax statuses ==
      those results;
    * a popped record is skipped unprocessed iff ub <= zOpt (DDSolver.cpp:707-711);
    * optimality cuts are tight at their path (RHS + coef . y-bar == sum_s obj_s / S, TOL
      relative), feasibility cuts cut their path off;
    * a closed loop's bound == sum_s obj_s / S of the matching that closed it, the incumbent
      == the best of them (DDSolver.cpp:723-731), and (highs, S <= 256) the best one == HiGHS
      on the reference's dual LP restated, over every scenario;
    * (replay) one refinement loop, step by step on the device, == ``ref_dd refine`` fed with
      the same cuts."""
    import time
    from oracle import subproblem_oracle as so
    from sgufp_solver_amd import instance
    from sgufp_solver_amd.pools import DOUBLE_MAX, DOUBLE_MIN, NodeRecord
    t0 = time.perf_counter()
    inst = instance.generate(instance.CONFIGS[cfg], seed)
    if not keep_lb:
        inst.lb[:] = 0                   # feasible scenarios: optimality cuts and incumbents
    work = tempfile.mkdtemp(prefix="sgufp_bnbpar_")
    net = os.path.join(work, "net.txt")
    inst.write(net)
    _, la, _ = E.probe_network(net)
    sn = so.from_instance(inst, la)
    eng = E.Engine(net, device, max(batch, sample))
    ijk = [decode_key(int(k)) for k in eng.slot_keys()]
    eng.bnb_set_trace(True)
    root = NodeRecord(0, DOUBLE_MIN, DOUBLE_MAX, [], [])
    z = DOUBLE_MIN
    if width:
        from sgufp_solver_amd.restricted import RestrictedExplorer
        z = RestrictedExplorer(eng, width).incumbent([root], z)
    eng.frontier_clear()
    eng.frontier_push([root])
    fail: List[str] = []
    rep = {"config": cfg, "seed": seed, "scenarios": int(inst.scenarios), "heuristic_width": width,
           "lower_bounds": "generated" if keep_lb else "zero",
           "rounds": 0, "batch": batch, "checked": 0, "mismatches": 0, "subproblems": 0, "opt_cuts": 0,
           "feas_cuts": 0, "closed": 0, "pruned_bound": 0, "relaxed": 0, "replayed": 0, "pool_last": 0,
           "incumbent_start": z, "highs_checked": 0}
    obj_of = {}                          # path -> sum_s obj_s / S of its subproblem
    feas_paths = set()
    best = None                          # (value, path) of the best closed loop
    replay_src = None
    after = None
    for r in range(rounds):
        if eng.frontier_size() == 0:
            break
        if after is None and rep["subproblems"] >= min_subproblems and rep["closed"] >= min_closed and \
                rep["feas_cuts"] >= min_feas_cuts:
            after = r
        if after is not None and r - after >= rounds_after:
            break
        eng.bnb_set_limits(round_iters, round_seconds)
        snap = snapshot_top(eng, batch)
        pool = pool_of(eng)
        z0 = z
        want = None
        if pool:
            idx = np.arange(snap.n) if snap.n <= sample else np.linspace(0, snap.n - 1, sample).astype(np.int64)
            recs = E.batch_to_records(E.batch_slice(snap, idx))
            got = eng.relax(recs, z0)
            want = ref_relax(net, pool, recs, z0, work)
            bad = compare(got, want)
            rep["checked"] += len(recs)
            rep["mismatches"] += len(bad)
            fail += [f"round {r}: {m}" for m in bad[:5]]
            rep["pool_last"] = len(pool)
            if replay and replay_src is None and any(w.status == E.NEEDS_SUBPROBLEM for w in want):
                k = next(i for i, w in enumerate(want) if w.status == E.NEEDS_SUBPROBLEM)
                replay_src = (list(pool), recs[k], z0)
        z, st = eng.bnb_step(z, batch)
        rep["rounds"] += 1
        popped = eng.bnb_trace(0)
        subs = eng.bnb_trace(1)
        closed = eng.bnb_trace(2)
        if len(popped) != st.popped:
            fail.append(f"round {r}: trace has {len(popped)} popped records, stats {st.popped}")
        for rec, code, _, ub_in, _ in popped:
            if (code == E.PRUNED_BOUND) != (ub_in <= z0):
                fail.append(f"round {r}: record {rec} ub {ub_in!r} z {z0!r} status {code}")
        rep["pruned_bound"] += int(st.pruned_bound)
        rep["relaxed"] += int(st.relaxed)
        if want is not None:
            by_rec = {rk: c for rk, c, _, _, _ in popped}
            for k, w in zip(idx, want):
                if snap.ub[k] > z0 and by_rec.get(int(k)) != w.status:
                    fail.append(f"round {r}: record {int(k)} round status {by_rec.get(int(k))} != {w.status}")
        for rec, typ, row, obj, path in subs:
            if typ not in (0, 1):
                fail.append(f"round {r}: subproblem of record {rec} has cut type {typ}")
                continue
            rhs, rows = eng.cut_rows(typ, row, 1)
            y = so.ybar_of_path(sn, path)
            v = _cut_at(float(rhs[0]), rows[0], ijk, y)
            if typ == 0:
                rep["opt_cuts"] += 1
                obj_of[tuple(path)] = obj
                if not abs(v - obj) <= TOL * max(1.0, abs(obj)):
                    fail.append(f"round {r}: optimality cut of record {rec} not tight: {v!r} vs {obj!r}")
            else:
                rep["feas_cuts"] += 1
                feas_paths.add(tuple(path))
                if not v < 0:
                    fail.append(f"round {r}: feasibility cut of record {rec} keeps its path ({v!r})")
        rep["subproblems"] += len(subs)
        for rec, _, _, ub, path in closed:
            p = tuple(path)
            if p in obj_of:
                if not abs(ub - obj_of[p]) <= TOL * max(1.0, abs(obj_of[p])):
                    fail.append(f"round {r}: closed record {rec} bound {ub!r} != E[Q] {obj_of[p]!r}")
                if best is None or ub > best[0]:
                    best = (ub, path)
            elif p not in feas_paths:
                fail.append(f"round {r}: closed record {rec} on a path no subproblem of the search solved")
        rep["closed"] += len(closed)
        print(f"[bnb parity {cfg}] round {r}: popped {st.popped} relaxed {st.relaxed} subproblems {len(subs)} "
              f"closed {len(closed)} pool {len(pool)} checked {rep['checked']} failures {len(fail)} "
              f"{time.perf_counter() - t0:.1f} s", file=sys.stderr, flush=True)
        zc = max([z0] + [c[3] for c in closed])
        if z != zc:
            fail.append(f"round {r}: incumbent {z!r} != max(zOpt, closed bounds) {zc!r}")
    rep["incumbent"] = z
    eng.close()
    if best is not None and highs and sn.S <= 256:
        y = so.ybar_of_path(sn, best[1])
        vals = [so.dual_lp(sn, y, s)[:2] for s in range(sn.S)]
        if not all(w == "optimal" for w, _ in vals):
            fail.append("best closed matching is infeasible for HiGHS")
        else:
            mean = sum(o for _, o in vals) / sn.S
            rep["highs_checked"] = sn.S
            rep["best_closed"] = best[0]
            rep["best_closed_highs"] = mean
            if not abs(best[0] - mean) <= TOL * max(1.0, abs(mean)):
                fail.append(f"best closed bound {best[0]!r} != HiGHS E[Q] {mean!r}")
    if replay_src is not None:
        pool, rec, zr = replay_src
        pe = E.Engine(net, device, 4)
        try:
            load_pool(pe, pool)
            extra, states = refine_replay(pe, rec, zr, 12)
        finally:
            pe.close()
        for step in range(1, len(extra) + 1):
            ref = ref_refine(net, pool, [rec], zr, extra[:step], work)[0]
            stt, ub, path = states[step]
            if ref.status != stt:
                fail.append(f"replay step {step}: status {stt} != reference {ref.status}")
            elif stt == E.NEEDS_SUBPROBLEM and (_bits(ref.ub) != _bits(ub) or ref.path != path):
                fail.append(f"replay step {step}: bound / path differ ({ub!r} vs {ref.ub!r})")
        rep["replayed"] = len(extra)
    rep["failures"] = fail
    rep["seconds"] = round(time.perf_counter() - t0, 2)
    return rep


# ---------------------------------------------------------------- parity at the timed pool sizes
def write_pool_bin(path: str, eng: E.Engine) -> int:
    """The context's pool (feasibility list, then optimality list, insertion order) as the
    binary dense-row file ``ref_dd`` reads for large pools (oracle/ref_driver.cpp
    read_cuts_bin).  Returns the number of cuts."""
    keys = np.asarray(eng.slot_keys(), dtype=np.uint64)
    ns = len(keys)
    types, rhs, rows = [], [], []
    for t in (1, 0):
        n = eng.cuts_count(t)
        if n:
            r, w = eng.cut_rows(t)
            types.append(np.full(n, t, np.int32))
            rhs.append(np.asarray(r, np.float64))
            rows.append(np.ascontiguousarray(np.asarray(w, np.float64)[:, :ns]))
    nc = int(sum(len(x) for x in types))
    with open(path, "wb") as fh:
        fh.write(np.array([nc, ns], dtype=np.int64).tobytes())
        fh.write(keys.tobytes())
        for part in (types, rhs):
            for x in part:
                fh.write(x.tobytes())
        for x in rows:
            fh.write(x.tobytes())
    return nc


def check_large_pool(cfg: str, seed: int, width: int, min_opt_cuts: int, batch: int = 1024, per_kind: int = 8,
                     round_seconds: float = 5.0, max_seconds: float = 240.0, device: int = 0, threads: int = 0,
                     need_rounds: int = 12, keep_lb: bool = False):
    """Parity at the pool sizes the timed B&B runs against: the seeded search of ``cfg`` (lower
    bounds 0; incumbent from the width-``width`` restricted-DD heuristic) runs untraced, with
    uncapped refinement loops, until its optimality list holds ``min_opt_cuts`` cuts.  The next
    round's batch (``batch`` records, what sgufp_bnb_step pops) is relaxed on the device under
    that pool and incumbent -- exact records through the cut-parallel phase (k_exact_cols /
    k_exact_root / k_exact_leaf / k_exact_fin), non-exact survivors through k_relax's batched
    sweeps -- and ``per_kind`` records of each outcome (exact leaves needing the subproblem,
    non-exact survivors with cutsets, records pruned by a cut) are compared bit for bit with
    ``ref_dd relaxp`` on the same pool (NodeExplorer.cpp:935-944 / 975-985, DD.cpp:3932-4023).
    The round itself then runs and its statuses must equal the device relaxation's."""
    import time
    from sgufp_solver_amd import instance
    from sgufp_solver_amd.pools import DOUBLE_MAX, DOUBLE_MIN, NodeRecord
    t0 = time.perf_counter()
    inst = instance.generate(instance.CONFIGS[cfg], seed)
    if not keep_lb:
        inst.lb[:] = 0
    work = tempfile.mkdtemp(prefix="sgufp_bigpool_")
    net = os.path.join(work, "net.txt")
    inst.write(net)
    eng = E.Engine(net, device, batch)
    root = NodeRecord(0, DOUBLE_MIN, DOUBLE_MAX, [], [])
    z = DOUBLE_MIN
    if width:
        from sgufp_solver_amd.restricted import RestrictedExplorer
        z = RestrictedExplorer(eng, width).incumbent([root], z)
    eng.frontier_clear()
    eng.frontier_push([root])
    rep = {"config": cfg, "seed": seed, "heuristic_width": width, "rounds": 0, "search_seconds": 0.0,
           "lower_bounds": "generated" if keep_lb else "zero"}
    diving = True
    # (with the generated lower bounds the paths are infeasible: the pool is feasibility cuts)
    count = (lambda: eng.cuts_count(0) + eng.cuts_count(1)) if keep_lb else (lambda: eng.cuts_count(0))
    while count() < min_opt_cuts and eng.frontier_size() and time.perf_counter() - t0 < max_seconds:
        eng.bnb_set_limits(0, round_seconds)
        z, st = eng.bnb_step(z, 64 if diving else batch)
        if st.exact:
            diving = False
        rep["rounds"] += 1
    rep["search_seconds"] = round(time.perf_counter() - t0, 2)
    rep["pool_feasibility"] = eng.cuts_count(1)
    rep["pool_optimality"] = eng.cuts_count(0)
    rep["incumbent"] = z
    fail: List[str] = []
    # the first batch (within a few more rounds) that holds both exact leaves and non-exact
    # survivors, so that the sample covers the cut-parallel exact phase and the non-exact one
    for attempt in range(need_rounds + 1):
        snap = snapshot_top(eng, batch)
        recs = E.batch_to_records(snap)
        got_all = eng.relax(recs, z)
        kinds = {"exact": [], "survivor": [], "pruned": []}
        for k, g in enumerate(got_all):
            if snap.ub[k] <= z:
                continue                                     # skipped unprocessed by the round
            kind = "exact" if g.status == E.NEEDS_SUBPROBLEM else ("survivor" if g.status == 0 else "pruned")
            if len(kinds[kind]) < per_kind:
                kinds[kind].append(k)
        if (kinds["exact"] and kinds["survivor"]) or attempt == need_rounds or not eng.frontier_size():
            break
        eng.bnb_set_limits(0, round_seconds)
        z, st = eng.bnb_step(z, batch)
        rep["rounds"] += 1
    rep["pool_feasibility"] = eng.cuts_count(1)
    rep["pool_optimality"] = eng.cuts_count(0)
    rep["incumbent"] = z
    idx = sorted(i for v in kinds.values() for i in v)
    rep["sampled"] = {k: len(v) for k, v in kinds.items()}
    rep["batch"] = len(recs)
    pool_path = os.path.join(work, "pool.bin")
    rep["pool_total"] = write_pool_bin(pool_path, eng)
    nodes = os.path.join(work, "nodes.txt")
    out = os.path.join(work, "ref.txt")
    pools.write_nodes(nodes, [recs[i] for i in idx])
    t1 = time.perf_counter()
    subprocess.run([REF_BIN, "relaxp", net, pool_path, nodes, z.hex(), str(threads or _threads()), out], check=True,
                   capture_output=True, timeout=1800)
    rep["reference_seconds"] = round(time.perf_counter() - t1, 2)
    want = pools.read_results(out)
    bad = compare([got_all[i] for i in idx], want)
    rep["checked"] = len(idx)
    rep["mismatches"] = len(bad)
    fail += bad[:10]
    # the round itself on the same batch, pool and incumbent
    eng.bnb_set_trace(True)
    eng.bnb_set_limits(1, round_seconds)
    z2, st = eng.bnb_step(z, batch)
    by_rec = {rk: c for rk, c, _, _, _ in eng.bnb_trace(0)}
    for i in idx:
        if by_rec.get(i) != got_all[i].status:
            fail.append(f"record {i}: round status {by_rec.get(i)} != device relaxation {got_all[i].status}")
    eng.close()
    rep["failures"] = fail
    rep["seconds"] = round(time.perf_counter() - t0, 2)
    return rep


def check_nx_survivors(cfg: str, seed: int, pool_sizes=(20000, 100000), per_pool: int = 8, batch: int = 1024,
                       round_seconds: float = 5.0, max_seconds: float = 300.0, device: int = 0, threads: int = 0,
                       need_rounds: int = 12, keep_lb: bool = False, round_iters: int = 4):
    """The survivor path of the non-exact cut-parallel phase at the pool sizes the timed B&B
    legs reach.  The UNSEEDED search of ``cfg`` (no incumbent: nothing is pruned by a bound, so
    the non-exact records of a round survive every cut and take the whole phase: k_nx_dag per
    64-cut block, k_exact_leaf<nx> leaf passes, k_nx_fin's outcome and cutset) runs until its
    optimality list holds each of ``pool_sizes`` cuts in turn.  There the next round's batch is
    relaxed on the device, sgufp_batch_routes says which records the phase settled
    (ROUTE_NX_PHASE) and ``per_pool`` survivors among them (status SUCCESS, cutset children:
    the branching indices) are compared bit for bit with ``ref_dd relaxp`` on a binary copy of
    the pool -- status, exact flag, lb / ub bits, argmax path, every child, DD sizes
    (NodeExplorer.cpp:975-985, DD.cpp:3932-4023, 4179-4218) -- together with up to per_pool / 2
    records of each other route present (in-order, fall-back re-run).  The round then runs on
    the same batch and its statuses must equal the device relaxation's.

    The search's own closed loops soon set an incumbent, and a round's batch may then hold exact
    records only.  So the survivors come from the first non-exact batch the search pushed (the
    root's cutset children, kept from round 1): at each pool size they are relaxed with no
    incumbent (DOUBLE_MIN, device and reference alike: every record survives every cut) and the
    phase's survivors among them are compared.  ``round_iters`` caps the refinement iterations
    per round (sgufp_bnb_set_limits) so that the pool passes each size gradually instead of in
    one round of uncapped loops; the survivors compared are those with the smallest DDs."""
    import time
    from sgufp_solver_amd import instance
    from sgufp_solver_amd.pools import DOUBLE_MAX, DOUBLE_MIN, NodeRecord
    t0 = time.perf_counter()
    inst = instance.generate(instance.CONFIGS[cfg], seed)
    if not keep_lb:
        inst.lb[:] = 0
    work = tempfile.mkdtemp(prefix="sgufp_nxsurv_")
    net = os.path.join(work, "net.txt")
    inst.write(net)
    eng = E.Engine(net, device, batch)
    eng.frontier_clear()
    eng.frontier_push([NodeRecord(0, DOUBLE_MIN, DOUBLE_MAX, [], [])])
    z = DOUBLE_MIN
    fail: List[str] = []
    rep = {"config": cfg, "seed": seed, "lower_bounds": "generated" if keep_lb else "zero", "rounds": 0,
           "pools": []}
    early = None                         # the root's cutset children (non-exact), kept from round 1
    for target in pool_sizes:
        while eng.cuts_count(0) < target and eng.frontier_size() and time.perf_counter() - t0 < max_seconds:
            eng.bnb_set_limits(round_iters, round_seconds)
            z, _ = eng.bnb_step(z, batch)
            rep["rounds"] += 1
            if early is None:
                early = E.batch_to_records(snapshot_top(eng, batch))
        if eng.cuts_count(0) < target:
            fail.append(f"pool {target}: the search stopped at {eng.cuts_count(0)} optimality cuts")
            break
        # the next round's batch under the search's incumbent: the other routes
        snap = snapshot_top(eng, batch)
        recs = E.batch_to_records(snap)
        got_all = eng.relax(recs, z)
        routes = eng.routes()
        by = {r: [] for r in (E.ROUTE_IN_ORDER, E.ROUTE_EXACT_PHASE, E.ROUTE_NX_PHASE, E.ROUTE_NX_FALLBACK)}
        for k, g in enumerate(got_all):
            if snap.ub[k] > z:
                by[int(routes[k])].append(k)
        # (at a first pool size of at most 3 x 10^4 only: the reference spends minutes per exact
        # record at 10^5 cuts, and the exact route at the timed pools has its own test)
        extra = []
        if target == pool_sizes[0] and target <= 30000:
            for r in (E.ROUTE_IN_ORDER, E.ROUTE_NX_FALLBACK, E.ROUTE_EXACT_PHASE, E.ROUTE_NX_PHASE):
                extra += by[r][:max(1, per_pool // 2)]
        idx = sorted(set(extra))
        # the survivors: the kept non-exact records with no incumbent
        got_e = eng.relax(early, DOUBLE_MIN)
        routes_e = eng.routes()
        surv = [k for k, g in enumerate(got_e)
                if routes_e[k] == E.ROUTE_NX_PHASE and g.status == E.SUCCESS and not g.exact and g.children]
        # the per_pool survivors with the smallest DDs (the reference sweeps each one's DD once per
        # cut on one host thread: minutes per record at 10^5 cuts for the largest)
        pick = sorted(sorted(surv, key=lambda k: (got_e[k].dd_nodes, k))[:per_pool])
        pool_path = os.path.join(work, f"pool_{target}.bin")
        total = write_pool_bin(pool_path, eng)
        t1 = time.perf_counter()
        bad = []
        for tag, zz, rs, gs in (("batch", z, [recs[i] for i in idx], [got_all[i] for i in idx]),
                                ("survivors", DOUBLE_MIN, [early[i] for i in pick], [got_e[i] for i in pick])):
            if not rs:
                continue
            nodes = os.path.join(work, f"nodes_{target}_{tag}.txt")
            out = os.path.join(work, f"ref_{target}_{tag}.txt")
            pools.write_nodes(nodes, rs)
            subprocess.run([REF_BIN, "relaxp", net, pool_path, nodes, zz.hex(), str(threads or _threads()), out],
                           check=True, capture_output=True, timeout=1800)
            bad += [f"{tag}: {m}" for m in compare(gs, pools.read_results(out))]
        fail += [f"pool {target}: {m}" for m in bad[:10]]
        n_ch = sum(len(got_e[i].children) for i in pick)
        entry = {"target": target, "pool_optimality": eng.cuts_count(0), "pool_feasibility": eng.cuts_count(1),
                 "pool_total": total, "incumbent": z, "batch": len(recs),
                 "routes_in_batch": {name: len(by[r]) for name, r in (("in_order", E.ROUTE_IN_ORDER),
                                                                      ("exact_phase", E.ROUTE_EXACT_PHASE),
                                                                      ("nx_phase", E.ROUTE_NX_PHASE),
                                                                      ("nx_fallback", E.ROUTE_NX_FALLBACK))},
                 "nx_survivors": len(surv), "survivor_candidates": len(early), "survivors_checked": len(pick),
                 "children_checked": n_ch, "checked": len(idx) + len(pick), "mismatches": len(bad),
                 "reference_seconds": round(time.perf_counter() - t1, 2)}
        rep["pools"].append(entry)
        print(f"[nx survivors {cfg}] pool {entry['pool_optimality']}: routes {entry['routes_in_batch']} "
              f"survivors checked {len(pick)} ({n_ch} children) mismatches {len(bad)} "
              f"ref {entry['reference_seconds']} s, {time.perf_counter() - t0:.1f} s", file=sys.stderr, flush=True)
        # the round itself on the same batch, pool and incumbent (its statuses vs the device
        # relaxation above, for the records checked)
        eng.bnb_set_trace(True)
        eng.bnb_set_limits(1, round_seconds)
        z, _ = eng.bnb_step(z, batch)
        rep["rounds"] += 1
        by_rec = {rk: c for rk, c, _, _, _ in eng.bnb_trace(0)}
        for i in idx:
            if by_rec.get(i) != got_all[i].status:
                fail.append(f"pool {target}: record {i}: round status {by_rec.get(i)} != device relaxation "
                            f"{got_all[i].status}")
        eng.bnb_set_trace(False)
    eng.close()
    rep["failures"] = fail
    rep["seconds"] = round(time.perf_counter() - t0, 2)
    return rep
