"""The RelaxedDDNew surface (DD.h:797-808) one call at a time on the device, against the
reference's own RelaxedDDNew driven the same way (`ref_dd api`, oracle/ref_driver.cpp).

Per record: buildTree -> isTreeExact; every pool cut newest first with the value each
applyFeasibilityCut / applyOptimalityCut call returns (bit patterns); getSolution after every
4th cut and at the end; getCutset(ub) of a non-exact tree (children bit for bit).  The empty
pool run is DDSolver::startSolver's root DD: buildTree(root) + getCutset(DOUBLE_MAX)
(DDSolver.cpp:788-791).  Fixtures: tests/golden/dd_api/ (make_dd_api.py); the live
reference is used as well when oracle/_ref/ref_dd is present.
"""
import gzip
import json
import os
import subprocess
import tempfile

import numpy as np
import pytest

from sgufp_solver_amd import pools
from tests import golden_io

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
API = os.path.join(HERE, "golden", "dd_api")
REF = os.path.join(ROOT, "oracle", "_ref", "ref_dd")


def parse_api(text):
    """ref_dd api output -> per record dict(exact, vals [(type, value)], sols [path], final,
    ub, children)."""
    lines = text.splitlines()
    n, _ = (int(x) for x in lines[0].split())
    i = 1
    out = []
    for _ in range(n):
        _, exact, applied, nsol = lines[i].split()
        i += 1
        vals = []
        for tok in lines[i].split()[1:]:
            vals.append((tok[0], int(tok[1:]) if tok[0] == "F" else float.fromhex(tok[1:])))
        i += 1
        assert len(vals) == int(applied)
        sols = []
        for _ in range(int(nsol)):
            sols.append([int(x) for x in lines[i].split()[2:]])
            i += 1
        rec = {"exact": int(exact), "vals": vals, "sols": sols, "final": None, "ub": None, "children": None}
        if lines[i].startswith("E"):
            i += 1
            out.append(rec)
            continue
        rec["final"] = [int(x) for x in lines[i].split()[2:]]
        i += 1
        if lines[i].startswith("E"):
            i += 1
            out.append(rec)
            continue
        _, ub, nc = lines[i].split()
        i += 1
        rec["ub"] = float.fromhex(ub)
        ch = []
        for _ in range(int(nc)):
            t = lines[i].split()
            i += 1
            gl, lb, cub, ns = int(t[0]), float.fromhex(t[1]), float.fromhex(t[2]), int(t[3])
            st = [int(x) for x in t[4:4 + ns]]
            nsol2 = int(t[4 + ns])
            sol = [int(x) for x in t[5 + ns:5 + ns + nsol2]]
            ch.append(pools.NodeRecord(gl, lb, cub, st, sol))
        rec["children"] = ch
        out.append(rec)
    return out


def manifest():
    with open(os.path.join(API, "manifest.json")) as fh:
        return json.load(fh)


def cases():
    return [(c["name"], k) for c in manifest() for k in range(len(c["runs"]))]


def device_trace(eng, nodes, cuts, inc):
    """The same calls as ref_dd api, through sgufp_dd_* (engine.Engine.dd_*)."""
    exact = eng.dd_build(nodes)
    out = []
    for k in range(len(nodes)):
        ex = int(exact[k])
        ub = nodes[k].ub
        vals, sols, pruned = [], [], False
        for c in reversed(cuts):
            v = eng.dd_apply(k, c, inc)
            if c.type == 1:
                vals.append(("F", int(v)))
                pruned = v == 0.0
            else:
                vals.append(("O", v))
                ub = v if ex else min(v, ub)
                pruned = v <= inc
            if pruned:
                break
            if len(vals) % 4 == 0:
                sols.append(eng.dd_solution(k))
        rec = {"exact": ex, "vals": vals, "sols": sols, "final": None, "ub": None, "children": None}
        if not pruned:
            rec["final"] = eng.dd_solution(k)
            if not ex:
                rec["ub"] = ub
                rec["children"] = eng.dd_cutset(k, ub)
        out.append(rec)
    return out


def compare(got, want):
    bad = []
    for k, (g, w) in enumerate(zip(got, want)):
        if g["exact"] != w["exact"]:
            bad.append(f"record {k}: exact {g['exact']} vs {w['exact']}")
            continue
        if len(g["vals"]) != len(w["vals"]):
            bad.append(f"record {k}: {len(g['vals'])} calls vs {len(w['vals'])}")
        for j, (a, b) in enumerate(zip(g["vals"], w["vals"])):
            if a[0] != b[0] or (a[0] == "F" and a[1] != b[1]) or (a[0] == "O" and golden_io.bits(a[1]) != golden_io.bits(b[1])):
                bad.append(f"record {k} call {j}: {a} vs {b}")
                break
        if g["sols"] != w["sols"]:
            bad.append(f"record {k}: intermediate getSolution differs")
        if g["final"] != w["final"]:
            bad.append(f"record {k}: final getSolution differs")
        if (g["ub"] is None) != (w["ub"] is None) or (g["ub"] is not None and golden_io.bits(g["ub"]) != golden_io.bits(w["ub"])):
            bad.append(f"record {k}: cutset ub {g['ub']} vs {w['ub']}")
        if w["children"] is not None:
            gc, wc = g["children"] or [], w["children"]
            if len(gc) != len(wc):
                bad.append(f"record {k}: {len(gc)} children vs {len(wc)}")
            else:
                for c, (x, y) in enumerate(zip(gc, wc)):
                    if (x.gl, x.states, x.sol) != (y.gl, y.states, y.sol) or golden_io.bits(x.lb) != golden_io.bits(y.lb) \
                            or golden_io.bits(x.ub) != golden_io.bits(y.ub):
                        bad.append(f"record {k} child {c} differs")
                        break
    if len(got) != len(want):
        bad.append(f"{len(got)} records vs {len(want)}")
    return bad


def test_api_fixtures_parse():
    """CPU: every committed trace parses and covers exact and non-exact trees, pruning
    calls of both types and cutsets."""
    kinds = set()
    for name, k in cases():
        c = [x for x in manifest() if x["name"] == name][0]
        with gzip.open(os.path.join(API, c["runs"][k]["file"]), "rb") as fh:
            recs = parse_api(fh.read().decode())
        for r in recs:
            kinds.add(("exact", r["exact"]))
            if r["vals"] and r["vals"][-1] in (("F", 0),):
                kinds.add("F-prune")
            if r["children"] is not None:
                kinds.add("cutset")
            if r["vals"] and r["vals"][-1][0] == "O" and r["final"] is None:
                kinds.add("O-prune")
    assert {("exact", 0), ("exact", 1), "F-prune", "O-prune", "cutset"} <= kinds, kinds


@pytest.mark.gpu
@pytest.mark.parametrize("name,k", cases())
def test_dd_api_matches_reference(native_lib, name, k):
    from sgufp_solver_amd import engine as E
    c = [x for x in manifest() if x["name"] == name][0]
    run = c["runs"][k]
    d = golden_io.case_dir(name)
    nodes = pools.read_nodes(os.path.join(API, c["nodes"]))
    cuts = pools.read_pool(os.path.join(d, "cuts.txt")) if run["pool"] else []
    inc = float.fromhex(run["incumbent"])
    with gzip.open(os.path.join(API, run["file"]), "rb") as fh:
        want = parse_api(fh.read().decode())
    eng = E.Engine(os.path.join(d, "net.txt"), 0, 64)
    try:
        got = device_trace(eng, nodes, cuts, inc)
    finally:
        eng.close()
    bad = compare(got, want)
    assert not bad, "\n".join(bad[:10])
    if os.path.exists(REF):
        # the live reference on the same inputs (it travels with the tree as a built binary)
        with tempfile.TemporaryDirectory() as t:
            cp = os.path.join(t, "cuts.txt")
            if cuts:
                pools.write_pool(cp, cuts)
            else:
                with open(cp, "w") as fh:
                    fh.write("0\n")
            o = os.path.join(t, "out.txt")
            subprocess.run([REF, "api", os.path.join(d, "net.txt"), cp, os.path.join(API, c["nodes"]), inc.hex(), o],
                           check=True, capture_output=True)
            with open(o) as fh:
                live = parse_api(fh.read())
        assert not compare(got, live)


@pytest.mark.gpu
@pytest.mark.parametrize("name,k", [("c2_s2_dfs", 1), ("c3_s1_dfs", 1), ("c3_s1_dfs", 2)])
def test_cpp_relaxeddd_matches_reference(native_lib, name, k):
    """The C++ API's Inavap::RelaxedDDNew (include/sgufp/inavap.hpp), driven call by call by
    tests/host/host_api_test.cpp "dd", against the same reference trace (run k = 2 of
    c3_s1_dfs is the empty pool: DDSolver::startSolver's buildTree(root) + getCutset)."""
    c = [x for x in manifest() if x["name"] == name][0]
    run = c["runs"][k]
    d = golden_io.case_dir(name)
    with tempfile.TemporaryDirectory() as t:
        cp = os.path.join(t, "cuts.txt")
        if run["pool"]:
            pools.write_pool(cp, pools.read_pool(os.path.join(d, "cuts.txt")))
        else:
            with open(cp, "w") as fh:
                fh.write("0\n")
        exe = os.path.join(ROOT, "sgufp_solver_amd", "lib", "host_api_test")
        r = subprocess.run([exe, "dd", os.path.join(d, "net.txt"), cp, os.path.join(API, c["nodes"]), run["incumbent"]],
                           capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    with gzip.open(os.path.join(API, run["file"]), "rb") as fh:
        want = parse_api(fh.read().decode())
    bad = compare(parse_api(r.stdout), want)
    assert not bad, "\n".join(bad[:10])


@pytest.mark.gpu
def test_dd_view_ends_with_a_batch_relaxation(native_lib):
    """sgufp_dd_* read a slot's DD through its own dense row (d_ddrow); a batch relaxation,
    refinement or B&B round rewrites the slot's last-cut index with a pool index, so after one
    of them the sgufp_dd_* view is gone: SGUFP_ERR_STATE, not an out-of-bounds read (round-5
    ADVICE).  A refine right after a build is allowed (the build left no cut-parallel state)."""
    from sgufp_solver_amd import engine as E
    c = [x for x in manifest() if x["name"] == "c2_s2_dfs"][0]
    d = golden_io.case_dir("c2_s2_dfs")
    nodes = pools.read_nodes(os.path.join(API, c["nodes"]))
    eng = E.Engine(os.path.join(d, "net.txt"), 0, 64)
    try:
        eng.add_cuts(pools.read_pool(os.path.join(d, "cuts.txt")))
        eng.dd_build(nodes)
        eng.dd_solution(0)                     # the view is live after the build
        eng.relax_async(pools.DOUBLE_MIN)      # the same staged batch, relaxed against the pool
        eng.sync()
        for call in (lambda: eng.dd_solution(0), lambda: eng.dd_cutset(0, pools.DOUBLE_MAX)):
            with pytest.raises(RuntimeError, match=r"\(-5\)"):
                call()
    finally:
        eng.close()


@pytest.mark.gpu
def test_warm_slot_arguments_checked(native_lib):
    """sgufp_subproblem_warm: a slot written twice, or read and written by one call, is an
    argument error; the ring keeps its size (2 x max(max_batch, 32) slots) across calls."""
    from sgufp_solver_amd import engine as E
    from sgufp_solver_amd import instance
    import tempfile as tf
    inst = instance.generate(instance.CONFIGS["C3"], 1, scenarios=4)
    with tf.TemporaryDirectory() as t:
        net = os.path.join(t, "net.txt")
        inst.write(net)
        _, la, _ = E.probe_network(net)
        rng = np.random.default_rng(5)
        paths = [instance.random_matching_path(inst, la, rng) for _ in range(3)]
        eng = E.Engine(net, 0, 16)
        try:
            eng.subproblem(paths[:2], [-1, -1], [0, 1])
            with pytest.raises(RuntimeError, match=r"\(-1\)"):
                eng.subproblem(paths[:2], [-1, -1], [2, 2])      # one slot written twice
            with pytest.raises(RuntimeError, match=r"\(-1\)"):
                eng.subproblem(paths[:2], [0, 3], [3, 4])        # slot 3 read and written
            with pytest.raises(RuntimeError, match=r"\(-1\)"):
                eng.subproblem(paths[:1], [64], [5])             # beyond 2 x max(16, 32) slots
            typ, _, _, _ = eng.subproblem(paths, [0, 1, -1], [40, 41, 63])   # 40 slots later: still valid
            assert (typ >= 0).all()
        finally:
            eng.close()
