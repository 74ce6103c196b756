"""Restricted decision diagram (Inavap::RestrictedDDNew, /root/reference/DD.cpp:3090-3505) under
the restricted cut phases of NodeExplorer::processX3 (NodeExplorer.cpp:605-656): compile with a
width limit, feasibility cuts then optimality cuts of the pool (newest first), the max path.

CPU: the clean-room restatement (oracle/dd_oracle.cpp "restricted") reproduces the reference's
own output (tests/golden/restricted/, made by oracle/_ref/ref_dd, see make_restricted.py)
byte for byte.  GPU: k_restrict through the C ABI, bit-exact on status, exactness, the bound's
bit pattern, the max path and the exact cutset (states, solution vector, global layer)."""
import os
import struct
import subprocess

import pytest

from tests import golden_io

CASES = [(c["name"], r) for c in golden_io.restricted_manifest() for r in c["runs"]]
IDS = [f"{c}-w{r['width']}-{r['file']}" for c, r in CASES]


@pytest.mark.parametrize("name,run", CASES, ids=IDS)
def test_oracle_restricted_matches_reference(oracle_bin, tmp_path, name, run):
    d = golden_io.restricted_dir(name)
    src = golden_io.case_dir(name)
    out = tmp_path / "r.txt"
    subprocess.run([oracle_bin, "restricted", f"{src}/net.txt", f"{src}/cuts.txt", f"{d}/nodes.txt", run["incumbent"],
                    str(run["width"]), str(out)], check=True)
    assert out.read_text() == golden_io.read_restricted(name, run["file"])


def test_restricted_fixtures_cover_every_outcome():
    seen = set()
    for name, run in CASES:
        for st, ex, lb, path, kids in golden_io.parse_restricted_text(golden_io.read_restricted(name, run["file"])):
            seen.add((st, ex))
    assert {(0, 0), (0, 1), (1, 0), (2, 0), (2, 1)} <= seen


def _bits(x):
    return struct.unpack("<Q", struct.pack("<d", x))[0]


@pytest.mark.gpu
@pytest.mark.parametrize("name,run", CASES, ids=IDS)
def test_restricted_matches_reference(name, run):
    from sgufp_solver_amd import engine as E
    from sgufp_solver_amd import pools
    src = golden_io.case_dir(name)
    d = golden_io.restricted_dir(name)
    nodes = pools.read_nodes(os.path.join(d, "nodes.txt"))
    e = E.Engine(os.path.join(src, "net.txt"), 0, max(256, len(nodes)))
    e.add_cuts(pools.read_pool(os.path.join(src, "cuts.txt")))
    got = e.restricted(nodes, float.fromhex(run["incumbent"]), int(run["width"]))
    e.close()
    want = golden_io.parse_restricted_text(golden_io.read_restricted(name, run["file"]))
    assert len(got) == len(want)
    bad = []
    for k, (g, w) in enumerate(zip(got, want)):
        gs, gx, glb, gp, gk = g
        ws, wx, wlb, wp, wk = w
        if (gs, gx) != (ws, wx) or _bits(glb) != _bits(wlb) or gp != wp:
            bad.append(f"node {k}: got {(gs, gx, glb.hex(), len(gp))} want {(ws, wx, wlb.hex(), len(wp))}")
            continue
        if len(gk) != len(wk):
            bad.append(f"node {k}: {len(gk)} cutset nodes, want {len(wk)}")
            continue
        for a, b in zip(gk, wk):
            if (a.gl, a.states, a.sol) != (b.gl, b.states, b.sol) or _bits(a.lb) != _bits(b.lb) or _bits(a.ub) != _bits(b.ub):
                bad.append(f"node {k}: cutset record differs: {a} vs {b}")
                break
    assert not bad, "\n".join(bad[:10])


# ------------------------------------------------------------------ primal heuristic (GPU)
HEUR = [("T1", 2, 3), ("T2", 1, 1), ("T3", 2, 3), ("T4", 3, 3)]


@pytest.mark.gpu
@pytest.mark.parametrize("cfg,seed,S", HEUR, ids=[f"{c}-{s}-{S}" for c, s, S in HEUR])
def test_restricted_heuristic_incumbent_is_a_feasible_value(cfg, seed, S):
    """processX3's restricted refinement on the root record: a converged bound is the value
    of its routing (the subproblem's mean objective at the final path, 1e-9 relative), never
    above the extensive-form optimum (1e-5, main.cpp:43,76), and seeding the DDSolver with it
    leaves the optimum unchanged."""
    import tempfile
    from oracle import extensive_form as ef
    from sgufp_solver_amd import engine as E
    from sgufp_solver_amd import instance
    from sgufp_solver_amd.pools import DOUBLE_MAX, DOUBLE_MIN, NodeRecord
    from sgufp_solver_amd.restricted import RestrictedExplorer
    from sgufp_solver_amd.solver import DDSolver
    inst = instance.generate(instance.CONFIGS[cfg], seed, scenarios=S)
    inst.lb[:] = 0
    d = tempfile.mkdtemp(prefix="sgufp_rh_")
    path = os.path.join(d, "net.txt")
    inst.write(path)
    opt = ef.solve(inst)
    eng = E.Engine(path, 0, 64)
    res = RestrictedExplorer(eng, 128).explore([NodeRecord(0, DOUBLE_MIN, DOUBLE_MAX, [], [])], DOUBLE_MIN)[0]
    assert res.status == 0 and res.converged, (res.status, res.iterations)
    typ, rhs, rows, obj_mean = eng.subproblem([res.path])
    eng.close()
    assert typ[0] == 0
    assert abs(res.lb - obj_mean[0]) <= 1e-9 * max(1.0, abs(obj_mean[0])), (res.lb, obj_mean[0])
    assert res.lb <= opt + 1e-5 * max(1.0, abs(opt)), (res.lb, opt)
    solver = DDSolver(path, max_batch=1024, max_rounds=20000, verbose=False, restricted_width=128)
    sol, _ = solver.start(DOUBLE_MIN)
    solver.eng.close()
    assert solver.heuristic_incumbent == res.lb
    assert abs(sol - opt) <= 1e-5 * max(1.0, abs(opt)), (sol, opt)
