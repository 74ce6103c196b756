"""The device B&B against the reference under the cuts the B&B itself makes.

Every cut the reference's search applies comes from GuroSolver::solveSubProblem
(NodeExplorer.cpp:957-969, grb.cpp:236-281); here it comes from k_sub_scenario.  Such rows
have integral / dyadic coefficients, so equal state values and signed zeros are common --
where the strict-`>` argmax (DD.cpp:3834), first-match back-tracking (DD.cpp:3808) and the
std::max / std::min tie rules decide.  Round by round the tests below run the device search
(sgufp_bnb_step with its round trace, include/sgufp_hip.h) and check:

* parity of the round's relaxation: the records the round pops, relaxed under the pool and
  incumbent the round sees, against the reference's own RelaxedDDNew (oracle/_ref/ref_dd
  relaxp): status, exact flag, lb / ub bits, argmax path, cutset children, DD sizes; and the
  round's own k_relax statuses (trace) equal those results;
* bound pruning: a popped record is skipped unprocessed iff ub <= zOpt (DDSolver.cpp:707-711);
* every optimality cut is tight at the path it was generated for (RHS + coef . y-bar ==
  sum_s obj_s / S), every feasibility cut cuts its path off;
* every closed loop's bound (the incumbent candidate, NodeExplorer.cpp:948-956) equals the
  expected scenario value of the matching that closed it, and the incumbent is the best of
  them -- for the incumbent's matching also against HiGHS on the reference's dual LP
  restated (all S scenarios);
* one refinement loop per round replayed step by step on the device (sgufp_batch_refine with
  the subproblem's cuts) against ``ref_dd refine`` fed with the same cuts.

BASELINE configs[2] (C3: 1k arcs, 64 scenarios, incumbent pruning -- seeded by the
restricted-DD heuristic, and unseeded), configs[3]'s network (C4, 256 scenarios) and
configs[4] (C5: 5k arcs, 512 scenarios, cut generation in the loop) are run for a bounded
number of rounds: none of them closes.
"""
import os

import pytest

from oracle import bnb_parity as bp

pytestmark = pytest.mark.gpu

# SGUFP_GPU_LONG=1: the checks whose reference side alone takes minutes (the survivors at 10^5
# optimality cuts: ~150 s of ref_dd per record; the screening-column variant of the exact phase).
# Off by default so that the whole `-m gpu` suite stays inside the driver's 900-s limit; their
# round-6 run is in profiles/r06_gpu_tests.txt (tools/gpu_r06_suite_b.sh sets it).
LONG = os.environ.get("SGUFP_GPU_LONG") == "1"


def _search_rounds(*args, **kw):
    rep = bp.check_search(*args, **kw)
    assert not rep["failures"], "\n".join(rep["failures"][:10])
    return rep


def test_bnb_parity_c3_seeded():
    """BASELINE configs[2]: C3 / 64 scenarios with incumbent pruning, the incumbent seeded by
    the width-64 restricted-DD heuristic (processX3's restricted half); two refinement
    iterations per round keep the pool small enough for the reference's CPU sweeps."""
    seen = _search_rounds("C3", 1, 64, rounds=80, batch=64, sample=32, min_subproblems=1, round_iters=2)
    assert seen["checked"] > 0 and seen["subproblems"] > 0 and seen["opt_cuts"] > 0
    assert seen["replayed"] > 0


def test_bnb_parity_c3_unseeded():
    """configs[2] from the root with no incumbent: the first exact leaves come from the search."""
    seen = _search_rounds("C3", 2, 0, rounds=80, batch=64, sample=32, min_subproblems=1, round_iters=2)
    assert seen["subproblems"] > 0


def test_bnb_parity_m1_loops_close():
    """A 64-scenario network small enough for the refinement loops to close (M1: 60 arcs, 13
    V-bar nodes): unbounded loops, closed bounds == the matchings' expected values, the
    incumbent == the best of them and == HiGHS on the reference's dual LP (64 scenarios)."""
    seen = _search_rounds("M1", 1, 0, rounds=200, batch=64, sample=48, min_closed=4)
    assert seen["closed"] >= 4 and seen["highs_checked"] == 64 and seen["replayed"] > 0


def test_bnb_parity_c4():
    """The headline network (C4: 1k arcs, 256 scenarios), seeded."""
    seen = _search_rounds("C4", 1, 128, rounds=80, batch=64, sample=24, min_subproblems=1, round_iters=2)
    assert seen["subproblems"] > 0


def test_bnb_parity_c5():
    """BASELINE configs[4]: 5k arcs, 512 scenarios, cut generation in the loop."""
    seen = _search_rounds("C5", 1, 0, rounds=80, batch=32, sample=8, round_seconds=3.0, replay=False,
                          min_subproblems=1, rounds_after=1, round_iters=1)
    assert seen["relaxed"] > 0 and seen["subproblems"] > 0


def test_bnb_parity_c4_seeded_at_timed_pool_size():
    """The pool sizes the seeded B&B leg runs against (10^4 cuts, not the 10^2-10^3 of the
    round-by-round checks above): the seeded C4 / 256 search with uncapped refinement loops
    until its optimality list holds 20 000 cuts, then the first batch of the next rounds that
    holds exact leaves (the cut-parallel exact phase) and non-exact records -- under the seeded
    incumbent a cut prunes those (the survivors are covered unseeded, below) -- against ref_dd
    relaxp on the same pool, bit for bit, 8 records of each outcome."""
    rep = bp.check_large_pool("C4", 1, 128, min_opt_cuts=20000, per_kind=8)
    assert not rep["failures"], "\n".join(rep["failures"][:10])
    assert rep["pool_optimality"] >= 20000, rep
    assert rep["sampled"]["exact"] >= 1 and rep["sampled"]["survivor"] + rep["sampled"]["pruned"] >= 1, rep
    assert rep["checked"] >= 8


def _survivors(rep, per_pool, sizes):
    assert not rep["failures"], "\n".join(rep["failures"][:10])
    assert [p["target"] for p in rep["pools"]] == list(sizes), rep
    for p in rep["pools"]:
        assert p["pool_optimality"] >= p["target"], p
        assert p["survivors_checked"] >= per_pool, p          # settled by k_nx_dag / leaf / k_nx_fin
        assert p["children_checked"] >= per_pool, p
        assert p["mismatches"] == 0, p


@pytest.mark.timeout(1500)
def test_bnb_parity_c4_survivors_at_timed_pool_sizes():
    """The survivor path of the non-exact cut-parallel phase at the pool sizes the unseeded
    timed leg (`bnb`) reaches -- 2 x 10^4 and 10^5 optimality cuts (its pool ends near 2.3 x
    10^5): with no incumbent every non-exact record survives every cut, so the round's
    non-exact records are settled by k_nx_dag / k_exact_leaf<nx> / k_nx_fin (sgufp_batch_routes
    says which).  At each pool size 8 such survivors -- status, bounds, argmax path and every
    cutset child (the branching indices) -- and records of the other routes are compared bit for
    bit with ref_dd relaxp (round-5 VERDICT item 1)."""
    sizes = (20000, 100000) if LONG else (20000,)
    rep = bp.check_nx_survivors("C4", 1, sizes, per_pool=8)
    print(rep)
    _survivors(rep, 8, sizes)


@pytest.mark.timeout(1500)
def test_bnb_parity_c3_survivors_at_large_pool():
    """The same on BASELINE configs[2]'s network (C3, 64 scenarios) at 3 x 10^4 optimality cuts
    (6 x 10^4 in round 6's profiles/r06_gpu_tests.txt; the size here keeps the GPU suite inside its
    time limit -- the reference sweeps each survivor's DD once per cut on one host thread)."""
    sizes = (30000,)
    rep = bp.check_nx_survivors("C3", 1, sizes, per_pool=8)
    print(rep)
    _survivors(rep, 8, sizes)


@pytest.mark.parametrize("knob,value", [("SGUFP_EXACT_FAST", "0"), ("SGUFP_EXACT_LAZY", "1"),
                                        ("SGUFP_EXACT_SCREEN", "64")])
def test_bnb_parity_exact_phase_variants(monkeypatch, knob, value):
    if knob == "SGUFP_EXACT_SCREEN" and not LONG:
        pytest.skip("screening columns (off by default): SGUFP_GPU_LONG=1")
    """The other ways the exact DDs' optimality phase can run (capi.cpp, exact_kernels.hip):
    k_relax's own in-order sweeps (deeper / wider exact DDs take it), lazy terminal weights
    completed on demand in k_exact_fin / k_refine, and screening columns swept first -- on M1,
    whose refinement loops close, so k_refine and the argmax paths are exercised too."""
    monkeypatch.setenv(knob, value)
    seen = _search_rounds("M1", 1, 0, rounds=120, batch=64, sample=6, min_closed=2, highs=False)
    assert seen["closed"] >= 2 and seen["replayed"] > 0


def test_bnb_parity_c3_generated_lower_bounds():
    """BASELINE configs[2] as generated (sink-arc lower bounds kept): the scenarios of the paths
    the search sends are infeasible, every subproblem returns the first infeasible scenario's
    ray as a feasibility cut (grb.cpp:284-351), the loop applies it with applyFeasibilityCut's
    cascade (DD.cpp:3842-3930, 4025-4177) -- round by round against ref_dd relaxp under the
    device-made F pool, each new cut checked to cut its path off (round-5 VERDICT item 2)."""
    seen = _search_rounds("C3", 1, 64, rounds=80, batch=64, sample=32, min_subproblems=1, round_iters=2,
                          keep_lb=True, min_feas_cuts=50)
    assert seen["feas_cuts"] >= 50 and seen["checked"] > 0 and seen["mismatches"] == 0


def test_bnb_parity_c5_generated_lower_bounds():
    """BASELINE configs[4] (5k arcs, 512 scenarios, cut generation in the loop) with its
    generated lower bounds kept: the subproblems run the 64-bit-key kernels (big-M costs of the
    lower bounds) and the loop's rounds are checked against ref_dd relaxp under the pools they
    make.  C5's V-bar nodes are sparse (f = 0.08): the paths its search sends meet every sink
    lower bound (r06k: 14 rounds of subproblems, optimality cuts only), so the feasibility-cut
    cascade at scale is pinned by the C3 test above and the C4 large-pool one below."""
    seen = _search_rounds("C5", 1, 0, rounds=80, batch=32, sample=8, round_seconds=3.0, replay=False,
                          min_subproblems=1, rounds_after=2, round_iters=1, keep_lb=True)
    assert seen["subproblems"] > 0 and seen["relaxed"] > 0 and seen["checked"] > 0
    assert seen["opt_cuts"] + seen["feas_cuts"] == seen["subproblems"]


def test_bnb_parity_c4_generated_lower_bounds_at_large_pool():
    """The seeded C4 / 256 search with the generated lower bounds until its pool holds 5 000
    feasibility cuts (the bench's bnb_gen leg reaches ~7k), then the next round's batch against
    ref_dd relaxp on the same pool (records pruned by a feasibility cut, survivors, exact leaves)."""
    rep = bp.check_large_pool("C4", 1, 128, min_opt_cuts=5000, per_kind=8, keep_lb=True)
    assert not rep["failures"], "\n".join(rep["failures"][:10])
    assert rep["pool_feasibility"] >= 5000, rep
    assert rep["checked"] >= 8
