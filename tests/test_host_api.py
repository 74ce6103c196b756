"""The C++ host mirror of the reference API (include/sgufp/inavap.hpp, libsgufp_host.so).

CPU: the library exports the reference's class surface (Network, Inavap::NodeExplorer::process,
Inavap::GuroSolver::solveSubProblem, Inavap::DDSolver::start / startSolver, Container::add).
GPU: tests/host/host_api_test.cpp solves seeded instances three times -- Inavap::DDSolver::start
(batched device rounds), the same as a one-rank RCCL shard with deferred refinement loops
(DDSolver::shard, the exchanges of shard.cpp after every round), and a reference-style
single-worker LIFO loop over
NodeExplorer::process with two global Containers (DDSolver.cpp:658-776) -- and both optima
must equal the extensive form within 1e-5 (main.cpp:43,76).
"""
import os
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "sgufp_solver_amd", "lib")


def test_host_library_exports_reference_api(native_lib):
    out = subprocess.run(["nm", "-DC", "--defined-only", os.path.join(LIB, "libsgufp_host.so")],
                         capture_output=True, text=True, check=True).stdout
    for sym in ["Network::Network(", "Inavap::NodeExplorer::process(", "Inavap::GuroSolver::solveSubProblem(",
                "Inavap::DDSolver::start(", "Inavap::DDSolver::startSolver(", "Inavap::Cut::get("]:
        assert sym in out, sym
    # Inavap::Container (add / get / destructor) is header-only: include/sgufp/inavap.hpp
    assert os.access(os.path.join(LIB, "host_api_test"), os.X_OK)


@pytest.mark.gpu
@pytest.mark.parametrize("cfg,seed,S,seeding", [("T1", 2, 3, "none"), ("T3", 1, 1, "opt-10"), ("T4", 1, 1, "none"),
                                                 ("T4", 3, 3, "opt-10")])
def test_host_api_solves_to_the_extensive_form_optimum(cfg, seed, S, seeding):
    from oracle import extensive_form as ef
    from sgufp_solver_amd import instance
    inst = instance.generate(instance.CONFIGS[cfg], seed, scenarios=S)
    path = os.path.join(tempfile.mkdtemp(prefix="sgufp_host_"), "net.txt")
    inst.write(path)
    opt = ef.solve(inst)
    known = (opt - 10.0).hex() if seeding == "opt-10" else "none"
    r = subprocess.run([os.path.join(LIB, "host_api_test"), path, known], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr
    got = {}
    for line in r.stdout.splitlines():
        parts = line.split()
        if parts and parts[0] in ("ddsolver", "explorer", "sharded"):
            got[parts[0]] = float.fromhex(parts[1])
    assert "Optimal solution:" in r.stdout
    for k in ("ddsolver", "explorer", "sharded"):
        assert abs(got[k] - opt) <= 1e-5 * max(1.0, abs(opt)), (k, got, opt)


def test_container_is_race_free_under_tsan(tmp_path):
    """SURVEY.md §5 (race detection): Inavap::Container, the lock-free cut pool of the C++ host
    API (include/sgufp/inavap.hpp; Cut.h:448-485 in the reference), under ThreadSanitizer with
    concurrent writers and readers walking the list (tests/host/container_tsan.cpp)."""
    import shutil
    import subprocess
    here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cxx = shutil.which("g++")
    if cxx is None:
        pytest.skip("g++ missing")
    exe = str(tmp_path / "container_tsan")
    r = subprocess.run([cxx, "-std=c++17", "-O1", "-g", "-fsanitize=thread", "-pthread",
                        f"-I{os.path.join(here, 'include')}", os.path.join(here, "tests", "host", "container_tsan.cpp"),
                        "-o", exe], capture_output=True, text=True)
    if r.returncode != 0:
        pytest.skip("ThreadSanitizer toolchain unavailable: " + r.stderr[-200:])
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1:exitcode=66")
    r = subprocess.run([exe], capture_output=True, text=True, env=env, timeout=120)
    if "unexpected memory mapping" in r.stderr:
        # the TSan runtime cannot map its shadow under this kernel's address-space randomisation
        # (an environment limit, seen on the GPU boxes): run it without randomisation
        setarch = shutil.which("setarch")
        if setarch:
            r = subprocess.run([setarch, os.uname().machine, "-R", exe], capture_output=True, text=True, env=env,
                               timeout=120)
        if "unexpected memory mapping" in r.stderr:
            pytest.skip("ThreadSanitizer cannot map its shadow memory here: " + r.stderr[-200:])
    assert "ThreadSanitizer" not in r.stderr, r.stderr[-2000:]
    assert r.returncode == 0, (r.returncode, r.stdout, r.stderr[-500:])
    assert "cuts 8000 (expected 8000)" in r.stdout


def _cpp_search(net, width, seconds, batch, round_seconds, round_iters, max_rounds):
    r = subprocess.run([os.path.join(LIB, "host_api_test"), "search", net, str(width), str(seconds), str(batch),
                        str(round_seconds), str(round_iters), str(max_rounds)], capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    out = {"counters": {}}
    for line in r.stdout.splitlines():
        p = line.split()
        if p[0] == "search":
            out.update(incumbent=float.fromhex(p[1]), heuristic=float.fromhex(p[2]), seconds=float(p[3]),
                       rounds=int(p[4]), complete=p[5] == "1")
        elif p[0] == "counter":
            out["counters"][p[1]] = int(p[2])
        elif p[0] == "pool":
            out["pool"] = [int(p[1]), int(p[2])]
    return out


@pytest.mark.gpu
def test_cpp_ddsolver_matches_python_driver_at_scale():
    """BASELINE configs[2] (C3, 1k arcs, 64 scenarios) through the C++ host path a maintainer
    links (Inavap::DDSolver with restricted-DD seeding, DDSolver.cpp:782-867) and through the
    Python driver the bench uses (solver.DDSolver): 30 rounds of 1 024 records with two
    refinement iterations per round (no wall-clock limit, so both searches are reproducible)
    must give the same incumbent, the same heuristic seed, the same counters round for round
    and the same pool."""
    from sgufp_solver_amd import instance
    from sgufp_solver_amd.pools import DOUBLE_MIN
    from sgufp_solver_amd.solver import DDSolver
    inst = instance.generate(instance.CONFIGS["C3"], 1)
    inst.lb[:] = 0
    net = os.path.join(tempfile.mkdtemp(prefix="sgufp_host_"), "net.txt")
    inst.write(net)
    # unseeded: the dive reaches exact leaves (subproblems, cuts, refinement) within the rounds
    # (seeded by the width-64 heuristic, 30 rounds of this search stayed above the exact layers)
    cpp = _cpp_search(net, 0, 0, 1024, 0, 2, 60)
    s = DDSolver(net, max_batch=1024, verbose=False, restricted_width=0, round_iters=2, stop_rounds=60)
    z = s.start_solver(DOUBLE_MIN)
    pool = [s.eng.cuts_count(1), s.eng.cuts_count(0)]
    s.eng.close()
    assert cpp["rounds"] == s.rounds == 60
    assert cpp["heuristic"] == (DOUBLE_MIN if s.heuristic_incumbent is None else s.heuristic_incumbent)
    assert cpp["incumbent"] == z
    assert cpp["counters"] == {k: int(v) for k, v in s.counters.items()}, (cpp["counters"], s.counters)
    assert cpp["pool"] == pool
    assert cpp["counters"]["subproblems"] > 0 and cpp["counters"]["relaxed"] > 1000
