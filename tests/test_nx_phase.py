"""Cut-parallel optimality phase of NON-exact DDs (k_nx_dag / k_exact_leaf<true> / k_nx_fin,
kNxPending in dd_device.hpp): with SGUFP_NX_MIN=1 and SGUFP_NX_SKIP=0 every non-exact record
that reaches its optimality cuts takes it -- whatever the pool size -- and must give the reference's results bit
for bit (fixtures of tests/golden, the bench workload against the in-order path), including
the records whose width-1 pruning might fire, which k_nx_fin hands back to k_relax
(kNxFallback).  The B&B pools of tests/test_bnb_parity.py (10^4+ O cuts) take the phase under
the default threshold."""
import os
import re

import numpy as np
import pytest

from sgufp_solver_amd import engine as E
from sgufp_solver_amd import frontier, instance, pools
from tests import golden_io

pytestmark = pytest.mark.gpu

STATS = re.compile(r"non-exact: dag items (\d+), fallbacks (\d+)")


def _stats(text):
    items = fb = 0
    for m in STATS.finditer(text):
        items += int(m.group(1))
        fb += int(m.group(2))
    return items, fb


@pytest.mark.parametrize("skip", ["0", "8"])
@pytest.mark.parametrize("name", sorted({c["name"] for c in golden_io.manifest()}))
def test_nx_phase_on_fixtures(monkeypatch, capfd, name, skip):
    """skip: optimality cuts k_relax applies in order before the hand-off (SGUFP_NX_SKIP; the
    phase then starts from the in-order terminal weights)."""
    monkeypatch.setenv("SGUFP_NX", "1")
    monkeypatch.setenv("SGUFP_NX_MIN", "1")
    monkeypatch.setenv("SGUFP_NX_SKIP", skip)
    monkeypatch.setenv("SGUFP_EXACT_STATS", "1")
    d = golden_io.case_dir(name)
    e = E.Engine(f"{d}/net.txt", 0, 256)
    e.add_cuts(pools.read_pool(golden_io.golden_file(d, "cuts.txt")))
    nodes = pools.read_nodes(os.path.join(d, "nodes.txt"))
    case = [c for c in golden_io.manifest() if c["name"] == name][0]
    try:
        for run in case["runs"]:
            got = e.relax(nodes, float.fromhex(run["incumbent"]))
            want = golden_io.parse_results_text(golden_io.read_golden(name, run["file"]))
            bad = golden_io.compare_results(got, want)
            assert not bad, f"{run['file']}: " + "\n".join(bad[:10])
    finally:
        e.close()


def test_nx_phase_engages_and_matches_in_order(monkeypatch, capfd, tmp_path):
    """The 1k-arc bench workload (C4, 1 024-record BFS frontier, 16 + 64 synthetic cuts) at
    DOUBLE_MIN and at the bench's incumbent rule: forced cut-parallel phase vs the in-order
    path (SGUFP_NX=0), every field equal; the phase took records (DAG work items > 0) and
    settled most of them itself."""
    inst = instance.generate(instance.CONFIGS["C4"], 1, scenarios=4)
    net = str(tmp_path / "net.txt")
    inst.write(net)
    pool = pools.synthetic_pool(inst, 16, 64, 1)
    monkeypatch.setenv("SGUFP_NX", "0")
    e0 = E.Engine(net, 0, 1024)
    recs = E.batch_to_records(frontier.bfs_frontier(e0, 1024))
    e0.add_cuts(pool)
    monkeypatch.setenv("SGUFP_NX", "1")
    monkeypatch.setenv("SGUFP_NX_MIN", "1")
    monkeypatch.setenv("SGUFP_NX_SKIP", "0")
    monkeypatch.setenv("SGUFP_EXACT_STATS", "1")
    e1 = E.Engine(net, 0, 1024)
    e1.add_cuts(pool)
    try:
        base = e0.relax(recs, pools.DOUBLE_MIN)
        fin = [g.ub for g in base if g.status in (0, 3)]
        incs = [pools.DOUBLE_MIN, float(np.percentile(fin, 40)), float(np.percentile(fin, 80))]
        capfd.readouterr()
        for inc in incs:
            want = base if inc == pools.DOUBLE_MIN else e0.relax(recs, inc)
            got = e1.relax(recs, inc)
            bad = golden_io.compare_results(got, want)
            assert not bad, f"incumbent {inc!r}: " + "\n".join(bad[:10])
        items, fb = _stats(capfd.readouterr().err)
        assert items > 0, "no record took the cut-parallel phase"
    finally:
        e0.close()
        e1.close()
