"""Diagnostics of the cut-parallel optimality phase of non-exact DDs (k_nx_*): the C4 bench
workload (1 024-record BFS frontier, 16 + 64 synthetic cuts) relaxed with the phase forced
(SGUFP_NX_MIN=1) and without it; prints the [exact] counter lines (SGUFP_EXACT_STATS) -- DAG
work items, fallbacks, DDs kept back by reason -- and whether every record agrees."""
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from sgufp_solver_amd import engine as E
    from sgufp_solver_amd import frontier, instance, pools
    from tests import golden_io
    cfg = sys.argv[1] if len(sys.argv) > 1 else "C4"
    inst = instance.generate(instance.CONFIGS[cfg], 1, scenarios=4)
    d = tempfile.mkdtemp(prefix="sgufp_nx_")
    net = os.path.join(d, "net.txt")
    inst.write(net)
    pool = pools.synthetic_pool(inst, 16, 64, 1)
    os.environ["SGUFP_NX"] = "0"
    e0 = E.Engine(net, 0, 1024)
    recs = E.batch_to_records(frontier.bfs_frontier(e0, 1024))
    e0.add_cuts(pool)
    os.environ["SGUFP_NX"] = "1"
    os.environ["SGUFP_NX_MIN"] = "1"
    os.environ["SGUFP_NX_SKIP"] = sys.argv[2] if len(sys.argv) > 2 else "0"
    os.environ["SGUFP_EXACT_STATS"] = "1"
    e1 = E.Engine(net, 0, 1024)
    e1.add_cuts(pool)
    base = e0.relax(recs, pools.DOUBLE_MIN)
    fin = [g.ub for g in base if g.status in (0, 3)]
    for inc in [pools.DOUBLE_MIN, float(np.percentile(fin, 40)), float(np.percentile(fin, 80))]:
        t0 = time.perf_counter()
        want = base if inc == pools.DOUBLE_MIN else e0.relax(recs, inc)
        t1 = time.perf_counter()
        got = e1.relax(recs, inc)
        t2 = time.perf_counter()
        bad = golden_io.compare_results(got, want)
        st = {}
        for g in got:
            st[g.status] = st.get(g.status, 0) + 1
        print(f"incumbent {inc!r}: mismatches {len(bad)} statuses {st} in-order {1e3 * (t1 - t0):.1f} ms "
              f"nx {1e3 * (t2 - t1):.1f} ms", flush=True)
        for b in bad[:5]:
            print("  ", b)
    e0.close()
    e1.close()


if __name__ == "__main__":
    main()
