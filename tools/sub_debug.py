"""Subproblem diagnostics (study tool): status / objective / dual of the device subproblem on
the GPU test's matchings against HiGHS; an error scenario's dual field is -(error site)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import subproblem_oracle as so  # noqa: E402
from tests.test_subproblem import _full_matching, _net, _path_of  # noqa: E402


def main(cfg, seed, S, zl, trials):
    from sgufp_solver_amd import engine as E
    inst, path, net = _net(cfg, seed, S, zl)
    eng = E.Engine(path, 0, 64)
    rng = np.random.default_rng(100 + seed)
    ys = [_full_matching(net, rng, 1.0 if t % 2 == 0 else 0.85) for t in range(trials)]
    paths = [_path_of(inst, net, y) for y in ys]
    eng.subproblem(paths)
    st, obj, dual = eng.subproblem_detail(len(paths))
    for k, y in enumerate(ys):
        for s in range(net.S):
            w = so.dual_lp(net, y, s)[:2]
            print(f"path {k} scen {s}: status {st[k, s]} obj {obj[k, s]} dual {dual[k, s]} | highs {w}")
    eng.close()


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), sys.argv[4] == "1", int(sys.argv[5]))
