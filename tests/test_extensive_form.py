"""The extensive-form oracle (oracle/extensive_form.py: StochasticModel.h:16-203 restated,
HiGHS milp) against brute force: the maximum over every V-bar matching of the mean
scenario flow value (oracle/subproblem_oracle.primal_lp, an independent LP model)."""
import itertools

import numpy as np
import pytest

from oracle import extensive_form as ef
from oracle import subproblem_oracle as so
from sgufp_solver_amd import instance


def _node_matchings(ins, outs):
    """All partial matchings between in-arc tails and out-arc heads of one V-bar node."""
    res = [()]
    for k in range(1, min(len(ins), len(outs)) + 1):
        for a in itertools.combinations(ins, k):
            for b in itertools.permutations(outs, k):
                res.append(tuple(zip(a, b)))
    return res


@pytest.mark.parametrize("seed,S", [(1, 1), (2, 2), (3, 2)])
def test_extensive_form_equals_brute_force(seed, S):
    inst = instance.generate(instance.CONFIGS["T0"], seed, scenarios=S)
    net = so.from_instance(inst, [])
    T, H = inst.tails, inst.heads
    per_node = []
    for q in inst.vbar:
        ins = sorted({int(T[a]) for a in range(inst.m) if int(H[a]) == q})
        outs = sorted({int(H[a]) for a in range(inst.m) if int(T[a]) == q})
        per_node.append([tuple((i, q, j) for i, j in mt) for mt in _node_matchings(ins, outs)])
    best = -np.inf
    for combo in itertools.product(*per_node):
        y = {t: 1 for part in combo for t in part}
        vals = [so.primal_lp(net, y, s) for s in range(S)]
        if all(v[0] == "optimal" for v in vals):
            best = max(best, sum(v[1] for v in vals) / S)
    got = ef.solve(inst)
    assert abs(got - best) <= 1e-6 * max(1.0, abs(best)), (got, best)
