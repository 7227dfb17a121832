"""QPs with more than 64 general rows on the device (porqua_amd/ipm.py): the reference's
linearised turnover budget and leverage constraint together (src/qp_problems.py:40-118,
2n + 1 inequality rows and n + 1 equality rows) through QuadraticProgram.solve with
solver_name='mi355x', against the oracle IPM on the same linearised problem."""
import numpy as np
import pytest

from oracle.qp_ipm import solve_qp
from porqua_amd.qp_problems import QuadraticProgram, solve_batch
from tests.conftest import load_golden

pytestmark = pytest.mark.gpu


def _problems(k, seed=0):
    g = load_golden("msci_mv_shrink")
    n = g["P"].shape[-1]
    rng = np.random.default_rng(seed)
    qps = []
    for i in range(k):
        qp = QuadraticProgram(P=g["P"][i], q=g["q"][i], A=np.ones((1, n)), b=np.ones(1), G=None, h=None,
                              lb=np.full(n, -0.1), ub=np.full(n, 0.3), params={"solver_name": "mi355x"})
        qp.linearize_turnover_constraint(rng.dirichlet(np.ones(n)), 0.4)
        qp.linearize_leverage_constraint(N=n, leverage_budget=1.3)
        qps.append(qp)
    return qps, n


def _check(sol, qp, n):
    o = solve_qp(qp["P"], qp["q"], G=qp["G"], h=qp["h"], A=qp["A"], b=qp["b"], lb=qp["lb"], ub=qp["ub"])
    assert sol.found
    x = sol.x
    assert abs(sol.obj - o.obj) <= 1e-6 * max(abs(o.obj), 1e-3), (sol.obj, o.obj)
    assert np.abs(qp["A"] @ x - qp["b"]).max() < 1e-8
    assert (qp["G"] @ x - qp["h"]).max() < 1e-8
    assert x[:n].min() > -0.1 - 1e-8 and x[:n].max() < 0.3 + 1e-8
    assert np.abs(x[:n]).sum() <= 1.3 + 1e-7


def test_turnover_and_leverage_single(device):
    qps, n = _problems(3)
    for qp in qps:
        assert qp._l1 == "unsupported"
        qp.solve()
        _check(qp["solution"], qp, n)


def test_turnover_and_leverage_batch(device):
    qps, n = _problems(6, seed=1)
    sols = solve_batch(qps)
    for s, qp in zip(sols, qps):
        _check(s, qp, n)
