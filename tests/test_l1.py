"""l1 row: transaction cost / turnover budget around x0.

Golden problems were captured from the reference's own Backtest.run + model_qpsolvers
(tools/capture_l1.py -> tests/golden/msci_l1_{tc,to}.npz: the 2n-variable linearised
problems of src/qp_problems.py:40-77, 120-157, with KKT-certified oracle optima).

* CPU: the package's linearisation reproduces the captured matrices; the signed split
  (porqua_amd/l1split.py) solved by the oracle IPM gives the golden weights / objective.
* GPU: QuadraticProgram(solver 'mi355x') with the linearisation solves the split on the
  device.  Bars: weights 1e-5 (L-inf), objective 1e-6 relative, violation 1e-7.
"""
import os

import numpy as np
import pytest

from oracle.qp_ipm import solve_qp
from porqua_amd.l1split import L1Split, merge_solution, split_problem
from porqua_amd.qp_problems import QuadraticProgram

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
KINDS = {"tc": "cost", "to": "budget"}


def _case(tag, i):
    g = np.load(os.path.join(GOLD, f"msci_l1_{tag}.npz"))
    n = g["P"].shape[-1] // 2
    base = dict(P=g["P"][i][:n, :n], q=g["q"][i][:n], A=g["A"][i][:, :n], b=np.atleast_1d(g["b"][i]),
                lb=g["lb"][i][:n], ub=g["ub"][i][:n], G=None, h=None)
    value = 0.002 if tag == "tc" else float(g["h"][i][-1])
    return g, n, base, L1Split(KINDS[tag], g["x0"], value)


def _qp(base, term, solver):
    qp = QuadraticProgram(P=base["P"].copy(), q=base["q"].copy(), A=base["A"].copy(), b=base["b"].copy(),
                          lb=base["lb"].copy(), ub=base["ub"].copy(), G=None, h=None,
                          params={"solver_name": solver})
    if term.kind == "cost":
        qp.linearize_turnover_objective(term.x0, transaction_cost=term.value)
    else:
        qp.linearize_turnover_constraint(term.x0, to_budget=term.value)
    return qp


@pytest.mark.parametrize("tag", ["tc", "to"])
def test_linearisation_matches_reference(tag):
    for i in (0, 7, 23):
        g, n, base, term = _case(tag, i)
        qp = _qp(base, term, "mi355x")
        # the captured P went through the reference's PD repair (src/qp_problems.py:189-191),
        # which adds ~1e-19 to the zero auxiliary block
        assert np.allclose(qp["P"], g["P"][i], rtol=0, atol=1e-15 * np.abs(g["P"][i]).max())
        for k in ("q", "G", "h", "lb", "ub"):
            assert np.array_equal(np.asarray(qp[k], dtype=float), g[k][i]), k
        assert np.array_equal(qp["A"].reshape(g["A"][i].shape), g["A"][i])


@pytest.mark.parametrize("tag", ["tc", "to"])
def test_split_solved_by_oracle_matches_golden(tag):
    for i in range(0, 24, 3):
        g, n, base, term = _case(tag, i)
        sp = split_problem(base, term)
        s = solve_qp(sp["P"], sp["q"], sp["G"], sp["h"], sp["A"], sp["b"], sp["lb"], sp["ub"])
        x, d = merge_solution(s.x, term)
        assert np.abs(x - g["x"][i][:n]).max() < 1e-6
        obj_ref = 0.5 * g["x"][i] @ g["P"][i] @ g["x"][i] + g["q"][i] @ g["x"][i]
        obj = 0.5 * x @ base["P"] @ x + base["q"] @ x + (term.value * d.sum() if term.kind == "cost" else 0.0)
        assert abs(obj - obj_ref) <= 1e-8 * max(1.0, abs(obj_ref))


def test_split_rejects_x0_outside_box():
    g, n, base, term = _case("tc", 0)
    bad = L1Split("cost", np.full(n, 2.0), 0.002)
    with pytest.raises(NotImplementedError):
        split_problem(base, bad)


@pytest.mark.gpu
@pytest.mark.parametrize("tag", ["tc", "to"])
def test_device_l1_matches_golden(tag):
    for i in range(24):
        g, n, base, term = _case(tag, i)
        qp = _qp(base, term, "mi355x")
        qp.solve()
        s = qp["solution"]
        assert s.found and s.extras.get("l1_split") == term.kind
        x = s.x[:n]
        assert np.abs(x - g["x"][i][:n]).max() < 1e-5, (i, np.abs(x - g["x"][i][:n]).max())
        obj_ref = float(g["obj"][i])
        assert abs(s.obj - obj_ref) <= 1e-6 * max(1.0, abs(obj_ref))
        viol = max(abs(x.sum() - 1.0), float(np.maximum(-x, 0).max()),
                   (np.abs(x - term.x0).sum() - term.value) if term.kind == "budget" else 0.0)
        assert viol <= 1e-7
