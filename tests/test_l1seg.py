"""Turnover + leverage as a segment split (porqua_amd/l1seg.py) against the reference's
linearised problem (src/qp_problems.py:40-157: auxiliary d / x+ x- variables and rows),
both solved by the oracle IPM on the CPU: the same optimal x and objective, for the budget
and the cost form of the turnover term, long-short boxes, x0 of both signs."""
import numpy as np
import pytest

from oracle.qp_ipm import solve_qp
from porqua_amd import l1seg
from porqua_amd.qp_problems import QuadraticProgram


def _problem(n, seed, box=(-0.15, 0.4)):
    rng = np.random.default_rng(seed)
    X = rng.normal(3e-4, 0.02, size=(3 * n, n))
    Xc = X - X.mean(0)
    P = 2 * Xc.T @ Xc / (3 * n - 1)
    q = -rng.normal(5e-4, 1e-3, n)
    x0 = rng.dirichlet(np.ones(n)) * 1.4 - 0.4 / n                  # some short positions
    x0 = np.clip(x0, box[0], box[1])
    return P, q, x0, np.full(n, box[0]), np.full(n, box[1])


@pytest.mark.parametrize("seed,tau,lev,cost", [(0, 0.3, 1.2, None), (1, 0.6, 1.05, None), (2, 10.0, 1.3, None),
                                               (3, None, 1.2, 2e-3), (4, 0.4, np.inf, None)])
def test_segment_split_matches_linearised_problem(seed, tau, lev, cost):
    n = 12
    P, q, x0, lb, ub = _problem(n, seed)
    A, b = np.ones((1, n)), np.ones(1)
    qp = QuadraticProgram(P=P, q=q, A=A, b=b, G=None, h=None, lb=lb, ub=ub, params={"solver_name": "cvxopt"})
    if cost is not None:
        qp.linearize_turnover_objective(x0, cost)
    else:
        qp.linearize_turnover_constraint(x0, tau)
    if np.isfinite(lev):
        qp.linearize_leverage_constraint(N=n, leverage_budget=lev)
    ref = solve_qp(qp["P"], qp["q"], G=qp["G"], h=qp["h"], A=qp["A"], b=qp["b"], lb=qp["lb"], ub=qp["ub"])
    sd = l1seg.segment_data(x0, lb, ub, cost=cost or 0.0, to_budget=None if cost is not None else tau,
                            lev_budget=lev)
    assert sd is not None
    sp = l1seg.segment_problem({"P": P, "q": q, "A": A, "b": b, "G": None, "h": None}, sd)
    sol = solve_qp(sp["P"], sp["q"], G=sp["G"], h=sp["h"], A=sp["A"], b=sp["b"], lb=sp["lb"], ub=sp["ub"])
    x = l1seg.merge(sol.x, n, sd["lb"])
    f = lambda v: 0.5 * v @ P @ v + q @ v + (cost or 0.0) * np.abs(v - x0).sum()   # noqa: E731
    fr, fs = f(ref.x[:n]), f(x)
    assert abs(fs - fr) <= 1e-7 * max(1.0, abs(fr)), (fs, fr)
    assert abs(sol.obj + sp["constant"] - fs) <= 1e-9 * max(1.0, abs(fs))      # the split's own value
    assert np.abs(x - ref.x[:n]).max() <= 1e-5, np.abs(x - ref.x[:n]).max()   # P > 0: unique optimum
    assert abs(x.sum() - 1) <= 1e-8 and x.min() >= lb[0] - 1e-9 and x.max() <= ub[0] + 1e-9
    if tau is not None and cost is None:
        assert np.abs(x - x0).sum() <= tau + 1e-7
    if np.isfinite(lev):
        assert np.abs(x).sum() <= lev + 1e-7


def test_segment_data_rejects_a_box_without_zero_or_x0():
    x0 = np.array([0.5, 0.5])
    assert l1seg.segment_data(x0, np.array([0.1, 0.0]), np.ones(2)) is None    # lb > 0: no breakpoint 0 inside
    assert l1seg.segment_data(x0, np.zeros(2), np.array([0.4, 1.0])) is None   # x0 above ub
    sd = l1seg.segment_data(x0, np.zeros(2), np.ones(2))                       # long-only: s1 has zero length
    assert np.array_equal(sd["hi"], [0, 0, 0.5, 0.5, 0.5, 0.5])


def test_in_order_filling_reproduces_both_l1_functions():
    rng = np.random.default_rng(5)
    n = 50
    x0 = rng.uniform(-0.2, 0.3, n)
    lb, ub = np.full(n, -0.3), np.full(n, 0.4)
    sd = l1seg.segment_data(x0, lb, ub)
    x = rng.uniform(-0.3, 0.4, n)
    # in-order filling of x
    hi = sd["hi"].reshape(3, n)
    s = np.zeros((3, n))
    rest = x - lb
    for k in range(3):
        s[k] = np.clip(rest, 0, hi[k])
        rest -= s[k]
    s = s.reshape(-1)
    assert np.allclose(l1seg.merge(s, n, lb), x)
    assert np.isclose(sd["t0"] + sd["t"] @ s, np.abs(x - x0).sum())
    assert np.isclose(sd["l0"] + sd["l"] @ s, np.abs(x).sum())
