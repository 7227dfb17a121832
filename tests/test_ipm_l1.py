"""Turnover + leverage together (porqua_amd/ipm_l1.py): the per-asset block elimination's
closed forms, and the IPM's algebra on the CPU with the device coupling factorisation
swapped for a dense torch solve (test scaffolding only: the product path has no CPU
factorisation), against the oracle IPM on the reference's linearised problem
(src/qp_problems.py:40-118)."""
import numpy as np
import pytest
import torch

from oracle.qp_ipm import solve_qp
from porqua_amd import ipm_l1
from porqua_amd.qp_problems import QuadraticProgram
from tests.conftest import load_golden


def test_block_closed_forms_match_projected_inverse():
    rng = np.random.default_rng(0)
    N = np.array([[1, 1, 0, 1, 0], [0, 1, 1, 0, 0], [0, 0, 0, 1, 1]], dtype=float).T
    E = np.array([[1, -1, 1, 0, 0], [1, 0, 0, -1, 1]], dtype=float)
    C = np.array([[1, 0, 0, 0, 0], [0, 1, 1, 0, 0], [0, 0, 0, 1, 1]], dtype=float)
    for _ in range(50):
        d = np.exp(rng.uniform(-8, 8, 5))
        H = np.diag(d)
        Hi = np.diag(1 / d)
        Pi = Hi - Hi @ E.T @ np.linalg.solve(E @ Hi @ E.T, E @ Hi)          # projected inverse
        Kref = C @ Pi @ C.T
        t = [torch.tensor([v], dtype=torch.float64) for v in d]
        det, cof, K = ipm_l1.block_k(*t)
        got = np.array([[K["xx"], K["xt"], K["xL"]], [K["xt"], K["tt"], K["tL"]], [K["xL"], K["tL"], K["LL"]]],
                       dtype=float).reshape(3, 3)
        assert np.allclose(got, Kref, rtol=1e-9, atol=1e-12 * np.abs(Kref).max())
        a = rng.standard_normal(3)
        w = np.array([float(v) for v in ipm_l1.block_solve(det, cof, *[torch.tensor([v]) for v in a])])
        assert np.allclose(w, np.linalg.solve(N.T @ H @ N, a), rtol=1e-9, atol=1e-12)


def _torch_gemv(U, x, trans=False):
    """Test scaffolding: the CPU stand-in of pq_gemv_batched (U[b] x[b] / U[b]' x[b])."""
    return torch.bmm(U.transpose(1, 2) if trans else U, x.unsqueeze(2)).squeeze(2)


class _DenseCoupling(ipm_l1._Coupling):
    """Test scaffolding: S formed densely by torch on the CPU, solved by torch.linalg."""

    def __init__(self, U, budget):
        self.U = U
        self.B, self.k0, self.n = U.shape
        self.budget = budget
        self.nb = 2 if budget else 1
        self.k = self.k0 + self.nb

    def factor(self, det, cof, K, dU, th_st, th_sL):
        self.det, self.cof, self.dU, self.th_st, self.th_sL = det, cof, dU, th_st, th_sL
        eye = torch.eye(self.k, dtype=torch.float64).expand(self.B, self.k, self.k)
        self.S = torch.stack([self.apply(eye[:, :, j]) for j in range(self.k)], 2)
        return torch.zeros(self.B, dtype=torch.bool)

    def solve(self, g, refine=2):
        return torch.linalg.solve(self.S, g)


def _reference_qp(P, q, x0, tau, L, lb, ub, tc=None):
    n = P.shape[0]
    qp = QuadraticProgram(P=P, q=q, A=np.ones((1, n)), b=np.ones(1), G=None, h=None, lb=lb, ub=ub,
                          params={"solver_name": "cvxopt"})
    if tc is not None:
        qp.linearize_turnover_objective(x0, tc)
    if tau is not None:
        qp.linearize_turnover_constraint(x0, tau)
    qp.linearize_leverage_constraint(N=n, leverage_budget=L)
    return qp


@pytest.mark.parametrize("form", ["budget", "cost"])
def test_l1_ipm_algebra_matches_oracle(monkeypatch, form):
    monkeypatch.setattr(ipm_l1, "_Coupling", _DenseCoupling)
    monkeypatch.setattr(ipm_l1, "_gemv", _torch_gemv)
    g = load_golden("msci_mv_shrink")
    n = g["P"].shape[-1]
    rng = np.random.default_rng(3)
    B = 3
    P, q = g["P"][:B], g["q"][:B]
    x0 = rng.dirichlet(np.ones(n))
    lb, ub = np.full(n, -0.1), np.full(n, 0.3)
    ev, V = np.linalg.eigh(P)
    UW = torch.from_numpy(np.ascontiguousarray(np.transpose(V * np.sqrt(np.clip(ev, 0, None))[:, None, :], (0, 2, 1))))
    terms = ipm_l1.L1Terms(x0=x0, cost=0.0 if form == "budget" else 0.002,
                           to_budget=0.4 if form == "budget" else None, lev_budget=1.3)
    res = ipm_l1.l1_ipm_batched(UW, None, torch.from_numpy(q), terms, A=np.ones((1, n)), b=np.ones(1),
                                lb=lb, ub=ub)
    for i in range(B):
        qp = _reference_qp(P[i], q[i], x0, 0.4 if form == "budget" else None, 1.3, lb, ub,
                           tc=0.002 if form == "cost" else None)
        o = solve_qp(qp["P"], qp["q"], G=qp["G"], h=qp["h"], A=qp["A"], b=qp["b"], lb=qp["lb"], ub=qp["ub"])
        x = res.x[i].numpy()
        assert int(res.status[i]) == 1, (i, float(res.merit[i]), int(res.iters[i]))
        assert np.abs(x - o.x[:n]).max() < 1e-6, np.abs(x - o.x[:n]).max()
        assert abs(float(res.obj[i]) - o.obj) <= 1e-7 * max(abs(o.obj), 1e-3)
        assert abs(x.sum() - 1) < 1e-9 and np.abs(x).sum() <= 1.3 + 1e-8
        if form == "budget":
            assert np.abs(x - x0).sum() <= 0.4 + 1e-8


def test_l1_ipm_window_form_matches_oracle(monkeypatch):
    """Window form (T' = T < n, pd > 0): P = 2 X'X / T + 2 l2 I from the raw window rows, the
    cost form with a leverage budget, long-short box, against the oracle on the reference's
    linearised problem."""
    monkeypatch.setattr(ipm_l1, "_Coupling", _DenseCoupling)
    monkeypatch.setattr(ipm_l1, "_gemv", _torch_gemv)
    from porqua_amd.synthetic import factor_panel
    n, Tw, B = 120, 60, 2
    _, R, y, _ = factor_panel(200, n, seed=5)
    rng = np.random.default_rng(1)
    x0 = rng.dirichlet(np.ones(n))
    lb, ub = np.full(n, -0.05), np.full(n, 0.2)
    ends = [100, 131]
    X = np.stack([R[e - Tw:e] for e in ends])
    Y = np.stack([y[e - Tw:e] for e in ends])
    l2 = 1e-3
    UW = torch.from_numpy(np.sqrt(2.0) * X)                       # P = 2 X'X + 2 l2 I
    pd = torch.full((B,), 2 * l2, dtype=torch.float64)
    q = torch.from_numpy(-2.0 * np.einsum("bti,bt->bi", X, Y))
    terms = ipm_l1.L1Terms(x0=x0, cost=1e-3, to_budget=None, lev_budget=1.4)
    res = ipm_l1.l1_ipm_batched(UW, pd, q, terms, A=np.ones((1, n)), b=np.ones(1), lb=lb, ub=ub)
    for i in range(B):
        P = 2 * X[i].T @ X[i] + 2 * l2 * np.eye(n)
        qp = _reference_qp(P, q[i].numpy(), x0, None, 1.4, lb, ub, tc=1e-3)
        o = solve_qp(qp["P"], qp["q"], G=qp["G"], h=qp["h"], A=qp["A"], b=qp["b"], lb=qp["lb"], ub=qp["ub"])
        x = res.x[i].numpy()
        assert int(res.status[i]) == 1, (i, float(res.merit[i]), int(res.iters[i]))
        assert np.abs(x - o.x[:n]).max() < 1e-6, np.abs(x - o.x[:n]).max()
        assert abs(float(res.obj[i]) - o.obj) <= 1e-7 * max(abs(o.obj), 1e-3), (float(res.obj[i]), o.obj)
        assert abs(x.sum() - 1) < 1e-9 and np.abs(x).sum() <= 1.4 + 1e-8
