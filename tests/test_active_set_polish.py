"""CPU check of the host logic of porqua_amd.ipm.active_set_polish (the exact solve on the
active set after the device IPM of the per-QP drop-in beyond 1024 assets): the K2 / K2L
factor is replaced by a dense torch inverse, the interior-point answer by the oracle's
unrefined IPM iterate; the polish must land on the oracle's refined optimum."""
import numpy as np
import torch

from oracle.qp_ipm import solve_qp
from porqua_amd import ipm
from porqua_amd.synthetic import dense_qp


class _DenseFactor:
    def __init__(self, B, m, dev):
        self.m = m

    def factor(self, H, shift, retries=3):
        try:
            torch.linalg.cholesky(H)
        except RuntimeError:
            return torch.ones(H.shape[0], dtype=torch.bool)
        self.Hinv = torch.linalg.inv(H)
        return torch.zeros(H.shape[0], dtype=torch.bool)

    def solve_mat(self, R):
        return self.Hinv @ R


def test_polish_reaches_the_oracle_optimum(monkeypatch):
    monkeypatch.setattr(ipm, "_NormalFactor", _DenseFactor)
    pr = dense_qp(240, T=120, seed=11)
    cons = {k: pr[k] for k in ("G", "h", "A", "b", "lb", "ub")}
    rough = solve_qp(pr["P"], pr["q"], tol=1e-7, refine=False, **cons)
    exact = solve_qp(pr["P"], pr["q"], **cons)
    assert np.abs(rough.x - exact.x).max() > 1e-9            # the IPM iterate alone is not exact
    T = lambda v: torch.from_numpy(np.asarray(v, dtype=np.float64))
    x, y, z, zb, ok = ipm.active_set_polish(T(pr["P"]), T(pr["q"]), T(pr["A"]), T(pr["b"]), T(pr["G"]), T(pr["h"]),
                                            T(pr["lb"]), T(pr["ub"]), T(rough.x), T(rough.y), T(rough.z),
                                            T(rough.z_box))
    assert ok
    assert np.abs(x.numpy() - exact.x).max() <= 1e-10
    g = pr["P"] @ x.numpy() + pr["q"] + pr["A"].T @ y.numpy() + pr["G"].T @ z.numpy() + zb.numpy()
    assert np.abs(g).max() <= 1e-12 * max(1.0, np.abs(pr["q"]).max()) + 1e-15


def test_dependent_active_rows_give_bounded_multipliers(monkeypatch):
    """Linearly dependent active rows (the budget row twice): x is the single-row optimum and
    the multipliers are the minimum-norm split of the single row's (each half), not scaled by
    the reciprocal of a regularising shift."""
    monkeypatch.setattr(ipm, "_NormalFactor", _DenseFactor)
    pr = dense_qp(120, T=80, seed=5)
    cons = {k: pr[k] for k in ("G", "h", "A", "b", "lb", "ub")}
    rough = solve_qp(pr["P"], pr["q"], tol=1e-7, refine=False, **cons)
    exact = solve_qp(pr["P"], pr["q"], **cons)
    T = lambda v: torch.from_numpy(np.asarray(v, dtype=np.float64))
    A2 = np.vstack([pr["A"], pr["A"]])
    b2 = np.concatenate([np.atleast_1d(pr["b"]), np.atleast_1d(pr["b"])])
    y2 = np.concatenate([rough.y, rough.y]) / 2.0
    x, y, z, zb, ok = ipm.active_set_polish(T(pr["P"]), T(pr["q"]), T(A2), T(b2), T(pr["G"]), T(pr["h"]),
                                            T(pr["lb"]), T(pr["ub"]), T(rough.x), T(y2), T(rough.z),
                                            T(rough.z_box))
    assert ok
    assert np.abs(x.numpy() - exact.x).max() <= 1e-10
    me = np.atleast_1d(pr["b"]).size
    ya, yb = y.numpy()[:me], y.numpy()[me:]
    assert np.abs(ya - yb).max() <= 1e-9 * max(1.0, np.abs(exact.y).max())
    assert np.abs((ya + yb) - exact.y).max() <= 1e-8 * max(1.0, np.abs(exact.y).max())
    g = pr["P"] @ x.numpy() + pr["q"] + A2.T @ y.numpy() + pr["G"].T @ z.numpy() + zb.numpy()
    assert np.abs(g).max() <= 1e-11 * max(1.0, np.abs(pr["q"]).max()) + 1e-15
