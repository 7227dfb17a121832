"""Deterministic synthetic return panels for the benchmark configurations.

Factor model  r_t = beta * f_t + B_s g_t + eps_t  with beta ~ N(1, 0.3^2),
f ~ N(3e-4, 0.01^2), 10 sector factors g ~ N(0, 0.005^2), eps ~ N(0, 0.02^2), a uniform
sector id per asset; benchmark y_t = R_t w_cap + N(0, 1e-4^2) with w_cap ~ Dirichlet(1);
business-day calendar starting 2005-01-03.  Seeds are fixed per configuration
(20240314 for configs 3-5).

Configs 1/2 (SPTR index replication on ``usa_returns``, absent from the reference tree) use
``usa_panel``: 494 synthetic assets on the last 4795 dates of the real SPTR calendar, each
loading on the real SPTR return, so least-squares tracking of SPTR is meaningful.
"""
from __future__ import annotations

import numpy as np

SEED = 20240314


def business_days(start: str, count: int) -> np.ndarray:
    """``count`` consecutive Mon-Fri dates (datetime64[D]) starting at ``start``."""
    d0 = np.datetime64(start, "D")
    days = d0 + np.arange(int(count * 7 / 5) + 14)
    wd = (days.astype("int64") + 3) % 7
    return days[wd < 5][:count]


def factor_panel(n_dates: int, n_assets: int, seed: int = SEED, n_sectors: int = 10):
    """Returns (dates, R [n_dates x n_assets] float64 C-order, y [n_dates], sector ids)."""
    rng = np.random.default_rng(seed)
    beta = rng.normal(1.0, 0.3, size=n_assets)
    sector = rng.integers(0, n_sectors, size=n_assets)
    f = rng.normal(3e-4, 0.01, size=n_dates)
    g = rng.normal(0.0, 0.005, size=(n_dates, n_sectors))
    R = np.empty((n_dates, n_assets), dtype=np.float64)
    chunk = 2048
    for s in range(0, n_dates, chunk):
        e = min(n_dates, s + chunk)
        eps = rng.normal(0.0, 0.02, size=(e - s, n_assets))
        R[s:e] = f[s:e, None] * beta[None, :] + g[s:e][:, sector] + eps
    w_cap = rng.dirichlet(np.ones(n_assets))
    y = R @ w_cap + rng.normal(0.0, 1e-4, size=n_dates)
    return business_days("2005-01-03", n_dates), R, y, sector


USA_SEED = 20240101


def usa_panel(sptr_days: np.ndarray, sptr: np.ndarray, n_assets: int = 494, n_rows: int = 4795,
              seed: int = USA_SEED, n_sectors: int = 11):
    """usa-shaped panel for configs 1/2 on the SPTR calendar: the last ``n_rows`` SPTR dates,
    r_t = beta * sptr_t + B_s g_t + eps_t with beta ~ N(1, 0.25^2), 11 sector factors
    g ~ N(0, 0.004^2), eps ~ N(0, 0.015^2).  Returns (dates datetime64[D], R [n_rows x
    n_assets], y = the real SPTR returns on those dates)."""
    days = np.asarray(sptr_days)[-n_rows:]
    y = np.asarray(sptr, dtype=np.float64)[-n_rows:]
    rng = np.random.default_rng(seed)
    beta = rng.normal(1.0, 0.25, size=n_assets)
    sector = rng.integers(0, n_sectors, size=n_assets)
    g = rng.normal(0.0, 0.004, size=(n_rows, n_sectors))
    eps = rng.normal(0.0, 0.015, size=(n_rows, n_assets))
    R = np.ascontiguousarray(y[:, None] * beta[None, :] + g[:, sector] + eps)
    return days.astype("datetime64[D]"), R, y


def dense_qp(n: int = 2000, T: int = 300, seed: int = 20240315, n_groups: int = 3):
    """A well-posed dense QP of the kind QuadraticProgram.solve receives (src/qp_problems.py:
    184-216), for the per-QP drop-in beyond 1024 assets: P = 2 (Sigma + 0.05 mean(diag Sigma)
    I) (linear_shrinkage, src/covariance.py:71-84, so P is PD and the optimum unique),
    q = -mu, budget 1'x = 1, box [0, 0.05], and ``n_groups`` group caps G x <= 0.36 (3 groups: feasible, binding).
    Returns dict(P, q, A, b, G, h, lb, ub)."""
    rng = np.random.default_rng(seed)
    X = rng.normal(3e-4, 0.02, size=(T, n)) + rng.normal(0.0, 0.01, size=(T, 1))
    Xc = X - X.mean(0)
    S = Xc.T @ Xc / (T - 1)
    S += 0.05 * np.mean(np.diag(S)) * np.eye(n)
    grp = rng.integers(0, n_groups, size=n)
    G = np.stack([(grp == g).astype(float) for g in range(n_groups)])
    return {"P": 2.0 * S, "q": -X.mean(0), "A": np.ones((1, n)), "b": np.ones(1), "G": G,
            "h": np.full(n_groups, 0.36), "lb": np.zeros(n), "ub": np.full(n, 0.05)}
