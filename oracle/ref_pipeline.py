"""numpy restatement of PorQua's per-date arithmetic (TEST INFRASTRUCTURE ONLY).

Each function names the reference lines it follows.  Nothing here is imported by the
product package ``porqua_amd``.
"""
from __future__ import annotations

import numpy as np

# ----------------------------------------------------------------------------
# a3: trailing windows  (src/builders.py:188-215, :218-251)
# ----------------------------------------------------------------------------


def window_rows(dates: np.ndarray, rebdate, width: int) -> np.ndarray:
    """Row indices of ``data[data.index <= rebdate].tail(width)`` with weekends dropped.

    ``dates`` is a sorted ``datetime64[D]`` array (src/builders.py:208-211: the slice keeps
    the rebalance day itself and removes rows whose weekday is Sat/Sun afterwards).
    """
    dates = np.asarray(dates, dtype="datetime64[D]")
    end = int(np.searchsorted(dates, np.datetime64(rebdate, "D"), side="right"))
    start = max(0, end - int(width))
    rows = np.arange(start, end)
    # numpy weekday: 1970-01-01 was a Thursday (weekday 3, Mon=0)
    wd = (dates[rows].astype("int64") + 3) % 7
    return rows[wd < 5]


# ----------------------------------------------------------------------------
# a4: covariance estimators  (src/covariance.py:40-84)
# ----------------------------------------------------------------------------


def cov_pearson(X: np.ndarray) -> np.ndarray:
    """``DataFrame.cov()`` on a NaN-free window == ``np.cov(X.T, ddof=1)``.

    Restates numpy's two-pass algorithm (numpy/lib/_function_base_impl.py, ``cov``):
    centre by the column mean, ``dot``, then multiply by ``1/(T-1)``.
    src/covariance.py:65-66.
    """
    X = np.array(X, dtype=np.float64, copy=True)
    T = X.shape[0]
    X -= X.mean(axis=0)
    c = X.T @ X
    c *= np.true_divide(1, T - 1)
    return c


def cov_pairwise(X: np.ndarray) -> np.ndarray:
    """DataFrame.cov() of a window with missing values (src/covariance.py:65-66 on NaN data):
    pandas' pairwise-complete covariance -- entry (i, j) from the rows where both columns are
    present, centred by those rows' own means, ddof 1; NaN when fewer than 2 common rows."""
    X = np.asarray(X, dtype=np.float64)
    n = X.shape[1]
    ok = ~np.isnan(X)
    S = np.full((n, n), np.nan)
    for i in range(n):
        for j in range(i + 1):
            m = ok[:, i] & ok[:, j]
            N = int(m.sum())
            if N < 2:
                continue
            xi, xj = X[m, i], X[m, j]
            S[i, j] = S[j, i] = ((xi - xi.mean()) * (xj - xj.mean())).sum() / (N - 1)
    return S


def cov_pairwise_rows(X: np.ndarray) -> np.ndarray:
    """cov_pairwise with the pair loop vectorised over j (one row i at a time): the same
    two-pass arithmetic per pair -- centre each column by its mean over the rows both columns
    share, then sum the products, ddof 1 -- in O(n) numpy passes of T x n, so the restatement
    reaches the config sizes (n = 1000, T = 252) in seconds."""
    X = np.asarray(X, dtype=np.float64)
    n = X.shape[1]
    ok = ~np.isnan(X)
    X0 = np.where(ok, X, 0.0)
    S = np.full((n, n), np.nan)
    for i in range(n):
        m = ok[:, i:i + 1] & ok                                    # rows shared by (i, j), all j
        N = m.sum(0)
        with np.errstate(invalid="ignore", divide="ignore"):
            mi = (m * X0[:, i:i + 1]).sum(0) / N                   # mean of column i over those rows
            mj = (m * X0).sum(0) / N                               # mean of column j over those rows
            s = (m * (X0[:, i:i + 1] - mi) * (X0 - mj)).sum(0) / (N - 1)
        S[i] = np.where(N >= 2, s, np.nan)
    return S


def cov_linear_shrinkage(X: np.ndarray, lam) -> np.ndarray:
    """src/covariance.py:71-84: Sigma + lam * mean(diag Sigma) * I (lam<0/None/NaN -> 0)."""
    if lam is None or np.isnan(lam) or lam < 0:
        lam = 0.0
    S = cov_pearson(X)
    if lam > 0:
        n = S.shape[0]
        S = S + lam * np.mean(np.diag(S)) * np.eye(n)
    return S


def cov_duv(X: np.ndarray) -> np.ndarray:
    """src/covariance.py:68-69."""
    return np.identity(np.asarray(X).shape[1])


def is_pd(B: np.ndarray) -> bool:
    """src/helper_functions.py:61-67 (Cholesky succeeds)."""
    try:
        np.linalg.cholesky(B)
        return True
    except np.linalg.LinAlgError:
        return False


def nearest_pd(A: np.ndarray) -> np.ndarray:
    """Higham / D'Errico nearest SPD, src/helper_functions.py:29-58."""
    B = (A + A.T) / 2
    _, s, V = np.linalg.svd(B)
    H = V.T @ (np.diag(s) @ V)
    A2 = (B + H) / 2
    A3 = (A2 + A2.T) / 2
    if is_pd(A3):
        return A3
    k = 1
    while not is_pd(A3):
        spacing = np.spacing(np.linalg.norm(A))
        mineig = np.min(np.real(np.linalg.eigvals(A3)))
        A3 += np.eye(A.shape[0]) * (-mineig * k**2 + spacing)
        k += 1
    return A3


def covariance_estimate(X, method="pearson", check_positive_definite=True, lam=None):
    """``Covariance.estimate`` dispatch, src/covariance.py:40-56."""
    if method == "pearson":
        S = cov_pearson(X)
    elif method == "duv":
        S = cov_duv(X)
    elif method == "linear_shrinkage":
        S = cov_linear_shrinkage(X, lam)
    else:
        raise NotImplementedError("This method is not implemented yet")
    if check_positive_definite and not is_pd(S):
        S = nearest_pd(S)
    return S


# ----------------------------------------------------------------------------
# a6: geometric mean  (src/mean_estimation.py:39-48)
# ----------------------------------------------------------------------------


def mean_geometric(X: np.ndarray, n_mom=None, n_rev=None, scalefactor=None) -> np.ndarray:
    X = np.asarray(X, dtype=np.float64)
    n_mom = X.shape[0] if n_mom is None else n_mom
    n_rev = 0 if n_rev is None else n_rev
    scalefactor = 1 if scalefactor is None else scalefactor
    X = X[-n_mom:][: n_mom - n_rev] if n_mom > 0 else X[:0]
    return np.exp(np.log(1 + X).mean(axis=0) * scalefactor) - 1


# ----------------------------------------------------------------------------
# a7 / a8: objectives  (src/optimization.py:168-174, :186-191, :206-226, :234-256)
# ----------------------------------------------------------------------------


def objective_mean_variance(X, risk_aversion=1.0, **cov_kw):
    S = covariance_estimate(X, **cov_kw)
    P = S * risk_aversion * 2
    q = -mean_geometric(X)
    return P, q, None


def objective_least_squares(X, y, l2_penalty=None, log_transform=False):
    X = np.asarray(X, dtype=np.float64)
    y = np.asarray(y, dtype=np.float64).reshape(-1)
    if log_transform:
        X = np.log(1 + X)
        y = np.log(1 + y)
    P = 2 * (X.T @ X)
    q = (-2 * X.T @ y).reshape(-1)
    const = float(y @ y)
    if l2_penalty is not None and l2_penalty != 0:
        P = P + 2 * l2_penalty * np.eye(X.shape[1])
    return P, q, const


def objective_qeqw(X):
    n = np.asarray(X).shape[1]
    return cov_duv(X) * 2, np.zeros(n), None


def objective_wls(X, y, tau, log_transform=False):
    X = np.asarray(X, dtype=np.float64)
    y = np.asarray(y, dtype=np.float64).reshape(-1)
    if log_transform:
        X = np.log(1 + X)
        y = np.log(1 + y)
    lam = np.exp(-np.log(2) / tau)
    w = lam ** np.arange(X.shape[0])
    w = np.flip(w / np.sum(w) * len(w))
    P = 2 * (X.T @ (w[:, None] * X))
    q = -2 * X.T @ (w * y)
    const = float(y @ (w * y))
    return P, q, const


# ----------------------------------------------------------------------------
# a10: Constraints.to_GhAb  (src/constraints.py:114-167), reproduced verbatim in
# behaviour, including the box-rows-twice quirk when every linear row is '='.
# ----------------------------------------------------------------------------


def to_GhAb(n, budget=None, box=None, linear=None, lbub_to_G=False):
    """budget: (a, sense, rhs) | None;  box: (lower, upper) arrays | None;
    linear: (Amat m x n, sense list, rhs m) | None."""
    A = b = G = h = None
    if budget is not None:
        a, sense, rhs = budget
        if sense == "=":
            A = np.array(a, dtype=float)
            b = np.array(rhs, dtype=float)
        else:
            G = np.array(a, dtype=float)
            h = np.array(rhs, dtype=float)
    G_tmp = h_tmp = None
    if lbub_to_G:
        I = np.eye(n)
        G_tmp = np.concatenate((-I, I), axis=0)
        h_tmp = np.concatenate((-np.asarray(box[0]), np.asarray(box[1])), axis=0)
        G = np.vstack((G, G_tmp)) if G is not None else G_tmp
        h = np.concatenate((h, h_tmp), axis=None) if h is not None else h_tmp
    if linear is not None:
        Amat = np.array(linear[0], dtype=float, copy=True)
        sense = np.asarray(linear[1])
        rhs = np.array(linear[2], dtype=float, copy=True)
        geq = sense == ">="
        Amat[geq] = -Amat[geq]
        rhs[geq] = -rhs[geq]
        eq = sense == "="
        if eq.sum() > 0:
            A = np.vstack((A, Amat[eq])) if A is not None else Amat[eq]
            b = np.concatenate((b, rhs[eq]), axis=None) if b is not None else rhs[eq]
            if eq.sum() < Amat.shape[0]:
                G_tmp, h_tmp = Amat[~eq], rhs[~eq]
        else:
            G_tmp, h_tmp = Amat, rhs
        if G_tmp is not None:
            G = np.vstack((G, G_tmp)) if G is not None else G_tmp
            h = np.concatenate((h, h_tmp), axis=None) if h is not None else h_tmp
    A = A.reshape(-1, A.shape[-1]) if A is not None else None
    G = G.reshape(-1, G.shape[-1]) if G is not None else None
    return {"G": G, "h": h, "A": A, "b": b}


def box_bounds(n, box_type="LongOnly", lower=None, upper=None):
    """src/constraints.py:178-204 defaults, expanded to length-n arrays."""
    if box_type == "Unbounded":
        lower = -np.inf if lower is None else lower
        upper = np.inf if upper is None else upper
    elif box_type == "LongShort":
        lower = -1 if lower is None else lower
        upper = 1 if upper is None else upper
    else:
        if lower is None:
            if upper is None:
                lower, upper = 0, 1
            else:
                lower = np.asarray(upper) * 0
        else:
            upper = np.asarray(lower) * 0 + 1 if upper is None else upper
    lo = np.broadcast_to(np.asarray(lower, dtype=float), (n,)).copy()
    up = np.broadcast_to(np.asarray(upper, dtype=float), (n,)).copy()
    return lo, up


def objective_value(P, q, x, constant=None, with_const=True):
    """src/qp_problems.py:219-221: 0.5 x'Px + q'x (+ const)."""
    c = 0 if constant is None or not with_const else constant
    return float(0.5 * (x @ P @ x) + q @ x) + c
