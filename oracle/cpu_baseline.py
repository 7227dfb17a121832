"""CPU baseline: the reference's per-date path restated in numpy, timed on host cores
(TEST / BENCH INFRASTRUCTURE ONLY -- bench.py's cpu_baseline leg).

Per rebalance date, exactly the arithmetic Backtest.run performs (src/backtest.py:201-224)
for MeanVariance-style min-variance with Pearson covariance:
  window (src/builders.py:208-211) -> X.cov() (src/covariance.py:65-66)
  -> isPD / nearestPD (src/covariance.py:52-54, src/helper_functions.py:29-67)
  -> P = 2 Sigma, q = 0 -> isPD(P) again (src/qp_problems.py:189-191)
  -> dense QP solve.
The QP is solved by ``oracle.qp_ipm`` (the cvxopt-coneqp algorithm family) with cvxopt's
default tolerances (1e-7), since qpsolvers / cvxopt are not installed ("reference CPU solver
unavailable"); this is the "port" baseline kind.
"""
from __future__ import annotations

import os
import time

import numpy as np

from .qp_ipm import solve_qp
from .ref_pipeline import cov_pearson, is_pd, nearest_pd


def blas_threads() -> int:
    try:
        from threadpoolctl import threadpool_info
        n = [d.get("num_threads", 1) for d in threadpool_info() if d.get("user_api") == "blas"]
        return int(max(n)) if n else 1
    except Exception:
        return os.cpu_count() or 1


def reference_date(X: np.ndarray, ub: float = 1.0, shrink: float = 0.0):
    n = X.shape[1]
    S = cov_pearson(X)
    if shrink > 0:
        S = S + shrink * np.mean(np.diag(S)) * np.eye(n)
    if not is_pd(S):
        S = nearest_pd(S)
    P = 2.0 * S
    q = np.zeros(n)
    if not is_pd(P):
        P = nearest_pd(P)
    sol = solve_qp(P, q, A=np.ones((1, n)), b=np.ones(1), lb=np.zeros(n), ub=np.full(n, ub),
                   tol=1e-7, refine=False)
    return sol


def time_reference(R: np.ndarray, ends, T: int, budget_s: float = 20.0, max_dates: int = 8):
    """Run the per-date reference path on dates ``ends`` (row index of the rebalance day)
    until ``budget_s`` seconds or ``max_dates`` dates; returns (qps, dates_done, seconds)."""
    t0 = time.perf_counter()
    done = 0
    for e in ends:
        reference_date(R[e - T + 1:e + 1])
        done += 1
        if done >= max_dates or time.perf_counter() - t0 > budget_s:
            break
    dt = time.perf_counter() - t0
    return done / dt, done, dt
