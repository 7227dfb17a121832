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

Two ways of running it, as BASELINE.md §3 plans, and the better one is the denominator:
  (a) serial: one date after another with multithreaded BLAS (how the reference runs);
  (b) pool: one single-threaded worker process per host core, dates spread over them.
A solver-only variant (no nearestPD: the IPM takes the PSD P as it is) is timed beside it.

Run as a CHILD process (``python -m oracle.cpu_baseline ...``), before the bench touches the
GPU; the pool's workers are spawned (fresh interpreters, single-threaded BLAS); prints one
JSON object.
"""
from __future__ import annotations

import json
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


def reference_date(X: np.ndarray, ub: float = 1.0, shrink: float = 0.0, repair: bool = True):
    n = X.shape[1]
    S = cov_pearson(X)
    if shrink > 0:
        S = S + shrink * np.mean(np.diag(S)) * np.eye(n)
    if repair and not is_pd(S):
        S = _nearest_pd(S)
    P = 2.0 * S
    q = np.zeros(n)
    if repair and not is_pd(P):
        P = _nearest_pd(P)
    sol = solve_qp(P, q, A=np.ones((1, n)), b=np.ones(1), lb=np.zeros(n), ub=np.full(n, ub),
                   tol=1e-7, refine=False)
    return sol


def _nearest_pd(A: np.ndarray) -> np.ndarray:
    """nearest_pd, retrying once with LAPACK gesvd when gesdd (numpy's SVD) does not converge
    -- the same repair, so the timed work is unchanged."""
    try:
        return nearest_pd(A)
    except np.linalg.LinAlgError:
        import scipy.linalg
        B = (A + A.T) / 2
        _, s, V = scipy.linalg.svd(B, lapack_driver="gesvd")
        A2 = (B + V.T @ (np.diag(s) @ V)) / 2
        A3 = (A2 + A2.T) / 2
        k = 1
        while not is_pd(A3):
            mineig = np.min(np.real(np.linalg.eigvals(A3)))
            A3 += np.eye(A.shape[0]) * (-mineig * k**2 + np.spacing(np.linalg.norm(A)))
            k += 1
        return A3


def time_reference(R: np.ndarray, ends, T: int, budget_s: float = 20.0, max_dates: int = 8, repair=True):
    """Run the per-date reference path on dates ``ends`` (row index of the rebalance day)
    until ``budget_s`` seconds or ``max_dates`` dates; returns (qps, dates_done, seconds)."""
    t0 = time.perf_counter()
    done = 0
    for e in ends:
        reference_date(R[e - T + 1:e + 1], repair=repair)
        done += 1
        if done >= max_dates or time.perf_counter() - t0 > budget_s:
            break
    dt = time.perf_counter() - t0
    return done / dt, done, dt


_POOL = {}


def _pool_init(n_dates, n, T, seed):
    from porqua_amd.synthetic import factor_panel
    _POOL["R"] = factor_panel(n_dates, n, seed=seed)[1]
    _POOL["T"] = T


def _pool_date(args):
    e, repair = args
    R, T = _POOL["R"], _POOL["T"]
    reference_date(R[e - T + 1:e + 1], repair=repair)
    return e


def time_pool(n_dates, n, T, ends, workers, seed, repair=True):
    """(b): ``workers`` single-threaded processes over ``ends``; returns (qps, done, seconds)
    timed from the first submitted date to the last result (pool start-up excluded)."""
    import multiprocessing as mp
    ctx = mp.get_context("spawn")   # fresh interpreters: no BLAS thread state copied by fork
    with ctx.Pool(workers, initializer=_pool_init, initargs=(n_dates, n, T, seed)) as pool:
        pool.map(_pool_date, [(ends[0], False)] * workers)     # warm: panel built, BLAS loaded
        t0 = time.perf_counter()
        done = len(pool.map(_pool_date, [(e, repair) for e in ends], chunksize=1))
        dt = time.perf_counter() - t0
    return done / dt, done, dt


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def host_cores() -> int:
    """Cores this job may use: the affinity mask, capped by OMP_NUM_THREADS when set (the GPU
    box exports the job's CPU share there; os.cpu_count() shows the whole machine)."""
    c = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        c = min(c, int(env))
    return max(1, c)


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1000)
    ap.add_argument("--window", type=int, default=252)
    ap.add_argument("--dates", type=int, default=4749)
    ap.add_argument("--seed", type=int, default=20240314)
    ap.add_argument("--serial-dates", type=int, default=6)
    ap.add_argument("--pool-rounds", type=int, default=2, help="dates per worker in the pool leg")
    ap.add_argument("--workers", type=int, default=0)
    ap.add_argument("--budget", type=float, default=20.0)
    a = ap.parse_args()
    from porqua_amd.synthetic import factor_panel
    T, D, n = a.window, a.dates, a.n
    n_rows = T - 1 + D
    workers = a.workers or host_cores()
    R = factor_panel(n_rows, n, seed=a.seed)[1]
    sample = np.linspace(T - 1, n_rows - 1, max(a.serial_dates, workers * a.pool_rounds)).astype(int)
    out = {"host_cores": host_cores(), "cpu_model": cpu_model(), "os_cpu_count": os.cpu_count()}
    qs, ds, ss = time_reference(R, sample[:a.serial_dates], T, budget_s=a.budget, max_dates=a.serial_dates)
    out["serial"] = {"qps": qs, "dates": ds, "seconds": ss, "blas_threads": blas_threads()}
    qo, do, so = time_reference(R, sample[:a.serial_dates], T, budget_s=a.budget, max_dates=a.serial_dates,
                                repair=False)
    out["serial_solver_only"] = {"qps": qo, "dates": do, "seconds": so}
    del R
    pool_ends = sample[:workers * a.pool_rounds]
    for k in ("OMP_NUM_THREADS", "OPENBLAS_NUM_THREADS", "MKL_NUM_THREADS"):
        os.environ[k] = "1"
    try:
        from threadpoolctl import threadpool_limits
        threadpool_limits(1)
    except Exception:
        pass
    qp, dp, sp = time_pool(n_rows, n, T, pool_ends, workers, a.seed)
    out["pool"] = {"qps": qp, "dates": dp, "seconds": sp, "workers": workers, "threads_per_worker": 1}
    qpo, dpo, spo = time_pool(n_rows, n, T, pool_ends, workers, a.seed, repair=False)
    out["pool_solver_only"] = {"qps": qpo, "dates": dpo, "seconds": spo, "workers": workers}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
