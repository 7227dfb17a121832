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

Workloads (``--workload``, the same synthetic inputs bench.py's GPU legs solve):
  config3  min-variance above, n = 1000 (the headline);
  config2  LeastSquares SPTR replication on the usa-shaped panel (n = 494, daily dates):
           P = 2 X'X, q = -2 X'y (src/optimization.py:206-226, uncentred), budget + box;
  config1  the same at the notebook's monthly rebalancing (every 21st date);
  config4  the same tracking objective at n = 3000 with the 20 sector caps G x <= 0.15
           (src/constraints.py:66-94, 114-167);
  config5  MeanVariance lambda sweep at n = 5000: Sigma by np.cov + nearestPD
           (src/covariance.py:40-56), P = 2 lam Sigma, q = -geometric mean
           (src/optimization.py:157-174, src/mean_estimation.py:39-48), budget + box;
each followed by the solve's own isPD / nearestPD of P (src/qp_problems.py:189-191), as the
reference runs it.  Samples are bounded by the per-QP cost: n = 3000 / 5000 QPs take tens of
seconds to minutes each on one core (nearestPD's SVD + eigvals dominate), so those legs time
one QP per worker.

Run as a CHILD process (``python -m oracle.cpu_baseline ...``), before the bench touches the
GPU; the pool's workers are spawned (fresh interpreters, single-threaded BLAS); prints one
JSON object on stdout and progress lines on stderr.
"""
from __future__ import annotations

import json
import os
import time

import numpy as np

from .qp_ipm import solve_qp
from .ref_pipeline import cov_pearson, is_pd, mean_geometric, nearest_pd


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


def reference_ls(X: np.ndarray, y: np.ndarray, G=None, h=None, repair: bool = True):
    """LeastSquares tracking date (src/optimization.py:206-226: P = 2 X'X uncentred, q = -2 X'y),
    budget + long-only box (+ G x <= h), the solve's PD repair (src/qp_problems.py:189-191)."""
    n = X.shape[1]
    P = 2.0 * (X.T @ X)
    q = -2.0 * (X.T @ y)
    if repair and not is_pd(P):
        P = _nearest_pd(P)
    return solve_qp(P, q, G=G, h=h, A=np.ones((1, n)), b=np.ones(1), lb=np.zeros(n), ub=np.ones(n),
                    tol=1e-7, refine=False)


def reference_mv(X: np.ndarray, lam: float, repair: bool = True):
    """MeanVariance date of the lambda sweep (src/optimization.py:157-174): Covariance.estimate
    (np.cov + isPD / nearestPD), P = 2 lam Sigma, q = -geometric mean, then the solve's repair."""
    n = X.shape[1]
    S = cov_pearson(X)
    if repair and not is_pd(S):
        S = _nearest_pd(S)
    P = 2.0 * lam * S
    q = -mean_geometric(X)
    if repair and not is_pd(P):
        P = _nearest_pd(P)
    return solve_qp(P, q, A=np.ones((1, n)), b=np.ones(1), lb=np.zeros(n), ub=np.ones(n), tol=1e-7, refine=False)


class Workload:
    """The synthetic inputs of one bench workload (built identically in every pool worker)
    and its per-QP reference call.  ``units``: the QP ids to sample (row index of the
    rebalance day, or (row, lambda index) for the sweep)."""

    def __init__(self, name: str, n: int, T: int, dates: int, seed: int, root: str = "."):
        from porqua_amd.synthetic import factor_panel, usa_panel
        self.name, self.T = name, T
        self.G = self.h = None
        if name in ("config1", "config2"):   # monthly (every 21st row) / daily rebalancing
            g = np.load(os.path.join(root, "tests", "golden", "sptr.npz"), allow_pickle=False)
            _, self.R, self.y = usa_panel(g["days"], g["returns"], n_assets=n)
            self.units = list(range(T - 1, self.R.shape[0], 21 if name == "config1" else 1))
        elif name == "config4":
            _, self.R, self.y, sec = factor_panel(T - 1 + dates, n, n_sectors=20)
            self.G = np.stack([(sec == k).astype(float) for k in range(20)])
            self.h = np.full(20, 0.15)
            self.units = list(range(T - 1, T - 1 + dates))
        elif name == "config5":
            stride, n_lam = 21, 64
            self.R = factor_panel(T - 1 + stride * dates, n)[1]
            self.lams = np.logspace(-1, 2, n_lam)
            ends = np.arange(T - 1, T - 1 + stride * dates, stride)
            self.units = [(int(e), k) for e in ends for k in range(n_lam)]
        else:
            self.R = factor_panel(T - 1 + dates, n, seed=seed)[1]
            self.units = list(range(T - 1, T - 1 + dates))

    def sample(self, k: int):
        """k evenly spaced QPs of the workload (for the sweep: spread over dates AND lambdas)."""
        pos = np.linspace(0, len(self.units) - 1, max(1, k)).astype(int)
        if self.name == "config5":   # stride through the (date, lambda) grid so lambdas vary too
            pos = (np.arange(k) * (len(self.units) // max(1, k) + 1)) % len(self.units)
        return [self.units[i] for i in pos]

    def solve(self, u, repair: bool = True):
        T = self.T
        if self.name in ("config1", "config2", "config4"):
            return reference_ls(self.R[u - T + 1:u + 1], self.y[u - T + 1:u + 1], self.G, self.h, repair)
        if self.name == "config5":
            e, k = u
            return reference_mv(self.R[e - T + 1:e + 1], float(self.lams[k]), repair)
        return reference_date(self.R[u - T + 1:u + 1], repair=repair)


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


def time_reference(wl: "Workload", units, budget_s: float = 20.0, max_dates: int = 8, repair=True):
    """Run the per-QP reference path on ``units`` until ``budget_s`` seconds or ``max_dates``
    QPs; returns (qps, dates_done, seconds)."""
    t0 = time.perf_counter()
    done = 0
    with _Heartbeat("serial" + ("" if repair else " solver-only")):
        for u in units:
            wl.solve(u, repair=repair)
            done += 1
            _progress(f"serial {done}/{min(len(units), max_dates)} ({time.perf_counter() - t0:.1f} s)")
            if done >= max_dates or time.perf_counter() - t0 > budget_s:
                break
    dt = time.perf_counter() - t0
    return done / dt, done, dt


def _progress(msg: str):
    import sys
    print(f"[cpu_baseline] {msg}", file=sys.stderr, flush=True)


class _Heartbeat:
    """A progress line every ``every`` seconds while a leg runs (one n = 5000 QP takes minutes
    on a core, and a run that prints nothing for minutes looks hung)."""

    def __init__(self, what: str, every: float = 30.0):
        import threading
        self.what, self.every = what, every
        self._stop = threading.Event()
        self._t = threading.Thread(target=self._run, daemon=True)

    def _run(self):
        t0 = time.perf_counter()
        while not self._stop.wait(self.every):
            _progress(f"{self.what}: running ({time.perf_counter() - t0:.0f} s)")

    def __enter__(self):
        self._t.start()
        return self

    def __exit__(self, *exc):
        self._stop.set()
        self._t.join()


_POOL = {}


def _pool_init(name, n, T, dates, seed, root):
    _POOL["wl"] = Workload(name, n, T, dates, seed, root)


def _pool_date(args):
    u, repair = args
    _POOL["wl"].solve(u, repair=repair)
    return 1


def time_pool(name, n, T, dates, seed, units, workers, repair=True, root="."):
    """(b): ``workers`` single-threaded processes over ``units``; returns (qps, done, seconds)
    timed from the first submitted QP to the last result (pool start-up and the workers'
    panel construction excluded).  Progress lines while it runs (a long leg stays visibly
    alive)."""
    import multiprocessing as mp
    ctx = mp.get_context("spawn")   # fresh interpreters: no BLAS thread state copied by fork
    with ctx.Pool(workers, initializer=_pool_init, initargs=(name, n, T, dates, seed, root)) as pool:
        # warm: panel built, BLAS loaded (the solver-only path, cheap next to the repair)
        with _Heartbeat("pool warm-up"):
            pool.map(_pool_date, [(units[0], False)] * workers)
        t0 = time.perf_counter()
        done = 0
        with _Heartbeat("pool" + ("" if repair else " solver-only")):
            for _ in pool.imap_unordered(_pool_date, [(u, repair) for u in units], chunksize=1):
                done += 1
                _progress(f"pool{'' if repair else ' solver-only'} {done}/{len(units)} "
                          f"({time.perf_counter() - t0:.1f} s)")
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
    ap.add_argument("--workload", choices=["config1", "config2", "config3", "config4", "config5"], default="config3")
    ap.add_argument("--n", type=int, default=1000)
    ap.add_argument("--window", type=int, default=252)
    ap.add_argument("--dates", type=int, default=4749)
    ap.add_argument("--seed", type=int, default=20240314)
    ap.add_argument("--serial-dates", type=int, default=6)
    ap.add_argument("--pool-rounds", type=int, default=2, help="QPs per worker in the pool leg")
    ap.add_argument("--workers", type=int, default=0)
    ap.add_argument("--budget", type=float, default=20.0)
    ap.add_argument("--no-solver-only", action="store_true", help="skip the solver-only legs")
    a = ap.parse_args()
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    T, n = a.window, a.n
    workers = a.workers or host_cores()
    wl = Workload(a.workload, n, T, a.dates, a.seed, root)
    sample = wl.sample(max(a.serial_dates, workers * a.pool_rounds))
    out = {"workload": a.workload, "n": n, "host_cores": host_cores(), "cpu_model": cpu_model(),
           "os_cpu_count": os.cpu_count()}
    qs, ds, ss = time_reference(wl, sample[:a.serial_dates], budget_s=a.budget, max_dates=a.serial_dates)
    out["serial"] = {"qps": qs, "dates": ds, "seconds": ss, "blas_threads": blas_threads()}
    if not a.no_solver_only:
        qo, do, so = time_reference(wl, sample[:a.serial_dates], budget_s=a.budget, max_dates=a.serial_dates,
                                    repair=False)
        out["serial_solver_only"] = {"qps": qo, "dates": do, "seconds": so}
    del wl
    pool_units = sample[:workers * a.pool_rounds]
    for k in ("OMP_NUM_THREADS", "OPENBLAS_NUM_THREADS", "MKL_NUM_THREADS"):
        os.environ[k] = "1"
    try:
        from threadpoolctl import threadpool_limits
        threadpool_limits(1)
    except Exception:
        pass
    qp, dp, sp = time_pool(a.workload, n, T, a.dates, a.seed, pool_units, workers, root=root)
    out["pool"] = {"qps": qp, "dates": dp, "seconds": sp, "workers": workers, "threads_per_worker": 1}
    if not a.no_solver_only:
        qpo, dpo, spo = time_pool(a.workload, n, T, a.dates, a.seed, pool_units, workers, repair=False, root=root)
        out["pool_solver_only"] = {"qps": qpo, "dates": dpo, "seconds": spo, "workers": workers}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
