#!/usr/bin/env python3
"""Oracle optima at the FULL benchmark shapes of configs 2, 4 and 5, on 16 evenly spaced
problems each (TEST INFRASTRUCTURE ONLY) -> tests/golden/config{2d,4f,5f}_oracle.npz.

The problems are exactly the ones tools/bench_configs.py times and tests/test_full_configs_gpu.py
certifies:
* config 2 daily: SPTR replication on the usa-shaped panel (porqua_amd.synthetic.usa_panel),
  every date from row 251 on (4544 daily LS tracking QPs, n = 494): P = 2 X'X, q = -2 X'y
  (src/optimization.py:206-226), budget + LongOnly box;
* config 4: factor_panel(10000, 3000, n_sectors=20), windows ending at rows 251 .. 9999
  (9749 QPs), LS tracking with budget, box [0, 1] and 20 sector caps <= 0.15
  (src/constraints.py:66-94, 114-167);
* config 5: factor_panel(251 + 21 * 64, 5000), 64 monthly windows x 64 risk aversions
  logspace(-1, 2, 64) (4096 QPs), P = 2 lam Sigma_pearson, q = -mu_geometric
  (src/optimization.py:168-174, src/mean_estimation.py:39-48), budget + box [0, 1].

Solved by oracle.qp_ipm.solve_qp (cvxopt coneqp restatement + active-set refinement,
KKT-certified).  Run on the CPU:  python tools/capture_full.py [2] [4] [5]   (~1 h on 8 cores)
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle.qp_ipm import solve_qp  # noqa: E402
from oracle.ref_pipeline import cov_pearson  # noqa: E402
from porqua_amd.synthetic import factor_panel, usa_panel  # noqa: E402

GOLD = os.path.join(ROOT, "tests", "golden")
NPICK = 16


def picks(total, k=NPICK):
    return np.unique(np.round(np.linspace(0, total - 1, k)).astype(np.int64))


def _save(name, **kw):
    np.savez_compressed(os.path.join(GOLD, name), **kw)
    print("wrote", name, flush=True)


def _solve(P, q, **cons):
    t = time.time()
    o = solve_qp(P, q, **cons)
    assert o.found
    return o, time.time() - t


def config2():
    g = np.load(os.path.join(GOLD, "sptr.npz"))
    days, R, y = usa_panel(g["days"], g["returns"])
    T, n = 252, R.shape[1]
    ends = np.arange(T - 1, R.shape[0])
    sel = picks(len(ends))
    xs, objs = [], []
    for p in sel:
        e = ends[p]
        X, yw = R[e - T + 1:e + 1], y[e - T + 1:e + 1]
        o, dt = _solve(2 * X.T @ X, -2 * X.T @ yw, A=np.ones((1, n)), b=np.ones(1), lb=np.zeros(n), ub=np.ones(n))
        xs.append(o.x)
        objs.append(o.obj)
        print("config2", p, e, o.obj, f"{dt:.1f}s", flush=True)
    _save("config2d_oracle.npz", problems=sel, ends=ends[sel], x=np.stack(xs), obj=np.array(objs), n=n, T=T,
          n_dates=len(ends))


def config4():
    n, T, ns, cap = 3000, 252, 20, 0.15
    dates, R, y, sec = factor_panel(10000, n, n_sectors=ns)
    ends = np.arange(T - 1, 10000)
    G = np.stack([(sec == g).astype(float) for g in range(ns)])
    sel = picks(len(ends))
    xs, objs = [], []
    for p in sel:
        e = ends[p]
        X = R[e - T + 1:e + 1]
        o, dt = _solve(2 * X.T @ X, -2 * X.T @ y[e - T + 1:e + 1], G=G, h=np.full(ns, cap), A=np.ones((1, n)),
                       b=np.ones(1), lb=np.zeros(n), ub=np.ones(n))
        xs.append(o.x)
        objs.append(o.obj)
        print("config4", p, e, o.obj, int((o.x > 1e-9).sum()), f"{dt:.1f}s", flush=True)
    _save("config4f_oracle.npz", problems=sel, ends=ends[sel], x=np.stack(xs), obj=np.array(objs), n=n, T=T,
          n_sectors=ns, cap=cap, n_dates=len(ends))


def config5():
    n, T, nd, L = 5000, 252, 64, 64
    dates, R, _, _ = factor_panel(T - 1 + 21 * nd, n)
    ends = np.arange(T - 1, T - 1 + 21 * nd, 21)
    lambdas = np.logspace(-1, 2, L)
    sel = picks(nd * L)
    xs, objs = [], []
    cache = {}
    for p in sel:
        d, j = divmod(int(p), L)
        e = ends[d]
        if d not in cache:
            W = R[e - T + 1:e + 1]
            cache = {d: (cov_pearson(W), np.exp(np.mean(np.log1p(W), axis=0)) - 1.0)}
        S, mu = cache[d]
        o, dt = _solve(2 * lambdas[j] * S, -mu, A=np.ones((1, n)), b=np.ones(1), lb=np.zeros(n), ub=np.ones(n))
        xs.append(o.x)
        objs.append(o.obj)
        print("config5", p, e, lambdas[j], o.obj, int((o.x > 1e-9).sum()), f"{dt:.1f}s", flush=True)
    _save("config5f_oracle.npz", problems=sel, ends=ends[sel // L], lam_index=sel % L, lambdas=lambdas,
          x=np.stack(xs), obj=np.array(objs), n=n, T=T, n_dates=nd)


if __name__ == "__main__":
    which = sys.argv[1:] or ["2", "4", "5"]
    for w in which:
        {"2": config2, "4": config4, "5": config5}[w]()
