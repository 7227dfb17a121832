#!/usr/bin/env python3
"""Oracle optima for the large-n configurations (BASELINE.json configs[3], configs[4]) at
the shapes the GPU tests run -> tests/golden/config4_oracle.npz, config5_oracle.npz.

* config 4: n = 3000 tracking least squares (P = 2 X'X uncentred, q = -2 X'y,
  src/optimization.py:206-226) with budget, long-only box and 20 sector caps <= 0.15,
  windows ending at panel rows 260 .. 265 (tests/test_large_n_gpu.py).
* config 5: n = 5000 mean-variance (P = 2 lam Sigma, q = -mu geometric,
  src/optimization.py:168-174, src/mean_estimation.py:39-48), budget + box [0, 1], windows
  ending at rows 300 and 321, risk aversions logspace(-1, 2, 4).

Solved by oracle.qp_ipm.solve_qp (KKT-certified).  Test infrastructure only.  Takes about
10 minutes on 8 cores:  python tools/capture_large.py [4|5]
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle.qp_ipm import solve_qp  # noqa: E402
from oracle.ref_pipeline import cov_pearson  # noqa: E402
from porqua_amd.synthetic import factor_panel  # noqa: E402

GOLD = os.path.join(ROOT, "tests", "golden")


def config4():
    n, T, ns, cap = 3000, 252, 20, 0.15
    ends = list(range(260, 266))
    dates, R, y, sec = factor_panel(max(ends) + 1, n, n_sectors=ns)
    G = np.stack([(sec == g).astype(float) for g in range(ns)])
    xs, objs, prim, dual = [], [], [], []
    for e in ends:
        t = time.time()
        X = R[e - T + 1:e + 1]
        P, q = 2 * X.T @ X, -2 * X.T @ y[e - T + 1:e + 1]
        o = solve_qp(P, q, G=G, h=np.full(ns, cap), A=np.ones((1, n)), b=np.ones(1), lb=np.zeros(n), ub=np.ones(n))
        assert o.found
        xs.append(o.x)
        objs.append(o.obj)
        prim.append(o.extras["kkt_primal"])
        dual.append(o.extras["kkt_dual"])
        print("config4", e, o.obj, f"{time.time() - t:.1f}s", flush=True)
    np.savez_compressed(os.path.join(GOLD, "config4_oracle.npz"), ends=np.array(ends), x=np.stack(xs),
                        obj=np.array(objs), kkt_primal=np.array(prim), kkt_dual=np.array(dual), n=n, T=T,
                        n_sectors=ns, cap=cap)


def config5():
    n, T = 5000, 252
    lambdas = np.logspace(-1, 2, 4)
    ends = [300, 321]
    dates, R, _, _ = factor_panel(max(ends) + 1, n)
    xs, objs, prim, dual, pairs = [], [], [], [], []
    for e in ends:
        W = R[e - T + 1:e + 1]
        S = cov_pearson(W)
        mu = np.exp(np.mean(np.log1p(W), axis=0)) - 1.0
        for j, lam in enumerate(lambdas):
            t = time.time()
            o = solve_qp(2 * lam * S, -mu, A=np.ones((1, n)), b=np.ones(1), lb=np.zeros(n), ub=np.ones(n))
            assert o.found
            xs.append(o.x)
            objs.append(o.obj)
            prim.append(o.extras["kkt_primal"])
            dual.append(o.extras["kkt_dual"])
            pairs.append((e, j))
            print("config5", e, lam, o.obj, int((o.x > 1e-9).sum()), f"{time.time() - t:.1f}s", flush=True)
    np.savez_compressed(os.path.join(GOLD, "config5_oracle.npz"), pairs=np.array(pairs), lambdas=lambdas,
                        x=np.stack(xs), obj=np.array(objs), kkt_primal=np.array(prim), kkt_dual=np.array(dual),
                        n=n, T=T)


if __name__ == "__main__":
    which = sys.argv[1:] or ["4", "5"]
    if "4" in which:
        config4()
    if "5" in which:
        config5()
