#!/usr/bin/env python3
"""Oracle optima of the headline workload (bench.py, BASELINE.json configs[2]) on 32
evenly spaced rebalance dates -> tests/golden/headline_c3.npz.

The problem is MinVarianceBacktest's: seed-20240314 factor panel (synthetic.factor_panel,
5000 rows x 1000 assets), 252-day windows ending at rows 251 .. 4999, P = 2 * Pearson
covariance (oracle.ref_pipeline.cov_pearson = np.cov two-pass, ddof 1, src/covariance.py:65-66),
q = 0, budget 1'x = 1, box [0, 1].  Each date is solved by oracle.qp_ipm.solve_qp (the
cvxopt-coneqp restatement + active-set refinement, KKT-certified).  Test infrastructure:
only the GPU parity test reads the fixture.  Run from the repo root:

    OPENBLAS_NUM_THREADS=1 python tools/capture_headline.py
"""
import os
import sys
from multiprocessing import Pool

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

N, T, D = 1000, 252, 4749
NPICK = 32
_R = None


def _init():
    global _R
    from porqua_amd.synthetic import factor_panel
    _R = factor_panel(T - 1 + D, N)[1]


def _solve(d):
    from oracle.qp_ipm import solve_qp
    from oracle.ref_pipeline import cov_pearson
    e = T - 1 + d
    P = 2.0 * cov_pearson(_R[e - T + 1:e + 1])
    o = solve_qp(P, np.zeros(N), A=np.ones((1, N)), b=np.ones(1), lb=np.zeros(N), ub=np.ones(N))
    return d, o.x, o.obj, o.extras["kkt_primal"], o.extras["kkt_dual"], int(o.found)


def main():
    picks = np.unique(np.linspace(0, D - 1, NPICK).round().astype(int))
    with Pool(min(8, os.cpu_count() or 1), initializer=_init) as pool:
        out = sorted(pool.map(_solve, picks))
    x = np.stack([o[1] for o in out])
    obj = np.array([o[2] for o in out])
    prim = np.array([o[3] for o in out])
    dual = np.array([o[4] for o in out])
    found = np.array([o[5] for o in out])
    assert found.all()
    nfree = ((x > 1e-9) & (x < 1 - 1e-9)).sum(1)
    print("dates", picks.tolist())
    print("obj", obj.min(), obj.max(), "prim", prim.max(), "dual", dual.max(), "nfree", nfree.min(), nfree.max())
    np.savez_compressed(os.path.join(ROOT, "tests", "golden", "headline_c3.npz"), date_index=picks, x=x, obj=obj,
                        kkt_primal=prim, kkt_dual=dual, n=N, T=T, D=D, seed=20240314)


if __name__ == "__main__":
    main()
