#!/usr/bin/env python3
"""Config 1 (BASELINE.json configs[0]): SPTR index replication, monthly rebalance, least-squares
tracking on CPU -> tests/golden/config1_oracle.npz.

The reference run (example/backtest.ipynb, cell 1) is LeastSquares(solver_name='cvxopt') with
a budget and a LongOnly box, width 252, rebdates = dates[dates > start][::21], on
data/usa_returns.parquet against data/SPTR.csv.  usa_returns is absent from the reference
tree, so the panel is porqua_amd.synthetic.usa_panel (494 assets on the last 4795 SPTR dates,
loading on the real SPTR); its calendar ends with SPTR on 2023-06-06, so start = 2022-06-01
gives the 13 monthly dates of SURVEY.md §8(a) (the notebook's 2023-01-01 would give 6).

Per date, the reference path restated by the oracle: window (src/builders.py:208-211), P = 2
X'X, q = -2 X'y (src/optimization.py:206-226), budget + box (src/constraints.py), solved by
oracle.qp_ipm (cvxopt-coneqp algorithm family, KKT-certified) -- the CPU reference of config 1,
timed per date.  Test infrastructure only:  python tools/capture_config1.py
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle.qp_ipm import solve_qp  # noqa: E402
from oracle.ref_pipeline import box_bounds, objective_least_squares, window_rows  # noqa: E402
from porqua_amd.synthetic import usa_panel  # noqa: E402

WIDTH, STRIDE, START = 252, 21, "2022-06-01"


def config1_dates(days):
    d = np.asarray(days, dtype="datetime64[D]")
    return d[d > np.datetime64(START)][::STRIDE]


def main():
    g = np.load(os.path.join(ROOT, "tests", "golden", "sptr.npz"))
    dates, R, y = usa_panel(g["days"], g["returns"])
    reb = config1_dates(dates)
    n = R.shape[1]
    lb, ub = box_bounds(n, "LongOnly")
    xs, objs, consts, secs, prim, dual = [], [], [], [], [], []
    for rd in reb:
        t0 = time.perf_counter()
        rows = window_rows(dates, rd, WIDTH)
        P, q, const = objective_least_squares(R[rows], y[rows])
        o = solve_qp(P, q, A=np.ones((1, n)), b=np.ones(1), lb=lb, ub=ub)
        secs.append(time.perf_counter() - t0)
        assert o.found
        xs.append(o.x)
        objs.append(o.obj)
        consts.append(const)
        prim.append(o.extras["kkt_primal"])
        dual.append(o.extras["kkt_dual"])
        print(str(rd), o.obj, int((o.x > 1e-8).sum()), f"{secs[-1]:.2f}s", file=sys.stderr)
    np.savez_compressed(os.path.join(ROOT, "tests", "golden", "config1_oracle.npz"),
                        rebdates=reb.astype("datetime64[D]").astype(np.int64), x=np.stack(xs), obj=np.array(objs),
                        constant=np.array(consts), seconds=np.array(secs), kkt_primal=np.array(prim),
                        kkt_dual=np.array(dual), width=WIDTH, stride=STRIDE, start=np.array(START))


if __name__ == "__main__":
    main()
