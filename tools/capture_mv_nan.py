#!/usr/bin/env python3
"""Golden vectors for a mean-variance backtest on a panel with missing values (assets that
enter late, leave early, and holes): the reference's own Backtest.run (src/backtest.py) with
the capturing qpsolvers stub of tools/capture_golden.py records the exact P, q, A, b, lb, ub
per rebalance date -- P from Covariance.estimate on NaN windows (pandas pairwise-complete
covariance + isPD/nearestPD), q from MeanEstimator (pandas skipna) -- and oracle.qp_ipm
solves them -> tests/golden/msci_mv_nan.npz.  Build container only (imports the reference).
Test infrastructure only:  python tools/capture_mv_nan.py"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import capture_golden as cg  # noqa: E402  (sets up the reference import + solver stub)


def nan_panel():
    X, y = cg.load_msci()
    X = X.copy()
    rng = np.random.default_rng(11)
    X.iloc[:3800, 3] = np.nan          # enters late (inside the backtest span)
    X.iloc[-700:, 7] = np.nan          # leaves early
    for c in (10, 11, 12, 15):
        X.iloc[rng.random(len(X)) < 0.03, c] = np.nan   # holes
    return X, y


def main():
    X, y = nan_panel()
    dates = X.index
    # every window sees >= 10 rows of the late entrant and >= 10 of the early leaver (an
    # all-NaN column makes the reference's P / q NaN: its solver call fails there)
    rebdates = dates[3820:len(dates) - 700 + 240:21].strftime("%Y-%m-%d").tolist()
    opt = cg.MeanVariance(solver_name="cvxopt")
    probs, consts, wins = cg.run_backtest(opt, X, y, rebdates, 252, {"upper": 0.25})
    xs, objs, kp, kd = cg.golden_solutions(probs)
    # the panel is tests/golden/msci_panel.npz with these entries set to NaN
    nan_rc = np.argwhere(np.isnan(X.to_numpy())).astype(np.int32)
    np.savez_compressed(os.path.join(cg.OUT, "msci_mv_nan.npz"), nan_rc=nan_rc, rebdates=np.array(rebdates),
                        P=cg.stack(probs, "P"), q=cg.stack(probs, "q"), lb=cg.stack(probs, "lb"),
                        ub=cg.stack(probs, "ub"), x=xs, obj=objs, kkt_primal=kp, kkt_dual=kd)
    print(len(rebdates), "dates; nan in panel:", int(np.isnan(X.to_numpy()).sum()), file=sys.stderr)


if __name__ == "__main__":
    main()
