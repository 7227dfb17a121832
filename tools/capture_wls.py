#!/usr/bin/env python3
"""Capture golden vectors for WeightedLeastSquares from the PorQua
reference (run in the build container only).

Runs the reference's own ``Backtest.run`` on the msci data through the capturing
``qpsolvers`` stub of ``tools/capture_golden.py``, so the captured problems are exactly what
``WeightedLeastSquares.set_objective`` (src/optimization.py:232-256) and
``Optimization.model_qpsolvers`` (src/optimization.py:91-143) produce:

* ``msci_wls``: tau = 252 (the reference's own use, src/_quick_and_dirty_interactive_testing.py:159-162),
  long-only box [0, 1];
* ``msci_wls_log``: tau = 21 with ``log_transform``, box [0, 0.3].

Golden optima come from ``oracle.qp_ipm`` (KKT-certified).
Usage:  python tools/capture_wls.py
"""
from __future__ import annotations

import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import capture_golden as cg  # noqa: E402  (sets up the stub and the reference imports)

from optimization import WeightedLeastSquares  # noqa: E402  (reference)


def main():
    X, y = cg.load_msci()
    dates = X.index
    rebdates = dates[dates > "2010-01-01"][::21].strftime("%Y-%m-%d").tolist()[:40]
    width = 252
    for tag, kw, box_kw in [("msci_wls", {"tau": 252}, {}),
                            ("msci_wls_log", {"tau": 21, "log_transform": True}, {"upper": 0.3})]:
        opt = WeightedLeastSquares(solver_name="cvxopt", **kw)
        probs, consts, wins = cg.run_backtest(opt, X, y, rebdates, width, box_kw)
        xs, objs, kp, kd = cg.golden_solutions(probs)
        np.savez_compressed(
            os.path.join(cg.OUT, f"{tag}.npz"), rebdates=np.array(rebdates), width=width,
            params=str(kw), box=str(box_kw),
            P=cg.stack(probs, "P"), q=cg.stack(probs, "q"), A=cg.stack(probs, "A"), b=cg.stack(probs, "b"),
            lb=cg.stack(probs, "lb"), ub=cg.stack(probs, "ub"),
            const=np.array(consts, dtype=float),
            win_first=cg.days([w[0] for w in wins]), win_last=cg.days([w[1] for w in wins]),
            win_len=np.array([w[2] for w in wins]),
            x=xs, obj=objs, kkt_primal=kp, kkt_dual=kd)
        print(tag, len(probs), "QPs, max KKT", kp.max(), kd.max())


if __name__ == "__main__":
    main()
