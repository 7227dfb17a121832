#!/usr/bin/env python3
"""Capture golden vectors for LAD from the PorQua reference (run in
the build container only).

Runs the reference's own ``Backtest.run`` on the msci data through the capturing
``qpsolvers`` stub of ``tools/capture_golden.py``: ``LAD.solve`` (src/optimization.py:286-294)
calls ``model_qpsolvers`` (:296-345), whose QuadraticProgram reaches the stub, so the
captured problems are exactly the reference's LP (P = 0, A_tilde = [A; X I -I],
b_tilde = [b; y], lb / ub padded for u, v).  ``msci_lad``: the defaults (use_level, use_log),
long-only box; ``msci_lad_ret``: use_level = False (returns), box [0, 0.3].

Optima come from scipy's HiGHS (``oracle/lad.py``); the LP optimum value is unique.
Usage:  python tools/capture_lad.py
"""
from __future__ import annotations

import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import capture_golden as cg  # noqa: E402  (sets up the stub and the reference imports)

from optimization import LAD  # noqa: E402  (reference)

from oracle.lad import solve_lp  # noqa: E402


def main():
    X, y = cg.load_msci()
    dates = X.index
    rebdates = dates[dates > "2010-01-01"][::21].strftime("%Y-%m-%d").tolist()[:24]
    width = 252
    for tag, kw, box_kw in [("msci_lad", {}, {}),
                            ("msci_lad_ret", {"use_level": False}, {"upper": 0.3})]:
        opt = LAD(solver_name="cvxopt", **kw)
        probs, _, wins = cg.run_backtest(opt, X, y, rebdates, width, box_kw)
        objs, xs = [], []
        for p in probs:
            s = solve_lp(p.q, p.A, np.asarray(p.b).reshape(-1), p.lb, p.ub, p.G, p.h)
            objs.append(s.fun)
            xs.append(s.x)
        np.savez_compressed(
            os.path.join(cg.OUT, f"{tag}.npz"), rebdates=np.array(rebdates), width=width,
            params=str(kw), box=str(box_kw),
            q=cg.stack(probs, "q"), A=cg.stack(probs, "A"), b=np.stack([np.asarray(p.b).reshape(-1) for p in probs]),
            lb=cg.stack(probs, "lb"), ub=cg.stack(probs, "ub"),
            P_absmax=np.array([np.abs(p.P).max() for p in probs]),
            win_len=np.array([w[2] for w in wins]), obj=np.array(objs), x=np.stack(xs))
        print(tag, len(probs), "LPs, obj range", min(objs), max(objs))


if __name__ == "__main__":
    main()
