#!/usr/bin/env python3
"""Capture golden vectors for the l1 row from the PorQua reference
(run in the build container only).

Runs the reference's own ``Backtest.run`` on the msci data through the capturing
``qpsolvers`` stub of ``tools/capture_golden.py`` with an extra optimization item builder
that adds an l1 term, so the captured problems are exactly what
``Optimization.model_qpsolvers`` (src/optimization.py:118-143) produces after
``linearize_turnover_objective`` / ``linearize_turnover_constraint``
(src/qp_problems.py:40-77, 120-157):

* ``msci_l1_tc``: MeanVariance (linear shrinkage 0.1) with ``transaction_cost = 0.002``
  around ``params['x0']`` = a fixed non-uniform portfolio;
* ``msci_l1_to``: LeastSquares (l2_penalty 1e-3) with ``add_l1('turnover', rhs=0.3, x0)``;
* ``msci_l1_lev``: MeanVariance (risk aversion 5) on a long/short box [-0.1, 0.3] with
  ``add_l1('leverage', rhs=1.5)`` (``linearize_leverage_constraint``, src/qp_problems.py:79-118).

Golden optima of the linearised problems come from ``oracle.qp_ipm`` (KKT-certified).
Usage:  python tools/capture_l1.py
"""
from __future__ import annotations

import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import capture_golden as cg  # noqa: E402  (sets up the stub and the reference imports)

from covariance import Covariance  # noqa: E402  (reference)
from optimization import LeastSquares, MeanVariance  # noqa: E402  (reference)


def main():
    X, y = cg.load_msci()
    n = X.shape[1]
    rng = np.random.default_rng(5)
    w0 = rng.dirichlet(np.ones(n))
    x0 = dict(zip(X.columns, w0))
    dates = X.index
    rebdates = [str(d.date()) for d in dates[dates > "2010-01-01"][::21][:24]]
    width = 252
    out = {}

    def add_turnover(bs, rebdate, **kw):
        bs.optimization.constraints.add_l1("turnover", rhs=kw["rhs"], x0=kw["x0"])

    def add_leverage(bs, rebdate, **kw):
        bs.optimization.constraints.add_l1("leverage", rhs=kw["rhs"])

    cases = {
        "tc": (MeanVariance(covariance=Covariance(method="linear_shrinkage", lambda_covmat_regularization=0.1),
                            solver_name="cvxopt", transaction_cost=0.002, x0=x0), None),
        "to": (LeastSquares(l2_penalty=1e-3, solver_name="cvxopt"),
               cg.OptimizationItemBuilder(bibfn=add_turnover, rhs=0.3, x0=x0)),
        "lev": (MeanVariance(covariance=Covariance(method="linear_shrinkage", lambda_covmat_regularization=0.1),
                             solver_name="cvxopt", risk_aversion=5.0),
                cg.OptimizationItemBuilder(bibfn=add_leverage, rhs=1.5)),
    }
    box = {"tc": {"box_type": "LongOnly"}, "to": {"box_type": "LongOnly"},
           "lev": {"box_type": "LongShort", "lower": -0.1, "upper": 0.3}}
    orig_run = cg.run_backtest
    for tag, (opt, extra) in cases.items():
        if extra is not None:
            def run_backtest(optimization, X_, y_, reb, w, box_kw, _extra=extra):
                # the same driver as capture_golden.run_backtest plus one more builder
                cg.CAPTURED.clear()
                builders_sel = {"data": cg.SelectionItemBuilder(bibfn=cg.bibfn_selection_data)}
                builders_opt = {
                    "return_series": cg.OptimizationItemBuilder(bibfn=cg.bibfn_return_series, width=w),
                    "bm_series": cg.OptimizationItemBuilder(bibfn=cg.bibfn_bm_series, width=w),
                    "budget_constraint": cg.OptimizationItemBuilder(bibfn=cg.bibfn_budget_constraint, budget=1),
                    "box_constraints": cg.OptimizationItemBuilder(bibfn=cg.bibfn_box_constraints, **box_kw),
                    "l1": _extra,
                }
                bs = cg.BacktestService(data={"return_series": X_, "bm_series": y_},
                                        selection_item_builders=builders_sel,
                                        optimization_item_builders=builders_opt,
                                        optimization=optimization, rebdates=reb, quiet=True)
                cg.Backtest().run(bs)
                return list(cg.CAPTURED), None, None
            probs, _, _ = run_backtest(opt, X, y, rebdates, width, box[tag])
        else:
            probs, _, _ = orig_run(opt, X, y, rebdates, width, box[tag])
        if tag == "lev":
            # reference defect: linearize_leverage_constraint pads a 0-d b (np.pad returns it
            # unchanged), so A has 1 + N rows and b one entry and qpsolvers rejects the
            # problem; the intended right-hand side [b; 0] is used for the golden optimum
            for p in probs:
                p.b = np.concatenate([np.atleast_1d(p.b), np.zeros(p.A.shape[0] - np.atleast_1d(p.b).size)])
        xs, objs, kp, kd = cg.golden_solutions(probs)
        rec = {k: cg.stack(probs, k) for k in ("P", "q", "G", "h", "A", "b", "lb", "ub")}
        rec = {k: v for k, v in rec.items() if v is not None}
        np.savez_compressed(os.path.join(cg.OUT, f"msci_l1_{tag}.npz"), rebdates=np.array(rebdates),
                            x0=w0, x=xs, obj=objs, kkt_primal=kp, kkt_dual=kd, **rec)
        out[tag] = {k: v.shape for k, v in rec.items()}
        print(tag, out[tag], "kkt", float(kp.max()), float(kd.max()))


if __name__ == "__main__":
    main()
