#!/usr/bin/env python3
"""Capture golden vectors from the PorQua reference (run in the build container only).

Imports ``/root/reference/src`` read-only (``sys.dont_write_bytecode``) with a *capturing*
``qpsolvers`` stub: the stub records the exact ``Problem(P, q, G, h, A, b, lb, ub)`` the
reference hands to ``qpsolvers.solve_problem`` (``src/qp_problems.py:192-214``) and
returns equal weights so the reference's own ``Backtest.run`` loop
(``src/backtest.py:201-224``) keeps going.  Outputs are small ``.npz`` fixtures under
``tests/golden/``; QP optima for them come from ``oracle.qp_ipm`` (the solver itself is
third-party and absent, see ``oracle/__init__.py``).

Data: ``data/msci_country_indices.csv`` and ``data/NDDLWI.csv`` are parsed here with
their real format (comma separated, ``dd-mm-YYYY``) because the reference loader expects
``sep=';'`` / ``%d/%m/%Y`` and raises on the shipped files (``src/data_loader.py:39-44``).

Usage:  python tools/capture_golden.py
"""
from __future__ import annotations

import os
import sys
import types
import warnings

import numpy as np
import pandas as pd

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
OUT = os.path.join(REPO, "tests", "golden")

sys.dont_write_bytecode = True
sys.path.insert(0, os.path.join(REF, "src"))
sys.path.insert(0, REPO)
warnings.simplefilter("ignore")

CAPTURED: list = []


class _StubProblem:
    def __init__(self, P, q, G=None, h=None, A=None, b=None, lb=None, ub=None):
        self.P, self.q, self.G, self.h, self.A, self.b, self.lb, self.ub = P, q, G, h, A, b, lb, ub


class _StubSolution:
    def __init__(self, n):
        self.found = True
        self.x = np.full(n, 1.0 / n)
        self.obj = None


def _solve_problem(problem, solver=None, initvals=None, verbose=False):
    CAPTURED.append(problem)
    return _StubSolution(len(problem.q))


_qps = types.ModuleType("qpsolvers")
_qps.Problem = _StubProblem
_qps.solve_problem = _solve_problem
sys.modules["qpsolvers"] = _qps

from backtest import Backtest, BacktestService  # noqa: E402  (reference)
from builders import (  # noqa: E402
    OptimizationItemBuilder, SelectionItemBuilder, bibfn_box_constraints, bibfn_bm_series,
    bibfn_budget_constraint, bibfn_return_series, bibfn_selection_data)
from constraints import Constraints  # noqa: E402
from covariance import Covariance  # noqa: E402
from optimization import LeastSquares, MeanVariance, QEQW  # noqa: E402

from oracle.qp_ipm import solve_qp  # noqa: E402


def load_msci():
    X = pd.read_csv(os.path.join(REF, "data", "msci_country_indices.csv"), index_col=0)
    X.index = pd.to_datetime(X.index, format="%d-%m-%Y")
    y = pd.read_csv(os.path.join(REF, "data", "NDDLWI.csv"), index_col=0)
    y.index = pd.to_datetime(y.index, format="%d-%m-%Y")
    return X.astype(float), y.astype(float)


def run_backtest(optimization, X, y, rebdates, width, box_kw):
    CAPTURED.clear()
    builders_sel = {"data": SelectionItemBuilder(bibfn=bibfn_selection_data)}
    builders_opt = {
        "return_series": OptimizationItemBuilder(bibfn=bibfn_return_series, width=width),
        "bm_series": OptimizationItemBuilder(bibfn=bibfn_bm_series, width=width),
        "budget_constraint": OptimizationItemBuilder(bibfn=bibfn_budget_constraint, budget=1),
        "box_constraints": OptimizationItemBuilder(bibfn=bibfn_box_constraints, **box_kw),
    }
    bs = BacktestService(data={"return_series": X, "bm_series": y},
                         selection_item_builders=builders_sel,
                         optimization_item_builders=builders_opt,
                         optimization=optimization, rebdates=rebdates, quiet=True)
    consts = []
    windows = []

    def append_fun(backtest, bs, rebalancing_date, what):
        consts.append(bs.optimization.objective.get("constant"))
        rs = bs.optimization_data["return_series"]
        windows.append((rs.index[0], rs.index[-1], len(rs)))

    bs.settings["append_fun"] = append_fun
    Backtest().run(bs)
    probs = list(CAPTURED)
    assert len(probs) == len(rebdates)
    return probs, consts, windows


def stack(probs, key):
    vals = [getattr(p, key) for p in probs]
    if any(v is None for v in vals):
        assert all(v is None for v in vals)
        return None
    return np.stack([np.asarray(v, dtype=float) for v in vals])


def golden_solutions(probs):
    xs, objs, kp, kd = [], [], [], []
    for p in probs:
        s = solve_qp(p.P, p.q, p.G, p.h, p.A, p.b, p.lb, p.ub)
        xs.append(s.x)
        objs.append(s.obj)
        kp.append(s.primal_residual())
        kd.append(s.dual_residual())
    return np.stack(xs), np.array(objs), np.array(kp), np.array(kd)


def days(idx):
    return np.asarray(pd.DatetimeIndex(idx).values.astype("datetime64[D]").astype(np.int64))


def main():
    os.makedirs(OUT, exist_ok=True)
    X, y = load_msci()
    dates = X.index
    np.savez_compressed(os.path.join(OUT, "msci_panel.npz"), dates=days(dates),
                        returns=X.to_numpy(), bm=y.to_numpy().reshape(-1),
                        columns=np.array(X.columns.tolist()))
    rebdates = dates[dates > "2010-01-01"][::21].strftime("%Y-%m-%d").tolist()
    width = 252

    # --- msci least-squares index tracking (src/optimization.py:198-229) -------------
    for tag, kw, box_kw in [
        ("msci_ls", {}, {}),
        ("msci_ls_l2", {"l2_penalty": 1e-3}, {"upper": 0.2}),
        ("msci_ls_log", {"log_transform": True}, {"upper": 0.3}),
    ]:
        opt = LeastSquares(solver_name="cvxopt", **kw)
        probs, consts, wins = run_backtest(opt, X, y, rebdates, width, box_kw)
        xs, objs, kp, kd = golden_solutions(probs)
        np.savez_compressed(
            os.path.join(OUT, f"{tag}.npz"), rebdates=np.array(rebdates), width=width,
            params=str(kw), box=str(box_kw),
            P=stack(probs, "P"), q=stack(probs, "q"), A=stack(probs, "A"), b=stack(probs, "b"),
            lb=stack(probs, "lb"), ub=stack(probs, "ub"),
            const=np.array(consts, dtype=float),
            win_first=days([w[0] for w in wins]), win_last=days([w[1] for w in wins]),
            win_len=np.array([w[2] for w in wins]),
            x=xs, obj=objs, kkt_primal=kp, kkt_dual=kd)
        print(tag, len(probs), "QPs, max KKT", kp.max(), kd.max())

    # --- msci mean-variance (src/optimization.py:157-177), Pearson + PD check --------
    for tag, cov_kw, ra in [("msci_mv", {}, 1.0),
                            ("msci_mv_shrink", {"method": "linear_shrinkage",
                                                "lambda_covmat_regularization": 0.1}, 3.0)]:
        opt = MeanVariance(covariance=Covariance(**cov_kw), solver_name="cvxopt",
                           risk_aversion=ra)
        probs, consts, wins = run_backtest(opt, X, y, rebdates, width, {"upper": 0.25})
        xs, objs, kp, kd = golden_solutions(probs)
        np.savez_compressed(
            os.path.join(OUT, f"{tag}.npz"), rebdates=np.array(rebdates), width=width,
            risk_aversion=ra, cov=str(cov_kw),
            P=stack(probs, "P"), q=stack(probs, "q"), A=stack(probs, "A"), b=stack(probs, "b"),
            lb=stack(probs, "lb"), ub=stack(probs, "ub"),
            win_first=days([w[0] for w in wins]), win_last=days([w[1] for w in wins]),
            win_len=np.array([w[2] for w in wins]),
            x=xs, obj=objs, kkt_primal=kp, kkt_dual=kd)
        print(tag, len(probs), "QPs, max KKT", kp.max(), kd.max())

    # --- QEQW (src/optimization.py:180-194) -----------------------------------------
    probs, _, _ = run_backtest(QEQW(solver_name="cvxopt"), X, y, rebdates[:5], width, {})
    xs, objs, kp, kd = golden_solutions(probs)
    np.savez_compressed(os.path.join(OUT, "msci_qeqw.npz"), P=stack(probs, "P"),
                        q=stack(probs, "q"), A=stack(probs, "A"), b=stack(probs, "b"),
                        lb=stack(probs, "lb"), ub=stack(probs, "ub"), x=xs, obj=objs)

    # --- Covariance.estimate on synthetic windows (src/covariance.py:40-84) ----------
    rng = np.random.default_rng(20240314)
    cases = {}
    for name, T, n, spec in [
        ("pearson_n_lt_T", 60, 40, {}),
        ("pearson_n_gt_T", 30, 50, {}),           # singular -> nearestPD fires
        ("pearson_nocheck", 30, 50, {"check_positive_definite": False}),
        ("shrink_0p1", 30, 50, {"method": "linear_shrinkage",
                                "lambda_covmat_regularization": 0.1}),
        ("shrink_neg", 60, 40, {"method": "linear_shrinkage",
                                "lambda_covmat_regularization": -1.0}),
        ("duv", 20, 12, {"method": "duv"}),
    ]:
        Xw = rng.normal(3e-4, 0.02, size=(T, n))
        df = pd.DataFrame(Xw, columns=[f"A{i}" for i in range(n)])
        est = Covariance(**spec).estimate(df)
        est = est.to_numpy() if hasattr(est, "to_numpy") else np.asarray(est)
        cases[f"{name}__X"] = Xw
        cases[f"{name}__cov"] = est
        cases[f"{name}__raw"] = df.cov().to_numpy()
        cases[f"{name}__spec"] = np.array(str(spec))
    np.savez_compressed(os.path.join(OUT, "cov_cases.npz"), **cases)

    # --- Constraints.to_GhAb (src/constraints.py:114-167; test shapes test:28-58) ----
    universe = X.columns
    r = np.random.default_rng(7)
    c = Constraints(selection=universe)
    c.add_budget()
    c.add_box("LongOnly")
    a1, a2, a3 = r.random(universe.size), r.random(universe.size), r.random(universe.size)
    c.add_linear(None, pd.Series(a1, index=universe), "<=", 1)
    c.add_linear(None, pd.Series(a2, index=universe), ">=", -1)
    c.add_linear(None, pd.Series(a3, index=universe), "=", 0.5)
    sub = universe[: universe.size // 2]
    blk = r.random((3, sub.size))
    c.add_linear(pd.DataFrame(blk, columns=sub), None, pd.Series(np.repeat("=", 3)),
                 pd.Series(np.ones(3)), None)
    g0, g1 = c.to_GhAb(), c.to_GhAb(True)
    c2 = Constraints(selection=universe)
    c2.add_budget()
    c2.add_box("LongShort")
    c2.add_linear(None, pd.Series(a3, index=universe), "=", 0.5)
    c2.add_linear(pd.DataFrame(blk, columns=sub), None, pd.Series(np.repeat("=", 3)),
                  pd.Series(np.ones(3)), None)
    g2 = c2.to_GhAb(True)   # all-'=' linear rows: box rows appear twice (reference quirk)
    np.savez_compressed(os.path.join(OUT, "ghab.npz"), a1=a1, a2=a2, a3=a3, blk=blk,
                        G0=g0["G"], h0=g0["h"], A0=g0["A"], b0=g0["b"],
                        G1=g1["G"], h1=g1["h"], A1=g1["A"], b1=g1["b"],
                        G2=g2["G"], h2=g2["h"], A2=g2["A"], b2=g2["b"])
    print("ghab shapes", g0["G"].shape, g0["A"].shape, g1["G"].shape, g2["G"].shape)
    print("wrote", sorted(os.listdir(OUT)))


if __name__ == "__main__":
    main()
