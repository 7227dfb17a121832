"""Reference-API parity on the device: the same calls the reference's tests and
quick-and-dirty script make (test/tests_quadratic_program.py, src/_quick_and_dirty_
interactive_testing.py), with solver_name='mi355x'."""
import numpy as np
import pandas as pd
import pytest

from oracle import ref_pipeline as rp
from porqua_amd.backtest import Backtest, BacktestService
from porqua_amd.builders import (OptimizationItemBuilder, SelectionItemBuilder, bibfn_box_constraints,
                                 bibfn_bm_series, bibfn_budget_constraint, bibfn_return_series,
                                 bibfn_selection_data)
from porqua_amd.constraints import Constraints
from porqua_amd.covariance import Covariance
from porqua_amd.helper_functions import isPD, nearestPD
from porqua_amd.mean_estimation import MeanEstimator
from porqua_amd.optimization import LeastSquares, MeanVariance, QEQW, WeightedLeastSquares
from porqua_amd.optimization_data import OptimizationData
from tests.conftest import load_golden

pytestmark = pytest.mark.gpu


def msci():
    g = load_golden("msci_panel")
    idx = pd.DatetimeIndex(g["dates"].astype("datetime64[D]"))
    cols = [str(c) for c in g["columns"]]
    return pd.DataFrame(g["returns"], index=idx, columns=cols), pd.DataFrame({"NDDLWI": g["bm"]}, index=idx)


def test_least_squares_reference_test(device):
    """TestLeastSquares (test:61-126): found, and solution.obj == objective_value(x, False)."""
    X, y = msci()
    opt = LeastSquares(solver_name="mi355x", sparse=True)
    opt.params["l2_penalty"] = 0
    c = Constraints(selection=X.columns)
    c.add_budget()
    c.add_box("LongOnly")
    opt.constraints = c
    opt.set_objective(OptimizationData(return_series=X, bm_series=y, align=True))
    opt.model_qpsolvers()
    opt.model.solve()
    sol = opt.model["solution"]
    assert sol.found
    assert sol.obj == pytest.approx(opt.model.objective_value(sol.x, False), abs=1e-7)
    assert sol.primal_residual() < 1e-9 and sol.dual_residual() < 1e-9
    from oracle.qp_ipm import solve_qp
    m = opt.model
    ref = solve_qp(m["P"], m["q"], A=m["A"], b=np.atleast_1d(m["b"]), lb=m["lb"], ub=m["ub"])
    assert np.abs(sol.x - ref.x).max() < 1e-5
    assert abs(sol.obj - ref.obj) <= 1e-6 * abs(ref.obj)


def test_covariance_estimate_matches_reference_golden(device):
    g = load_golden("cov_cases")
    for name in ["pearson_n_lt_T", "pearson_n_gt_T", "shrink_0p1", "shrink_neg"]:
        X = pd.DataFrame(g[f"{name}__X"])
        spec = eval(str(g[f"{name}__spec"]))
        S = Covariance(**spec).estimate(X)
        S = S.to_numpy() if hasattr(S, "to_numpy") else S
        ref = g[f"{name}__cov"]
        assert np.linalg.norm(S - ref) <= 1e-12 * np.linalg.norm(ref), name
    S = Covariance(method="duv").estimate(pd.DataFrame(g["duv__X"]))
    assert np.array_equal(S, g["duv__cov"])


def test_pd_check_and_repair_on_device(device):
    g = load_golden("cov_cases")
    raw = g["pearson_n_gt_T__raw"]
    assert not isPD(raw) and isPD(g["pearson_n_lt_T__raw"])
    rep = nearestPD(raw)
    assert isPD(rep) and np.linalg.norm(rep - raw) <= 1e-12 * np.linalg.norm(raw)


def test_geometric_mean(device):
    X = pd.DataFrame(np.random.default_rng(3).normal(3e-4, 0.02, (120, 9)))
    for kw in [{}, {"n_mom": 60, "n_rev": 5}, {"scalefactor": 252}]:
        mu = MeanEstimator(**kw).estimate(X).to_numpy()
        ref = rp.mean_geometric(X.to_numpy(), kw.get("n_mom"), kw.get("n_rev"), kw.get("scalefactor"))
        assert np.allclose(mu, ref, rtol=1e-12, atol=1e-15)


def _service(opt, X, y, rebdates, box_kw, width=252):
    return BacktestService(
        data={"return_series": X, "bm_series": y},
        selection_item_builders={"data": SelectionItemBuilder(bibfn=bibfn_selection_data)},
        optimization_item_builders={
            "return_series": OptimizationItemBuilder(bibfn=bibfn_return_series, width=width),
            "bm_series": OptimizationItemBuilder(bibfn=bibfn_bm_series, width=width),
            "budget_constraint": OptimizationItemBuilder(bibfn=bibfn_budget_constraint, budget=1),
            "box_constraints": OptimizationItemBuilder(bibfn=bibfn_box_constraints, **box_kw)},
        optimization=opt, rebdates=rebdates, quiet=True)


@pytest.mark.parametrize("tag,make,box", [
    ("msci_ls", lambda: LeastSquares(solver_name="mi355x"), {}),
    ("msci_ls_l2", lambda: LeastSquares(solver_name="mi355x", l2_penalty=1e-3), {"upper": 0.2}),
    ("msci_ls_log", lambda: LeastSquares(solver_name="mi355x", log_transform=True), {"upper": 0.3}),
    ("msci_mv", lambda: MeanVariance(solver_name="mi355x"), {"upper": 0.25}),
    ("msci_mv_shrink", lambda: MeanVariance(covariance=Covariance(method="linear_shrinkage",
                                                                  lambda_covmat_regularization=0.1),
                                            solver_name="mi355x", risk_aversion=3.0), {"upper": 0.25}),
    ("msci_wls", lambda: WeightedLeastSquares(solver_name="mi355x", tau=252), {}),
    ("msci_wls_log", lambda: WeightedLeastSquares(solver_name="mi355x", tau=21, log_transform=True),
     {"upper": 0.3}),
])
def test_backtest_batched_matches_golden(device, tag, make, box):
    X, y = msci()
    g = load_golden(tag)
    rebdates = [str(d) for d in g["rebdates"]]
    bt = Backtest()
    bt.run(_service(make(), X, y, rebdates, box))
    assert bt.stats["solved"] == len(rebdates)          # the batched path ran
    W = bt.strategy.get_weights_df().to_numpy(dtype=float)
    assert W.shape == g["x"].shape
    assert np.abs(W - g["x"]).max() < 1e-5
    obj = np.array([0.5 * w @ P @ w + q.reshape(-1) @ w for w, P, q in zip(W, g["P"], g["q"])])
    assert np.max(np.abs(obj - g["obj"]) / np.maximum(np.abs(g["obj"]), 1e-12)) < 1e-6


def test_backtest_serial_equals_batched(device):
    X, y = msci()
    g = load_golden("msci_mv")
    rebdates = [str(d) for d in g["rebdates"][:12]]
    bt1 = Backtest()
    bt1.run(_service(MeanVariance(solver_name="mi355x"), X, y, rebdates, {"upper": 0.25}))
    bs = _service(MeanVariance(solver_name="mi355x"), X, y, rebdates, {"upper": 0.25})
    bs.settings["batched"] = False
    bt2 = Backtest()
    bt2.run(bs)
    W1 = bt1.strategy.get_weights_df().to_numpy(dtype=float)
    W2 = bt2.strategy.get_weights_df().to_numpy(dtype=float)
    assert np.abs(W1 - W2).max() < 1e-7
    assert np.abs(W1 - g["x"][:12]).max() < 1e-5


def test_qeqw_backtest(device):
    X, y = msci()
    rebdates = [str(d.date()) for d in X.index[400:1400:200]]
    bt = Backtest()
    bt.run(_service(QEQW(solver_name="mi355x"), X, y, rebdates, {}))
    W = bt.strategy.get_weights_df().to_numpy(dtype=float)
    assert np.allclose(W, 1.0 / 24, atol=1e-9)


def _synthetic(n, D, seed):
    from porqua_amd.synthetic import factor_panel
    dates, R, y, _ = factor_panel(D, n, seed=seed)
    idx = pd.DatetimeIndex(dates)
    return (pd.DataFrame(R, index=idx, columns=[f"a{i}" for i in range(n)]),
            pd.DataFrame({"bm": y}, index=idx))


def test_wls_serial_equals_batched(device):
    """WeightedLeastSquares: the per-date set_objective (weighted Gram on the device) and the
    batched row-scaled panel (one scaled panel + a per-date scalar) give the same weights."""
    X, y = msci()
    g = load_golden("msci_wls_log")
    rebdates = [str(d) for d in g["rebdates"][:10]]
    W = []
    for batched in (True, False):
        bs = _service(WeightedLeastSquares(solver_name="mi355x", tau=21, log_transform=True), X, y,
                      rebdates, {"upper": 0.3})
        bs.settings["batched"] = batched
        bt = Backtest()
        bt.run(bs)
        W.append(bt.strategy.get_weights_df().to_numpy(dtype=float))
    assert np.abs(W[0] - W[1]).max() < 1e-7
    assert np.abs(W[0] - g["x"][:10]).max() < 1e-5


@pytest.mark.parametrize("kind", ["mv", "mv_shrink", "ls", "wls"])
def test_backtest_lowrank_path_matches_oracle(device, kind):
    """Backtest.run with n > width: sliding K1 (lower triangle), Woodbury factor, grouped
    ADMM and window-form polish; weights checked against the oracle IPM per date."""
    from oracle.qp_ipm import solve_qp
    n, D, width = 300, 160, 60
    X, y = _synthetic(n, D, seed=11)
    rebdates = [str(d.date()) for d in X.index[width + 5:width + 5 + 24]]
    make = {"mv": lambda: MeanVariance(solver_name="mi355x"),
            "mv_shrink": lambda: MeanVariance(covariance=Covariance(method="linear_shrinkage",
                                                                    lambda_covmat_regularization=0.1),
                                              solver_name="mi355x", risk_aversion=2.0),
            "ls": lambda: LeastSquares(solver_name="mi355x"),
            "wls": lambda: WeightedLeastSquares(solver_name="mi355x", tau=30)}[kind]
    bt = Backtest()
    bt.run(_service(make(), X, y, rebdates, {"upper": 0.1}, width=width))
    assert bt.stats["solved"] == len(rebdates) and bt.stats["path"] == "lowrank"
    W = bt.strategy.get_weights_df().to_numpy(dtype=float)
    Xv, yv = X.to_numpy(), y.to_numpy()[:, 0]
    for i in (0, 11, len(rebdates) - 1):
        e = X.index.get_loc(pd.Timestamp(rebdates[i]))
        Xw, yw = Xv[e - width + 1:e + 1], yv[e - width + 1:e + 1]
        if kind == "ls":
            P, q = 2 * Xw.T @ Xw, -2 * Xw.T @ yw
        elif kind == "wls":
            P, q, _ = rp.objective_wls(Xw, yw, 30)
        else:
            S = rp.cov_pearson(Xw)
            ra = 2.0 if kind == "mv_shrink" else 1.0
            if kind == "mv_shrink":
                S = S + 0.1 * np.mean(np.diag(S)) * np.eye(n)
            P, q = 2 * ra * S, -rp.mean_geometric(Xw, None, None, None)
        o = solve_qp(P, q, A=np.ones((1, n)), b=np.ones(1), lb=np.zeros(n), ub=np.full(n, 0.1))
        obj = 0.5 * W[i] @ P @ W[i] + q @ W[i]
        assert abs(obj - o.obj) <= 1e-6 * max(abs(o.obj), 1e-12), (kind, i, obj, o.obj)
        if kind not in ("ls", "wls"):   # LS: rank(X'X) <= width < n, the optimum is a face (compare value)
            assert np.abs(W[i] - o.x).max() < 1e-5, (kind, i, np.abs(W[i] - o.x).max())
        assert abs(W[i].sum() - 1) < 1e-7 and W[i].min() > -1e-7 and W[i].max() < 0.1 + 1e-7


def test_backtests_keep_their_weights_across_runs(device):
    """The batched path's page-locked weight panel is reused only when no Portfolio of the
    previous backtest still views it, and its lazy Portfolio objects are built while the
    device solves: a second backtest (other risk aversion) must not change the first one's
    weights, read before or after it, and a repeated run gives the same weights."""
    n, D, width = 300, 160, 60
    X, y = _synthetic(n, D, seed=12)
    rebdates = [str(d.date()) for d in X.index[width + 5:width + 5 + 24]]
    bt1 = Backtest()
    bt1.run(_service(MeanVariance(solver_name="mi355x"), X, y, rebdates, {"upper": 0.1}, width=width))
    first_read = dict(bt1.strategy.portfolios[0].weights)        # one portfolio read early
    bt2 = Backtest()
    bt2.run(_service(MeanVariance(solver_name="mi355x", risk_aversion=50.0), X, y, rebdates, {"upper": 0.1},
                     width=width))
    W1 = bt1.strategy.get_weights_df().to_numpy(dtype=float)
    W2 = bt2.strategy.get_weights_df().to_numpy(dtype=float)
    assert np.abs(W1 - W2).max() > 1e-3                          # different problems
    assert bt1.strategy.portfolios[0].weights == first_read
    del bt2
    bt3 = Backtest()                                              # reuses bt2's released panel
    bt3.run(_service(MeanVariance(solver_name="mi355x"), X, y, rebdates, {"upper": 0.1}, width=width))
    W3 = bt3.strategy.get_weights_df().to_numpy(dtype=float)
    assert np.abs(W3 - W1).max() < 1e-9
    assert np.array_equal(bt1.strategy.get_weights_df().to_numpy(dtype=float), W1)


def test_nearest_pd_higham_on_device_matches_reference(device):
    """nearestPD (src/helper_functions.py:29-58) on the device: the projection and the
    eigenvalue shifts on the hand-written block-Jacobi eigensolver, the PD tests on K2.  Checked against the
    reference's repaired covariance (golden) and against the oracle restatement on
    genuinely indefinite matrices, where the projection and several shifts act."""
    g = load_golden("cov_cases")
    rep = nearestPD(g["pearson_n_gt_T__raw"])
    ref = g["pearson_n_gt_T__cov"]
    assert isPD(rep) and np.linalg.norm(rep - ref) <= 1e-12 * np.linalg.norm(ref)
    rng = np.random.default_rng(4)
    M = rng.normal(size=(3, 60, 60))
    A = M + np.swapaxes(M, 1, 2) - 2.0 * np.eye(60)[None]          # indefinite
    out = nearestPD(A)
    for i in range(3):
        o = rp.nearest_pd(A[i])
        assert isPD(out[i])
        assert np.linalg.norm(out[i] - o) <= 1e-10 * np.linalg.norm(o), np.linalg.norm(out[i] - o)
