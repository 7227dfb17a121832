"""BASELINE.json configs[0..1]: SPTR index replication on the usa panel, monthly rebalance,
least-squares tracking -- the reference's example/backtest.ipynb run (LeastSquares, budget +
LongOnly box, width 252, rebdates[::21]) through the drop-in API with solver_name='mi355x'
(config 2: all rebalance dates batched on the device), against the CPU reference restated by
the oracle (config 1; tools/capture_config1.py -> tests/golden/config1_oracle.npz).

The panel is porqua_amd.synthetic.usa_panel on the real SPTR calendar (tests/golden/sptr.npz,
captured from the reference's data/SPTR.csv by tools/capture_sptr.py); usa_returns itself is
absent from the reference tree.  494 assets > 252 rows: the Gram is rank-deficient, but each
optimum has fewer free weights than rows, so it is unique and the weights are compared."""
import numpy as np
import pandas as pd
import pytest

from porqua_amd.backtest import Backtest, BacktestService
from porqua_amd.builders import (OptimizationItemBuilder, SelectionItemBuilder, bibfn_box_constraints,
                                 bibfn_bm_series, bibfn_budget_constraint, bibfn_return_series,
                                 bibfn_selection_data)
from porqua_amd.optimization import LeastSquares
from porqua_amd.synthetic import usa_panel
from tests.conftest import load_golden

pytestmark = pytest.mark.gpu


def usa_data():
    g = load_golden("sptr")
    days, R, y = usa_panel(g["days"], g["returns"])
    idx = pd.DatetimeIndex(days)
    X = pd.DataFrame(R, index=idx, columns=[f"u{i:03d}" for i in range(R.shape[1])])
    return X, pd.DataFrame({"SPTR": y}, index=idx)


def service(X, y, rebdates, width=252, params=None):
    return BacktestService(
        data={"return_series": X, "bm_series": y},
        selection_item_builders={"data": SelectionItemBuilder(bibfn=bibfn_selection_data)},
        optimization_item_builders={
            "return_series": OptimizationItemBuilder(bibfn=bibfn_return_series, width=width),
            "bm_series": OptimizationItemBuilder(bibfn=bibfn_bm_series, width=width, align=True),
            "budget_constraint": OptimizationItemBuilder(bibfn=bibfn_budget_constraint, budget=1),
            "box_constraints": OptimizationItemBuilder(bibfn=bibfn_box_constraints, box_type="LongOnly")},
        optimization=LeastSquares(solver_name="mi355x", **(params or {})), rebdates=rebdates, quiet=True)


def test_config2_sptr_replication_matches_config1_oracle(device):
    X, y = usa_data()
    gold = load_golden("config1_oracle")
    reb = gold["rebdates"].astype("datetime64[D]")
    d = X.index.values.astype("datetime64[D]")
    assert np.array_equal(reb, d[d > np.datetime64(str(gold["start"]))][::int(gold["stride"])])
    rebdates = [str(r) for r in reb]
    assert len(rebdates) == 13 and X.shape == (4795, 494)
    bt = Backtest()
    bt.run(service(X, y, rebdates))
    assert bt.stats["solved"] == len(rebdates)            # the batched device path ran
    W = bt.strategy.get_weights_df().to_numpy(dtype=float)
    Xv, yv = X.to_numpy(), y.to_numpy()[:, 0]
    T = int(gold["width"])
    for i, rd in enumerate(rebdates):
        e = X.index.get_loc(pd.Timestamp(rd))
        Xw, yw = Xv[e - T + 1:e + 1], yv[e - T + 1:e + 1]
        P, q = 2 * Xw.T @ Xw, -2 * Xw.T @ yw
        w = W[i]
        assert abs(w.sum() - 1) <= 1e-7 and w.min() >= -1e-7 and w.max() <= 1 + 1e-7
        obj = 0.5 * w @ P @ w + q @ w
        assert abs(obj - gold["obj"][i]) <= 1e-6 * abs(gold["obj"][i]), (rd, obj, gold["obj"][i])
        if (gold["x"][i] > 1e-8).sum() < T:                 # fewer free weights than rows: unique
            assert np.abs(w - gold["x"][i]).max() <= 1e-5, (rd, np.abs(w - gold["x"][i]).max())


def test_config2_daily_sptr_replication_all_dates(device):
    """Every date of the last year of the usa panel rebalanced (252 daily LS tracking QPs in
    one batch): all solved, feasible, and the tracking objective matches the oracle on a
    sample of dates."""
    from oracle.qp_ipm import solve_qp
    X, y = usa_data()
    rebdates = [str(r.date()) for r in X.index[-252:]]
    bt = Backtest()
    bt.run(service(X, y, rebdates))
    assert bt.stats["solved"] == len(rebdates)
    W = bt.strategy.get_weights_df().to_numpy(dtype=float)
    assert np.abs(W.sum(1) - 1).max() <= 1e-7 and W.min() >= -1e-7
    Xv, yv = X.to_numpy(), y.to_numpy()[:, 0]
    n = Xv.shape[1]
    for i in (0, 125, 251):
        e = X.index.get_loc(pd.Timestamp(rebdates[i]))
        Xw, yw = Xv[e - 251:e + 1], yv[e - 251:e + 1]
        P, q = 2 * Xw.T @ Xw, -2 * Xw.T @ yw
        o = solve_qp(P, q, A=np.ones((1, n)), b=np.ones(1), lb=np.zeros(n), ub=np.ones(n))
        obj = 0.5 * W[i] @ P @ W[i] + q @ W[i]
        assert abs(obj - o.obj) <= 1e-6 * abs(o.obj)
