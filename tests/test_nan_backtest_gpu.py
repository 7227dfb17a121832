"""Mean-variance backtest on a panel with missing values (assets entering late, leaving
early, holes) through Backtest.run(solver_name='mi355x'): the batched device path (pairwise-
complete covariance for all dates in one launch, PD check / nearestPD repair of the dates that
need it, skipna geometric means) against the reference's own P, q per date and the oracle's
optimum (tools/capture_mv_nan.py -> tests/golden/msci_mv_nan.npz), and against the serial
per-date path."""
import numpy as np
import pandas as pd
import pytest

from porqua_amd.backtest import Backtest
from porqua_amd.optimization import MeanVariance
from tests.conftest import load_golden
from tests.test_api_gpu import _service, msci

pytestmark = pytest.mark.gpu


def nan_panel():
    X, y = msci()
    g = load_golden("msci_mv_nan")
    V = X.to_numpy().copy()
    V[g["nan_rc"][:, 0], g["nan_rc"][:, 1]] = np.nan
    return pd.DataFrame(V, index=X.index, columns=X.columns), y, g


def test_mean_variance_backtest_with_missing_values_matches_reference(device):
    X, y, g = nan_panel()
    rebdates = [str(d) for d in g["rebdates"]]
    bt = Backtest()
    bt.run(_service(MeanVariance(solver_name="mi355x"), X, y, rebdates, {"upper": 0.25}))
    assert bt.stats["solved"] == len(rebdates) and bt.stats["path"] == "dense"   # batched
    W = bt.strategy.get_weights_df().to_numpy(dtype=float)
    assert np.abs(W - g["x"]).max() < 1e-5
    obj = np.array([0.5 * w @ P @ w + q @ w for w, P, q in zip(W, g["P"], g["q"])])
    assert np.max(np.abs(obj - g["obj"]) / np.maximum(np.abs(g["obj"]), 1e-12)) < 1e-6


def test_missing_values_serial_equals_batched(device):
    X, y, g = nan_panel()
    rebdates = [str(d) for d in g["rebdates"][:10]]
    W = []
    for batched in (True, False):
        bs = _service(MeanVariance(solver_name="mi355x"), X, y, rebdates, {"upper": 0.25})
        bs.settings["batched"] = batched
        bt = Backtest()
        bt.run(bs)
        W.append(bt.strategy.get_weights_df().to_numpy(dtype=float))
    assert np.abs(W[0] - W[1]).max() < 1e-7
    assert np.abs(W[0] - g["x"][:10]).max() < 1e-5


def test_missing_values_at_config3_scale(device):
    """the batched NaN path at n = 1000 over 600 daily dates (config 3's panel with
    2 % holes and 40 late-listed assets): every date solved in one batched run with the PD
    check / repair on the device (no (B, n, n) host copies), and the serial per-date path
    agreeing on sampled dates."""
    from porqua_amd.synthetic import factor_panel
    n, T, D = 1000, 252, 600
    dates, R, yv, _ = factor_panel(T - 1 + D, n)
    rng = np.random.default_rng(7)
    R = R.copy()
    R[rng.random(R.shape) < 0.02] = np.nan
    R[: T // 2, :40] = np.nan                                  # listed half a window late
    idx = pd.DatetimeIndex(dates)
    X = pd.DataFrame(R, index=idx, columns=[f"a{i}" for i in range(n)])
    y = pd.DataFrame({"bm": yv}, index=idx)
    rebdates = [str(d.date()) for d in idx[T - 1:]]
    bt = Backtest()
    bt.run(_service(MeanVariance(solver_name="mi355x"), X, y, rebdates, {"upper": 0.1}))
    assert bt.stats["solved"] == len(rebdates)
    W = bt.strategy.get_weights_df().to_numpy(dtype=float)
    assert np.all(np.isfinite(W)) and np.abs(W.sum(1) - 1).max() < 1e-9 and W.min() > -1e-9
    sample = [0, len(rebdates) // 2, len(rebdates) - 1]
    bs = _service(MeanVariance(solver_name="mi355x"), X, y, [rebdates[i] for i in sample], {"upper": 0.1})
    bs.settings["batched"] = False
    bt2 = Backtest()
    bt2.run(bs)
    W2 = bt2.strategy.get_weights_df().to_numpy(dtype=float)
    assert np.abs(W[sample] - W2).max() < 1e-6, np.abs(W[sample] - W2).max()
