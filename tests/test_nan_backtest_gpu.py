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
