"""Strategy simulation row: Strategy.simulate / Portfolio.turnover
(src/portfolio.py:111-123, 209-296).

* CPU: the numpy oracle (oracle/simulate.py) against the golden vectors captured from the
  reference's own portfolio.py (tests/golden/msci_simulate.npz, tools/capture_simulate.py);
  the host staging of the device launch; the reference's error behaviour.
* GPU: pq_simulate_periods through Strategy.simulate / turnover_pairs against the same
  golden vectors, and against the oracle on a config-3-sized panel (n = 1000, 4749 daily
  holding periods).  Tolerance: 1e-13 absolute on daily returns / weights (FP64 sums in a
  different order than pandas), 1e-12 on turnover.
"""
import os

import numpy as np
import pandas as pd
import pytest

from oracle import simulate as osim
from porqua_amd.portfolio import Portfolio, Strategy

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")


def _load():
    g = np.load(os.path.join(GOLD, "msci_simulate.npz"))
    p = np.load(os.path.join(GOLD, "msci_panel.npz"))
    dates = pd.DatetimeIndex(p["dates"].astype("datetime64[D]"))
    names = [str(c) for c in p["columns"]]
    X = pd.DataFrame(p["returns"], index=dates, columns=names)
    return g, X, names


def _strategy(names, reb, W):
    return Strategy([Portfolio(rebalancing_date=str(d), weights=dict(zip(names, W[i])))
                     for i, d in enumerate(reb)])


def _days(X):
    return X.index.values.astype("datetime64[D]").astype(np.int64)


@pytest.mark.parametrize("tag", ["long", "ls"])
def test_oracle_simulate_matches_reference(tag):
    g, X, _ = _load()
    reb = g["rebdates"].astype("datetime64[D]").astype(np.int64)
    W = g["W_" + tag]
    for fc in (0, 1):
        d, r = osim.simulate(X.to_numpy(), _days(X), reb, W, fc=fc / 100)
        assert np.array_equal(d, g[f"sim_{tag}_fc{fc}_days"])
        assert np.abs(r - g[f"sim_{tag}_fc{fc}_ret"]).max() < 1e-14
    for rs in (0, 1):
        e, t = osim.turnover_pairs(X.to_numpy(), _days(X), reb, W, bool(rs))
        assert np.abs(e - g[f"float_end_{tag}_r{rs}"]).max() < 1e-14
        assert np.abs(t - g[f"turnover_{tag}_r{rs}"]).max() < 1e-14


def test_host_pair_helpers_match_reference():
    """Portfolio.float_weights / turnover (host, pandas) on a few golden pairs."""
    g, X, names = _load()
    reb = [str(d) for d in g["rebdates"]]
    for tag in ("long", "ls"):
        W = g["W_" + tag]
        for i in (1, 50, 165):
            for rs in (0, 1):
                a = Portfolio(rebalancing_date=reb[i - 1], weights=dict(zip(names, W[i - 1])))
                b = Portfolio(rebalancing_date=reb[i], weights=dict(zip(names, W[i])))
                wf = a.float_weights(return_series=X, end_date=reb[i], rescale=bool(rs))
                assert np.abs(wf.iloc[-1].values - g[f"float_end_{tag}_r{rs}"][i - 1]).max() < 1e-14
                to = b.turnover(portfolio=a, return_series=X, rescale=bool(rs))
                assert abs(to - g[f"turnover_{tag}_r{rs}"][i - 1]) < 1e-13


def test_staging_rows_match_oracle_periods():
    g, X, names = _load()
    reb = g["rebdates"]
    S = _strategy(names, reb, g["W_long"])
    nm, W, days, row0, nrows = S._stage(X, last_end=True)
    assert nm == names and np.array_equal(W, g["W_long"])
    rd = reb.astype("datetime64[D]").astype(np.int64)
    for i in range(len(rd)):
        end = rd[i + 1] if i + 1 < len(rd) else days[-1]
        s, e = osim.period_rows(days, rd[i], end)
        assert (row0[i], nrows[i]) == (s, e - s)
    # returns per period = nrows - 1, and their count equals the reference's series length
    assert int((nrows - 1).sum()) == len(g["sim_long_fc0_ret"])


def test_reference_error_behaviour_is_kept():
    g, X, names = _load()
    assert str(g["raises_simulate_vc"]) == "TypeError"
    assert str(g["raises_strategy_turnover"]) == "TypeError"
    S = _strategy(names, g["rebdates"][:3], g["W_long"])
    with pytest.raises(TypeError):
        S.turnover(return_series=X, rescale=False)
    with pytest.raises(TypeError):
        S.simulate(return_series=X, fc=0, vc=0.002)
    with pytest.raises(ValueError):
        Strategy([]).simulate(return_series=X)
    bad = Strategy([Portfolio(rebalancing_date="2010-01-04", weights={"nope": 1.0})])
    with pytest.raises(ValueError):
        bad._stage(X, last_end=True)
    early = Strategy([Portfolio(rebalancing_date="1900-01-04", weights={names[0]: 1.0})])
    with pytest.raises(ValueError):
        early._stage(X, last_end=True)


@pytest.mark.gpu
@pytest.mark.parametrize("tag", ["long", "ls"])
def test_device_simulate_matches_reference(tag):
    g, X, names = _load()
    S = _strategy(names, g["rebdates"], g["W_" + tag])
    for fc in (0, 1):
        r = S.simulate(return_series=X, fc=fc / 100)
        days = r.index.values.astype("datetime64[D]").astype(np.int64)
        assert np.array_equal(days, g[f"sim_{tag}_fc{fc}_days"])
        assert np.abs(r.values - g[f"sim_{tag}_fc{fc}_ret"]).max() < 1e-13
    for rs in (0, 1):
        to = S.turnover_pairs(return_series=X, rescale=bool(rs))
        assert list(to.index) == [str(d) for d in g["rebdates"][1:]]
        assert np.abs(to.values - g[f"turnover_{tag}_r{rs}"]).max() < 1e-12


@pytest.mark.gpu
def test_device_float_end_weights_match_reference():
    import torch
    from porqua_amd import engine
    g, X, names = _load()
    S = _strategy(names, g["rebdates"], g["W_ls"])
    nm, W, days, row0, nrows = S._stage(X, last_end=True)
    dev = engine.default_device()
    for rs in (0, 1):
        _, wend, to = engine.simulate_periods(torch.as_tensor(X[nm].to_numpy(), device=dev),
                                              torch.as_tensor(W, device=dev), row0, nrows,
                                              rescale=bool(rs), want_end=True)
        we = wend.cpu().numpy()
        assert np.abs(we[:-1] - g[f"float_end_ls_r{rs}"]).max() < 1e-13
        assert np.abs(to.cpu().numpy()[:-1] - g[f"turnover_ls_r{rs}"]).max() < 1e-12


@pytest.mark.gpu
def test_device_simulate_config3_size_matches_oracle():
    """n = 1000 assets, 4749 daily holding periods (config 3), long/short weights with
    NaN returns sprinkled in (fillna(0)); plus one monthly (stride 21) run."""
    from porqua_amd import synthetic
    rng = np.random.default_rng(11)
    dates, R = synthetic.factor_panel(5000, 1000, seed=20240314)[:2]
    R = R.copy()
    R[rng.integers(0, 5000, 200), rng.integers(0, 1000, 200)] = np.nan
    X = pd.DataFrame(R, index=pd.DatetimeIndex(dates), columns=[f"A{i}" for i in range(1000)])
    for stride in (1, 21):
        reb = X.index[251::stride][:-1]
        W = rng.dirichlet(np.ones(1000), len(reb)) + rng.normal(0, 1e-3, (len(reb), 1000))
        S = _strategy(list(X.columns), [d.strftime("%Y-%m-%d") for d in reb], W)
        r = S.simulate(return_series=X, fc=0.005)
        d, ro = osim.simulate(R, _days(X), reb.values.astype("datetime64[D]").astype(np.int64), W, fc=0.005)
        assert np.array_equal(r.index.values.astype("datetime64[D]").astype(np.int64), d)
        assert np.abs(r.values - ro).max() < 1e-13
