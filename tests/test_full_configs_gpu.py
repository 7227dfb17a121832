"""Parity at the FULL benchmark sizes of configs 2, 4 and 5 (BASELINE.json configs[1], [3],
[4]): every problem of the batch the benchmark times is KKT-certified from the panel rows
(workloads.window_certificate: P x recomputed with torch, not by the engine), and 16 evenly
spaced problems of each batch are compared with oracle optima committed as fixtures
(tools/capture_full.py -> tests/golden/config{2d,4f,5f}_oracle.npz; oracle.qp_ipm,
KKT-certified):

* objective within 1e-6 relative (north_star), violation <= 1e-7;
* weights within 1e-5 where the optimum is unique (support below rank(P) <= T - 1); config 4's
  optima keep all 3000 weights free on a rank-252 P, so only the objective is defined there.

Reference: src/qp_problems.py:184-221 (solve, objective_value), src/optimization.py:168-174
(MeanVariance), 206-226 (LeastSquares), src/constraints.py:66-94, 114-167 (sector caps)."""
import numpy as np
import pytest
import torch

from porqua_amd import _lib, engine
from porqua_amd.sweep import mean_variance_sweep
from porqua_amd.synthetic import factor_panel
from porqua_amd.workloads import TrackingBacktest, sweep_certificate
from tests.conftest import load_golden

pytestmark = pytest.mark.gpu

VIOL, STAT = 1e-7, 1e-7


def _check_cert(cert, B):
    assert cert["problems"] == B
    assert cert["status_counts"] == {str(_lib.PQ_SOLVED): B}, cert
    assert cert["max_violation"] <= VIOL, cert
    assert cert["max_rel_stationarity"] <= STAT, cert
    assert cert["max_rel_complementarity"] <= STAT and cert["max_dual_sign"] <= STAT, cert


def test_config4_full_batch_certified_and_matches_oracle(device):
    wl = TrackingBacktest(device=device)               # 9749 daily dates, n = 3000, 21 general rows
    assert wl.D == 9749 and wl.qb.mg == 21
    res = wl.step()
    cert = wl.certificate(res)
    _check_cert(cert, wl.D)
    gold = load_golden("config4f_oracle")
    assert int(gold["n_dates"]) == wl.D
    x = res.x.cpu().numpy()
    T, R, y = wl.T, wl.R_rank, wl.y_rank
    for p, e, xo, oo in zip(gold["problems"], gold["ends"], gold["x"], gold["obj"]):
        assert wl.ends_local[p] == e
        X = R[e - T + 1:e + 1]
        v = X @ x[p]
        obj = v @ v - 2 * (y[e - T + 1:e + 1] @ v)       # 0.5 x'(2X'X)x + (-2X'y)'x
        assert abs(obj - oo) <= 1e-6 * abs(oo), (p, obj, oo)
        if (xo > 1e-9).sum() < T - 1:
            assert np.abs(x[p] - xo).max() <= 1e-5, p


def test_config5_full_sweep_certified_and_matches_oracle(device):
    n, T, nd, L = 5000, 252, 64, 64
    dates, R, _, _ = factor_panel(T - 1 + 21 * nd, n)
    ends = np.arange(T - 1, T - 1 + 21 * nd, 21)
    rows, tlen = engine.window_rows(dates, dates[ends], T)
    pan = engine.Panel(R, device=device)
    lambdas = np.logspace(-1, 2, L)
    res, meta = mean_variance_sweep(pan, rows, tlen, lambdas)
    cert = sweep_certificate(pan, res, meta)
    _check_cert(cert, nd * L)
    gold = load_golden("config5f_oracle")
    assert np.allclose(gold["lambdas"], lambdas)
    x = res.x.cpu().numpy()
    for p, e, j, xo, oo in zip(gold["problems"], gold["ends"], gold["lam_index"], gold["x"], gold["obj"]):
        d = p // L
        assert ends[d] == e and p % L == j
        W = R[e - T + 1:e + 1]
        Wc = W - W.mean(0)
        mu = np.exp(np.mean(np.log1p(W), axis=0)) - 1.0
        v = Wc @ x[p]
        obj = lambdas[j] * (v @ v) / (T - 1) - mu @ x[p]   # 0.5 x'(2 lam Sigma)x - mu'x
        assert abs(obj - oo) <= 1e-6 * abs(oo), (p, obj, oo)
        if (xo > 1e-9).sum() < T - 1:
            assert np.abs(x[p] - xo).max() <= 1e-5, p


def _budget_box_certificate(R, ends, T, W, q, scale=2.0, chunk=256):
    """Multiplier-free KKT check of budget + box [0, 1] solutions with P = scale X'X over the
    windows ending at ``ends``: y = -median of (P x + q) over the free weights; stationarity
    on the free weights and the sign of the bound multipliers, relative to max(|Px|, |q|, |y|)."""
    dev = R.device
    worst_stat, worst_sign = 0.0, 0.0
    ar = torch.arange(T, device=dev)
    for s in range(0, len(ends), chunk):
        e = torch.as_tensor(ends[s:s + chunk], device=dev)
        X = R[(e[:, None] - T + 1 + ar[None, :]).long()]
        x = W[s:s + chunk]
        Px = scale * torch.bmm(X.transpose(1, 2), torch.bmm(X, x[:, :, None]))[:, :, 0]
        g = Px + q[s:s + chunk]
        free = (x > 1e-9) & (x < 1 - 1e-9)
        gf = torch.where(free, g, torch.full_like(g, float("nan")))
        yv = -torch.nanmedian(gf, dim=1).values
        r = g + yv[:, None]
        sc = torch.stack([Px.abs().amax(1), q[s:s + chunk].abs().amax(1), yv.abs()]).amax(0)
        worst_stat = max(worst_stat, float((torch.where(free, r.abs(), 0.0).amax(1) / sc).max()))
        lo = x <= 1e-9
        up = x >= 1 - 1e-9
        sign = torch.maximum(torch.where(lo, (-r).clamp(min=0), 0.0), torch.where(up, r.clamp(min=0), 0.0))
        worst_sign = max(worst_sign, float((sign.amax(1) / sc).max()))
    return worst_stat, worst_sign


def test_config2_daily_all_dates_through_backtest_run(device):
    """Every daily date of the usa-shaped panel (4544 LS tracking QPs, n = 494) through
    Backtest.run with solver_name='mi355x': all solved, feasible, KKT-certified, and equal to
    the oracle on 16 evenly spaced dates."""
    import pandas as pd
    from porqua_amd.backtest import Backtest
    from tests.test_configs12_gpu import service, usa_data
    X, y = usa_data()
    T = 252
    rebdates = [str(r.date()) for r in X.index[T - 1:]]
    assert len(rebdates) == 4544
    bt = Backtest()
    bt.run(service(X, y, rebdates))
    assert bt.stats["solved"] == len(rebdates) and bt.stats["path"] == "lowrank"
    Wn = bt.strategy.get_weights_df().to_numpy(dtype=float)
    assert np.abs(Wn.sum(1) - 1).max() <= VIOL and Wn.min() >= -VIOL and Wn.max() <= 1 + VIOL
    Xv, yv = X.to_numpy(), y.to_numpy()[:, 0]
    ends = np.array([X.index.get_loc(pd.Timestamp(r)) for r in rebdates])
    Rd = torch.from_numpy(Xv).to(device)
    yd = torch.from_numpy(yv).to(device)
    ar = torch.arange(T, device=device)
    idx = (torch.from_numpy(ends).to(device)[:, None] - T + 1 + ar[None, :]).long()
    q = -2.0 * torch.bmm(Rd[idx].transpose(1, 2), yd[idx][:, :, None])[:, :, 0]
    stat, sign = _budget_box_certificate(Rd, ends, T, torch.from_numpy(Wn).to(device), q)
    assert stat <= STAT and sign <= STAT, (stat, sign)
    gold = load_golden("config2d_oracle")
    assert int(gold["n_dates"]) == len(rebdates)
    for p, e, xo, oo in zip(gold["problems"], gold["ends"], gold["x"], gold["obj"]):
        assert ends[p] == e
        Xw, yw = Xv[e - T + 1:e + 1], yv[e - T + 1:e + 1]
        v = Xw @ Wn[p]
        obj = v @ v - 2 * (yw @ v)
        assert abs(obj - oo) <= 1e-6 * abs(oo), (p, obj, oo)
        if (xo > 1e-8).sum() < T - 1:
            assert np.abs(Wn[p] - xo).max() <= 1e-5, (p, np.abs(Wn[p] - xo).max())
