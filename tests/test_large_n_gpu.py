"""BASELINE.json configs[3] and configs[4] beyond the 1024-asset LDS limit of the dense
kernels, on the window path (grouped low-rank ADMM + window polish):

  * config 4 shape: n = 3000 tracking-error least squares (uncentred Gram, q = -2 X'y,
    LeastSquares.set_objective, src/optimization.py:206-226) with budget + 20 sector caps
    (G 20 x n, the group rows of Constraints.to_GhAb, src/constraints.py:114-167) and a
    long-only box -- 21 general rows;
  * config 5 shape: n = 5000 mean-variance risk-aversion x date sweep (porqua_amd.sweep).

Both compare every solved problem against oracle optima committed as fixtures
(tools/capture_large.py -> tests/golden/config4_oracle.npz, config5_oracle.npz; oracle.qp_ipm,
KKT-certified): the objective to 1e-6 relative everywhere, the weights to 1e-5 where the
optimum is unique (support well below rank(P) <= T = 252), plus feasibility and the
relative KKT certificate (tests/kkt.py)."""
import numpy as np
import pytest
import torch

from oracle.qp_ipm import solve_qp
from oracle.ref_pipeline import cov_pearson
from porqua_amd import _lib, engine
from porqua_amd.sweep import mean_variance_sweep
from porqua_amd.synthetic import factor_panel
from tests.conftest import load_golden
from tests.kkt import kkt_residuals

pytestmark = pytest.mark.gpu


def test_config4_tracking_n3000_sector_caps(device):
    n, T, ns, cap = 3000, 252, 20, 0.15
    ends = list(range(260, 266))
    dates, R, y, sec = factor_panel(max(ends) + 1, n, n_sectors=ns)
    rows, tlen = engine.window_rows(dates, dates[ends], T)
    pan = engine.Panel(R, y, device=device)
    r_d, t_d = pan.rows_to_device(rows, tlen)
    B = len(ends)
    G = np.stack([(sec == g).astype(float) for g in range(ns)])
    h = np.full(ns, cap)
    qb = engine.QPBatch.from_dense(np.zeros((1, n, n)), np.zeros((1, n)), A=np.ones((1, n)), b=np.ones(1),
                                   G=G, h=h, lb=np.zeros(n), ub=np.ones(n), device=device)
    qb.batch = B
    qb.P = None
    xty, _ = pan.gram_xy(r_d, t_d)
    qb.q = (-2.0 * xty).contiguous()
    qb.p_scale = torch.full((B,), 2.0, dtype=torch.float64, device=device)
    lr = engine.LowRank(pan, r_d, t_d, mu=None)
    gp = engine.GroupPlan(rows, tlen, device)
    ws = engine.Workspace(qb, dense=False)
    assert qb.mg == 21 and engine.grouped_applicable(qb, lr, gp, ws)
    res = engine.solve_lowrank(qb, lr, engine.Settings(rho0_rel=0.5), ws=ws, groups=gp)
    st = res.status.cpu().numpy()
    x = res.x.cpu().numpy()
    yv = res.y.cpu().numpy()
    zb = res.z_box.cpu().numpy()
    assert np.all(st == _lib.PQ_SOLVED), st
    gold = load_golden("config4_oracle")
    assert list(gold["ends"]) == ends
    for i, e in enumerate(ends):
        X = R[e - T + 1:e + 1]
        P, q = 2 * X.T @ X, -2 * X.T @ y[e - T + 1:e + 1]
        assert abs(x[i].sum() - 1) <= 1e-7 and x[i].min() >= -1e-7 and (G @ x[i]).max() <= cap + 1e-7
        k = kkt_residuals(P, q, x[i], A=np.ones((1, n)), b=np.ones(1), G=G, h=h, lb=np.zeros(n),
                          ub=np.ones(n), y=yv[i], z_box=zb[i])
        assert max(k.values()) <= 1e-7, k
        obj = 0.5 * x[i] @ P @ x[i] + q @ x[i]
        assert abs(obj - gold["obj"][i]) <= 1e-6 * abs(gold["obj"][i]), (e, obj, gold["obj"][i])
        if (gold["x"][i] > 1e-9).sum() < T // 2:   # unique optimum: the weights too
            assert np.abs(x[i] - gold["x"][i]).max() <= 1e-5
    # the first date once more against a fresh oracle solve (the fixture's own pin)
    X = R[ends[0] - T + 1:ends[0] + 1]
    o = solve_qp(2 * X.T @ X, -2 * X.T @ y[ends[0] - T + 1:ends[0] + 1], G=G, h=h, A=np.ones((1, n)), b=np.ones(1),
                 lb=np.zeros(n), ub=np.ones(n))
    assert abs(o.obj - gold["obj"][0]) <= 1e-8 * abs(o.obj)


def test_config5_risk_aversion_sweep_n5000(device):
    n, T = 5000, 252
    lambdas = np.logspace(-1, 2, 4)
    ends = [300, 321]
    dates, R, y, sec = factor_panel(max(ends) + 1, n)
    rows, tlen = engine.window_rows(dates, dates[ends], T)
    pan = engine.Panel(R, device=device)
    res, meta = mean_variance_sweep(pan, rows, tlen, lambdas)
    assert meta["grouped"]
    st = res.status.cpu().numpy()
    x = res.x.cpu().numpy()
    yv = res.y.cpu().numpy()
    zb = res.z_box.cpu().numpy()
    assert np.all(st == _lib.PQ_SOLVED), st
    gold = load_golden("config5_oracle")
    assert np.allclose(gold["lambdas"], lambdas)
    for d, e in enumerate(ends):
        W = R[e - T + 1:e + 1]
        S = cov_pearson(W)
        mu = np.exp(np.mean(np.log1p(W), axis=0)) - 1.0
        for j, lam in enumerate(lambdas):
            p = d * len(lambdas) + j
            assert tuple(gold["pairs"][p]) == (e, j)
            P = 2 * lam * S
            k = kkt_residuals(P, -mu, x[p], A=np.ones((1, n)), b=np.ones(1), lb=np.zeros(n), ub=np.ones(n),
                              y=yv[p], z_box=zb[p])
            assert max(k.values()) <= 1e-7, (lam, k)
            obj = 0.5 * x[p] @ P @ x[p] - mu @ x[p]
            assert abs(res.obj[p].item() - obj) <= 1e-9 * max(1.0, abs(obj))
            assert abs(obj - gold["obj"][p]) <= 1e-6 * abs(gold["obj"][p]), (e, lam, obj, gold["obj"][p])
            if (gold["x"][p] > 1e-9).sum() < T // 2:
                assert np.abs(x[p] - gold["x"][p]).max() <= 1e-5, (e, lam)


def test_sweep_small_risk_aversion_needs_no_admm_retry(device):
    """Nearly linear objectives (risk aversion 0.1 .. 1, q = -mu dominates P): the q-aware
    initial rho and the re-polish with more refinement steps keep every problem off the
    slow eps-1e-7 ADMM retry (regression: 4000-iteration tails in the config-5 sweep)."""
    n, T = 1000, 252
    lambdas = np.logspace(-1, 0, 16)
    ends = [260, 281]
    dates, R, y, sec = factor_panel(max(ends) + 1, n)
    rows, tlen = engine.window_rows(dates, dates[ends], T)
    pan = engine.Panel(R, device=device)
    res, meta = mean_variance_sweep(pan, rows, tlen, lambdas)
    st = res.status.cpu().numpy()
    assert np.all(st == _lib.PQ_SOLVED), st
    assert int(res.iters.max().item()) < 300, int(res.iters.max().item())
    x, yv, zb = res.x.cpu().numpy(), res.y.cpu().numpy(), res.z_box.cpu().numpy()
    for d, e in enumerate(ends):
        W = R[e - T + 1:e + 1]
        S = cov_pearson(W)
        mu = np.exp(np.mean(np.log1p(W), axis=0)) - 1.0
        for j in (0, 7, 15):
            p = d * len(lambdas) + j
            k = kkt_residuals(2 * lambdas[j] * S, -mu, x[p], A=np.ones((1, n)), b=np.ones(1), lb=np.zeros(n),
                              ub=np.ones(n), y=yv[p], z_box=zb[p])
            assert max(k.values()) <= 1e-7, (lambdas[j], k)
