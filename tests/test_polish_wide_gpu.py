"""Wide rounds of the grouped polish (polish_gw.hip): dates whose free set exceeds the LDS
solve (k > min(128, ldk)) with at most 8 bordered rows (active general rows + variables at
a bound) solve the round's regularised KKT system by a group capacitance of P + d I with
MFMA window passes over the slide group's union rows, instead of the per-date Woodbury
kernel (polish_w.hip).  Against that per-date kernel on the same ADMM point: the same status,
objective to 1e-10 relative, and a KKT certificate recomputed with torch from the panel rows
(workloads.window_certificate) at the parity bars; weights are compared where the optimum is
unique (P = 2 X'X + a ridge: positive definite).  Uncentred windows (the tracking objectives)
only: centred windows keep the per-date kernel (engine._pg_wide_setup)."""
import numpy as np
import pytest
import torch

from porqua_amd import _lib, engine
from porqua_amd.synthetic import factor_panel
from porqua_amd.workloads import window_certificate

pytestmark = pytest.mark.gpu
F64 = torch.float64


def _problem(device, n, T, D, lb, ub, centred, sectors=0, cap=0.15, ridge=0.0, stride=1):
    ends = list(range(T + 5, T + 5 + D * stride, stride))
    dates, R, y, sec = factor_panel(max(ends) + 1, n, n_sectors=max(sectors, 1))
    rows, tlen = engine.window_rows(dates, dates[ends], T)
    pan = engine.Panel(R, y, device=device)
    r_d, t_d = pan.rows_to_device(rows, tlen)
    G = h = None
    if sectors:
        G = np.stack([(sec == g).astype(float) for g in range(sectors)])
        h = np.full(sectors, cap)
    qb = engine.QPBatch.from_dense(None, None, A=np.ones((1, n)), b=np.ones(1), G=G, h=h, lb=np.full(n, lb),
                                   ub=np.full(n, ub), device=device, n=n)
    qb.batch = D
    qb.p_scale = torch.full((D,), 2.0, dtype=F64, device=device)
    if ridge:
        qb.p_diag = torch.full((D,), ridge, dtype=F64, device=device)
    if centred:
        mu = pan.window_means(r_d, t_d)
        qb.q = (-0.05 * mu).contiguous()
        lr = engine.LowRank(pan, r_d, t_d, mu=mu, w_scale=1.0 / (t_d.to(F64) - 1.0))
    else:
        xty, _ = pan.gram_xy(r_d, t_d)
        qb.q = (-2.0 * xty).contiguous()
        lr = engine.LowRank(pan, r_d, t_d, mu=None)
    gp = engine.GroupPlan(rows, tlen, device)
    return pan, qb, lr, gp


def _solve(qb, lr, gp, wide, settings):
    ws = engine.Workspace(qb, dense=False)
    res = engine.solve_lowrank(qb, lr, settings, ws=ws, groups=gp, wide_polish=wide)
    torch.cuda.synchronize()
    return res, ws


def _cert(pan, qb, lr, res):
    n, mg = qb.n, qb.mg
    scale = qb.p_scale * (lr.w_scale if lr.w_scale is not None else 1.0)
    return window_certificate(pan.R, lr.rows, lr.tlen, lr.mu, scale, qb.q[:, :n], res, lb=qb.lb[0, :n],
                              ub=qb.ub[0, :n], C=qb.Cg[0, :mg, :n], lg=qb.lg[0, :mg], ug=qb.ug[0, :mg],
                              p_diag=qb.p_diag)


@pytest.mark.parametrize("case", ["tracking_sectors", "tracking_budget", "tracking_ridge"])
def test_wide_rounds_match_per_date_polish(device, case):
    if case == "tracking_sectors":     # config 4 in miniature: n = 600, 21 general rows, every asset free
        pan, qb, lr, gp = _problem(device, 600, 120, 48, 0.0, 1.0, False, sectors=20, cap=0.15)
        st = engine.Settings(rho0_rel=0.1, rho0_qrel=0.0)
    elif case == "tracking_budget":    # config 2's shape, long-short box: few weights at a bound
        pan, qb, lr, gp = _problem(device, 494, 252, 40, -0.5, 1.0, False)
        st = engine.Settings(rho0_rel=0.1, rho0_qrel=0.0)
    else:                              # long-short box that nothing touches, PD by the ridge
        pan, qb, lr, gp = _problem(device, 400, 120, 40, -1.0, 1.0, False, ridge=1e-4)
        st = engine.Settings(rho0_rel=0.1, rho0_qrel=0.0)
    ra, wa = _solve(qb, lr, gp, False, st)
    sa, oa, xa = ra.status.cpu().numpy().copy(), ra.obj.cpu().numpy().copy(), ra.x.cpu().numpy().copy()
    ca = _cert(pan, qb, lr, ra)
    rb, wb = _solve(qb, lr, gp, True, st)
    sb, ob, xb = rb.status.cpu().numpy(), rb.obj.cpu().numpy(), rb.x.cpu().numpy()
    cb = _cert(pan, qb, lr, rb)
    rec = wb.pg_record()
    wide_used = (rec[:, _lib.PQ_PG_W] == 1.0).cpu().numpy()
    assert wide_used.mean() >= 0.8, wide_used.mean()                 # the wide rounds took the dates
    assert rb.polish_fallbacks <= 0.2 * qb.batch, rb.polish_fallbacks
    assert np.array_equal(sa, sb) and np.all(sb == _lib.PQ_SOLVED), (sa, sb)
    assert np.abs(oa - ob).max() <= 1e-10 * max(np.abs(oa).max(), 1e-12), np.abs(oa - ob).max()
    for c in (ca, cb):
        assert c["max_violation"] <= 1e-9, c
        assert c["max_rel_stationarity"] <= 1e-8, c
        assert c["max_rel_complementarity"] <= 1e-8 and c["max_dual_sign"] <= 1e-8, c
    if case == "tracking_ridge":       # unique optimum
        assert np.abs(xa - xb).max() <= 1e-9, np.abs(xa - xb).max()


def test_centred_windows_keep_the_per_date_kernel(device):
    pan, qb, lr, gp = _problem(device, 400, 120, 24, -1.0, 1.0, True, ridge=1e-4)
    rb, wb = _solve(qb, lr, gp, True, None)
    assert not bool((wb.pg_record()[:, _lib.PQ_PG_W] == 1.0).any())
    assert bool((rb.status == _lib.PQ_SOLVED).all())
    c = _cert(pan, qb, lr, rb)
    assert c["max_violation"] <= 1e-9 and c["max_rel_stationarity"] <= 1e-8, c
