"""Group capacitance (admm_gcap.hip): one capacitance matrix per slide group plus a
per-date low-rank Woodbury correction, against the per-date capacitance path it replaces
(pq_admm_lr_grouped, fused form).

* With one fixed rho for every date (no adaptation) the two are the same ADMM in exact
  arithmetic: the same iteration counts (to rounding) and the same polished weights.
* With the default scale-aware rho (one value per group, the mean of its dates') both
  reach the same optimum.
* Adaptive rho: a group-level refactorisation (every 5 iterations, tight eps) still ends at
  the same optimum.
* Uncentred windows (LeastSquares tracking, P = 2 X'X, q = -2 X'y, src/optimization.py:206-226):
  the group form without the mean column, against the per-date path.
"""
import dataclasses

import numpy as np
import pytest
import torch

from porqua_amd import _lib, engine
from porqua_amd.synthetic import factor_panel

pytestmark = pytest.mark.gpu


def _problem(device, n, T, D, ub, stride=1, centred=True, budget=True, caps=0, cus=256):
    ends = list(range(T + 5, T + 5 + D * stride, stride))
    dates, R, y, sec = factor_panel(max(ends) + 1, n)
    rows, tlen = engine.window_rows(dates, dates[ends], T)
    pan = engine.Panel(R, y, device=device)
    r_d, t_d = pan.rows_to_device(rows, tlen)
    G = np.stack([(sec == g).astype(float) for g in range(caps)]) if caps else None
    qb = engine.QPBatch.from_dense(np.zeros((1, n, n)), np.zeros((1, n)), A=np.ones((1, n)) if budget else None,
                                   b=np.ones(1) if budget else None, G=G, h=np.full(caps, 0.3) if caps else None,
                                   lb=np.zeros(n), ub=np.full(n, ub), device=device)
    qb.batch = D
    qb.P = None
    qb.p_scale = torch.full((D,), 2.0, dtype=torch.float64, device=device)
    qb.q = torch.zeros((D, qb.ld), dtype=torch.float64, device=device)
    if centred:
        mu = pan.window_means(r_d, t_d)
        lr = engine.LowRank(pan, r_d, t_d, mu=mu, w_scale=1.0 / (t_d.to(torch.float64) - 1.0))
    else:   # tracking least squares: P = 2 X'X, q = -2 X'y
        xty, _ = pan.gram_xy(r_d, t_d)
        qb.q = (-2.0 * xty).contiguous()
        lr = engine.LowRank(pan, r_d, t_d, mu=None)
    gp = engine.GroupPlan(rows, tlen, device, cus=cus)
    return qb, lr, gp


def _run(qb, lr, gp, gcap, settings, polish=True):
    # the per-date and the group form compared at the same ADMM stop (Settings.eps_grouped,
    # the looser stop before the grouped polish, applies to the group form only)
    settings = dataclasses.replace(settings or engine.Settings(), eps_grouped=0.0)
    ws = engine.Workspace(qb, dense=False)
    res = engine.solve_lowrank(qb, lr, settings, ws=ws, groups=gp, gcap=gcap, polish=polish)
    torch.cuda.synchronize()
    return (res.x.cpu().numpy().copy(), res.status.cpu().numpy().copy(), res.iters.cpu().numpy().copy(),
            res.capacitance, res.refactors)


@pytest.mark.parametrize("n,T,D,ub,stride", [(1000, 252, 48, 1.0, 1), (400, 120, 40, 0.05, 1), (300, 60, 30, 0.2, 3),
                                              (600, 252, 13, 0.2, 21)])
def test_gcap_same_iterates_with_one_rho(device, n, T, D, ub, stride):
    qb, lr, gp = _problem(device, n, T, D, ub, stride)
    # one fixed rho, no adaptation: the per-date and the group form are the same iteration
    st = engine.Settings(rho0_rel=0.0, rho0=0.01, rho0_qrel=0.0, adapt_interval=0)
    xa, sa, ia, cap_a, _ = _run(qb, lr, gp, False, st)
    xb, sb, ib, cap_b, _ = _run(qb, lr, gp, True, st)
    assert cap_a == "band" and cap_b == "group"
    assert np.all(sa == _lib.PQ_SOLVED) and np.all(sb == _lib.PQ_SOLVED), (sa, sb)
    assert np.abs(ia - ib).max() <= 1, (ia, ib)
    assert np.abs(xa - xb).max() <= 1e-9, np.abs(xa - xb).max()


def test_gcap_default_rho_same_optimum(device):
    qb, lr, gp = _problem(device, 1000, 252, 64, 1.0)
    xa, sa, ia, _, _ = _run(qb, lr, gp, False, None)
    xb, sb, ib, cap, _ = _run(qb, lr, gp, True, None)
    assert cap == "group"
    assert np.all(sa == _lib.PQ_SOLVED) and np.all(sb == _lib.PQ_SOLVED)
    assert np.abs(xa - xb).max() <= 1e-8, np.abs(xa - xb).max()
    assert abs(ib.mean() - ia.mean()) <= 2.0, (ia.mean(), ib.mean())


def test_gcap_group_rho_adaptation(device):
    qb, lr, gp = _problem(device, 400, 120, 40, 0.1)
    st = engine.Settings(adapt_interval=5, eps_abs=1e-6, eps_rel=1e-6, rho0_rel=0.0, rho0=1e-5, rho0_qrel=0.0)
    xa, sa, _, _, _ = _run(qb, lr, gp, False, engine.Settings())
    xb, sb, ib, cap, refactors = _run(qb, lr, gp, True, st)
    assert cap == "group" and refactors > 0
    assert np.all(sb == _lib.PQ_SOLVED), sb
    assert np.abs(xa - xb).max() <= 1e-8


@pytest.mark.parametrize("n,T,D,ub,stride", [(1000, 252, 48, 1.0, 1), (494, 252, 40, 1.0, 1), (300, 60, 30, 0.2, 3),
                                              (494, 252, 13, 1.0, 21)])
def test_gcap_uncentred_same_iterates_with_one_rho(device, n, T, D, ub, stride):
    """The ADMM iterates themselves (no polish): the tracking P = 2 X'X has rank T < n, so
    the optimum can be a face and polished points of two exact solvers need not coincide."""
    qb, lr, gp = _problem(device, n, T, D, ub, stride, centred=False)
    st = engine.Settings(rho0_rel=0.0, rho0=0.05, rho0_qrel=0.0, adapt_interval=0)
    xa, sa, ia, cap_a, _ = _run(qb, lr, gp, False, st, polish=False)
    xb, sb, ib, cap_b, _ = _run(qb, lr, gp, True, st, polish=False)
    assert cap_a == "band" and cap_b == "group"
    assert np.all(sa == _lib.PQ_SOLVED) and np.all(sb == _lib.PQ_SOLVED), (sa, sb)
    assert np.array_equal(ia, ib), (ia, ib)
    # uncentred windows leave the market mode in X_U X_U' (the centred case removes it), so
    # the Woodbury correction H_b is worse conditioned and rounding differences between the
    # per-date and the group form grow to ~2e-9 over ~20 iterations (measured; x ~ 1e-3)
    assert np.abs(xa - xb).max() <= 1e-8, np.abs(xa - xb).max()


def _objective(qb, lr, x):
    """1/2 x'P x + q'x with P = 2 X'X of each date's window (torch, independent of the engine)."""
    R = lr.panel.R
    X = R[lr.rows.long()] * (torch.arange(lr.tmax, device=R.device)[None, :] < lr.tlen[:, None]).to(R.dtype)[:, :, None]
    xt = torch.from_numpy(x).to(R.device)
    v = torch.bmm(X, xt[:, :, None])[:, :, 0]
    return ((v * v).sum(1) + (qb.q[:, :x.shape[1]] * xt).sum(1)).cpu().numpy()


def test_gcap_uncentred_tracking_default_settings(device):
    qb, lr, gp = _problem(device, 1000, 252, 64, 1.0, centred=False)
    st = engine.Settings(rho0_rel=0.1, rho0_qrel=0.0)   # the tracking workloads' settings
    xa, sa, _, _, _ = _run(qb, lr, gp, False, st)
    xb, sb, _, cap, _ = _run(qb, lr, gp, True, st)
    assert cap == "group"
    assert np.all(sa == _lib.PQ_SOLVED) and np.all(sb == _lib.PQ_SOLVED)
    fa, fb = _objective(qb, lr, xa), _objective(qb, lr, xb)
    assert np.abs(fa - fb).max() <= 1e-9 * np.abs(fa).max(), np.abs(fa - fb).max()
    assert np.abs(xb.sum(1) - 1).max() < 1e-10 and xb.min() > -1e-10


@pytest.mark.parametrize("budget,caps", [(False, 0), (True, 2)])
def test_gcap_general_row_variants_same_iterates(device, budget, caps):
    """The kernel's general-row variants beyond the budget alone: none (box only, k_admm_gcap<0>;
    q = -mu so the optimum is not the origin) and the budget with two sector caps (three
    register-resident rows): the same ADMM iterates as the per-date form with one fixed rho.
    (Round 4's k_admm_gcap<0> read an undefined Cg register in its epilogue and reported every
    box-only date SOLVED after one iteration: gpurun_out/r04n_pytest.txt.)"""
    qb, lr, gp = _problem(device, 600, 150, 40, 0.2, budget=budget, caps=caps)
    if not budget:
        qb.q = (-lr.mu * 50.0).contiguous()
    assert qb.mg == int(budget) + caps
    st = engine.Settings(rho0_rel=0.0, rho0=0.01, rho0_qrel=0.0, adapt_interval=0)
    xa, sa, ia, cap_a, _ = _run(qb, lr, gp, False, st, polish=False)
    xb, sb, ib, cap_b, _ = _run(qb, lr, gp, True, st, polish=False)
    assert cap_a == "band" and cap_b == "group"
    assert np.all(sa == _lib.PQ_SOLVED) and np.all(sb == _lib.PQ_SOLVED), (sa, sb)
    assert ia.min() > 1, ia
    assert np.abs(ia - ib).max() <= 1, (ia, ib)
    assert np.abs(xa - xb).max() <= 1e-9, np.abs(xa - xb).max()


def test_box_only_problems_group_form_same_optimum(device):
    """Box only (mg = 0) with the default settings and the polish: the group form is taken
    and reaches the per-date form's optimum (weights 1e-8, inside the box)."""
    qb, lr, gp = _problem(device, 600, 150, 40, 0.2, budget=False)
    qb.q = (-lr.mu * 50.0).contiguous()
    assert qb.mg == 0
    xa, sa, ia, cap_a, _ = _run(qb, lr, gp, False, None)
    xb, sb, ib, cap_b, _ = _run(qb, lr, gp, True, None)
    assert cap_b == "group"
    assert np.all(sa == _lib.PQ_SOLVED) and np.all(sb == _lib.PQ_SOLVED), (sa, sb)
    assert ib.min() > 1, ib
    assert np.abs(xa - xb).max() <= 1e-8, np.abs(xa - xb).max()
    assert xb.min() > -1e-9 and xb.max() < 0.2 + 1e-9


def test_gcap_nan_iterate_is_not_solved(device):
    """A date whose data carries a NaN (here its q) cannot pass the convergence test: the
    residual maxima are fmax reductions, which drop NaN, so the kernel checks a NaN-carrying
    sum and fails the date (PQ_NON_CONVEX, found = False) while its group's other dates solve."""
    qb, lr, gp = _problem(device, 600, 150, 40, 0.2, budget=True)
    qb.q = (-lr.mu * 5.0).contiguous()
    qb.q[7, 3] = float("nan")
    st = engine.Settings(rho0_rel=0.0, rho0=0.01, rho0_qrel=0.0, adapt_interval=0)
    _, sb, _, cap_b, _ = _run(qb, lr, gp, True, st, polish=False)
    assert cap_b == "group"
    assert sb[7] == _lib.PQ_NON_CONVEX, sb
    assert np.all(np.delete(sb, 7) == _lib.PQ_SOLVED), sb


@pytest.mark.parametrize("centred,mg_caps", [(True, 0), (False, 0), (True, 2), (True, 8), (False, 8)])
def test_gcap_32_date_groups_same_iterates(device, centred, mg_caps):
    """The 32-date form (two MFMA column blocks, one 512-thread workgroup per group; the plan
    GroupPlan.gcap_plan builds CU-balanced groups of up to 32 dates -- here 19, with cus = 16):
    the same ADMM iterates as the per-date form with one fixed rho, centred and uncentred
    windows, the budget alone, with two sector caps (register-resident rows) and with eight
    (mg = 9: the column-sparse wide form, config 4's shape)."""
    qb, lr, gp = _problem(device, 600, 120, 300, 0.2, centred=centred, caps=mg_caps, cus=16)
    g32 = gp.gcap_plan()
    assert g32 is not gp and int(g32.sizes.max()) > 16 and int(gp.sizes.max()) <= 16
    st = engine.Settings(rho0_rel=0.0, rho0=0.01, rho0_qrel=0.0, adapt_interval=0, eps_grouped=0.0)
    ws = engine.Workspace(qb, dense=False)
    ra = engine.solve_lowrank(qb, lr, st, ws=ws, groups=gp, gcap=False, polish=False)
    xa, sa, ia = ra.x.cpu().numpy().copy(), ra.status.cpu().numpy().copy(), ra.iters.cpu().numpy().copy()
    ws2 = engine.Workspace(qb, dense=False)
    rb = engine.solve_lowrank(qb, lr, st, ws=ws2, groups=gp, gcap=True, polish=False)
    torch.cuda.synchronize()
    assert rb.capacitance == "group" and ws2.gcap_groups is g32
    xb, sb, ib = rb.x.cpu().numpy(), rb.status.cpu().numpy(), rb.iters.cpu().numpy()
    assert np.all(sa == _lib.PQ_SOLVED) and np.all(sb == _lib.PQ_SOLVED), (sa, sb)
    assert np.abs(ia - ib).max() <= 1, (ia, ib)
    # rounding differences between the per-date and any group form grow with the iterations:
    # on this problem with the caps the 16-date form differs from the per-date one by 1.2e-9
    # and the 32-date one by 1.6e-9 (tools/diag_gcap32.py, profiles/r05k_diag_gcap32.log)
    tol = (1e-9 if not mg_caps else 3e-9) if centred else 1e-8
    if mg_caps > 4:   # the wide form: bounded by twice the 16-date wide form's own drift
        old_wide = engine.GCAP32_WIDE
        try:
            engine.GCAP32_WIDE = False
            ws3 = engine.Workspace(qb, dense=False)
            rc = engine.solve_lowrank(qb, lr, st, ws=ws3, groups=gp, gcap=True, polish=False)
            torch.cuda.synchronize()
            assert ws3.gcap_groups is gp
            d16 = np.abs(xa - rc.x.cpu().numpy()).max()
        finally:
            engine.GCAP32_WIDE = old_wide
        tol = max(tol, 2.0 * d16)
    assert np.abs(xa - xb).max() <= tol, (np.abs(xa - xb).max(), tol)


def test_gcap_32_date_groups_polished_optimum(device):
    """Default settings, the whole solve (loose ADMM stop, grouped polish on its 16-date plan):
    the 32-date group form reaches the optimum of the 16-date one."""
    import porqua_amd.engine as eng
    qb, lr, gp = _problem(device, 1000, 252, 400, 1.0, cus=16)
    assert int(gp.gcap_plan().sizes.max()) > 16
    ws = engine.Workspace(qb, dense=False)
    rb = engine.solve_lowrank(qb, lr, None, ws=ws, groups=gp)
    xb, sb = rb.x.cpu().numpy().copy(), rb.status.cpu().numpy().copy()
    assert ws.gcap_groups is gp.gcap_plan()
    old = eng.GCAP_MAX_DATES
    try:
        eng.GCAP_MAX_DATES = 16
        qb2, lr2, gp2 = _problem(device, 1000, 252, 400, 1.0, cus=16)
        ws2 = engine.Workspace(qb2, dense=False)
        ra = engine.solve_lowrank(qb2, lr2, None, ws=ws2, groups=gp2)
        assert ws2.gcap_groups is gp2
    finally:
        eng.GCAP_MAX_DATES = old
    torch.cuda.synchronize()
    xa, sa = ra.x.cpu().numpy(), ra.status.cpu().numpy()
    assert np.all(sa == _lib.PQ_SOLVED) and np.all(sb == _lib.PQ_SOLVED)
    assert np.abs(xa - xb).max() <= 1e-8, np.abs(xa - xb).max()
