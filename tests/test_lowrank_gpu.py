"""Woodbury (low-rank) engine path for T + mg < n: same QP, same polished optimum as the
dense path and the oracle."""
import numpy as np
import pytest
import torch

from oracle.qp_ipm import solve_qp
from oracle.ref_pipeline import cov_pearson
from porqua_amd import engine
from porqua_amd.synthetic import factor_panel

pytestmark = pytest.mark.gpu


def _setup(n, T, ends, centred=True, D=None, seed=None):
    D = D or (max(ends) + 1)
    dates, R, y, sec = factor_panel(D, n, seed=seed or 20240314)
    rows, tlen = engine.window_rows(dates, dates[ends], T)
    pan = engine.Panel(R, y)
    r_d, t_d = pan.rows_to_device(rows, tlen)
    mu = pan.window_means(r_d, t_d) if centred else None
    return dates, R, y, sec, pan, r_d, t_d, mu


@pytest.mark.parametrize("shrink,groups", [(0.0, False), (0.1, False), (0.0, True)])
def test_lowrank_matches_dense_and_oracle_min_variance(device, shrink, groups):
    n, T = 1000, 252
    ends = [300, 451, 599]
    dates, R, y, sec, pan, r_d, t_d, mu = _setup(n, T, ends)
    B = len(ends)
    G = h = None
    if groups:
        G = np.stack([(sec == g).astype(float) for g in range(3)])
        h = np.full(3, 0.12)
    qb = engine.QPBatch.from_dense(np.zeros((1, n, n)), np.zeros((1, n)), A=np.ones((1, n)), b=np.ones(1),
                                   G=G, h=h, lb=np.zeros(n), ub=np.ones(n), device=device)
    qb.batch = B
    qb.P = pan.cov(r_d, t_d, mode=0, mu=mu)
    qb.q = torch.zeros((B, qb.ld), dtype=torch.float64, device=device)
    qb.p_scale = torch.full((B,), 2.0, dtype=torch.float64, device=device)
    if shrink:
        qb.p_diag = 2.0 * shrink * torch.diagonal(qb.P, dim1=1, dim2=2)[:, :n].mean(dim=1)
    lr = engine.LowRank(pan, r_d, t_d, mu=mu, w_scale=1.0 / (t_d.to(torch.float64) - 1.0))
    res_lr = engine.solve_lowrank(qb, lr)
    x_lr = res_lr.x.cpu().numpy().copy()
    st_lr = res_lr.status.cpu().numpy().copy()
    it_lr = res_lr.iters.cpu().numpy().copy()
    res_d = engine.solve(qb)
    x_d = res_d.x.cpu().numpy()
    assert np.all(st_lr == 1) and np.all(res_d.status.cpu().numpy() == 1)
    assert np.abs(x_lr - x_d).max() < 1e-9
    assert np.abs(it_lr - res_d.iters.cpu().numpy()).max() <= 2   # same iterates up to rounding
    for i, e in enumerate(ends):
        S = cov_pearson(R[e - T + 1:e + 1])
        P = 2 * S + (2 * shrink * np.mean(np.diag(S)) * np.eye(n) if shrink else 0)
        o = solve_qp(P, np.zeros(n), G=G, h=h, A=np.ones((1, n)), b=np.ones(1), lb=np.zeros(n), ub=np.ones(n))
        assert np.abs(x_lr[i] - o.x).max() < 1e-5
        assert abs(0.5 * x_lr[i] @ P @ x_lr[i] - o.obj) <= 1e-6 * abs(o.obj)


def test_lowrank_least_squares_uncentred(device):
    n, T = 600, 120
    ends = [200, 333]
    dates, R, y, sec, pan, r_d, t_d, _ = _setup(n, T, ends, centred=False, D=400)
    B = len(ends)
    qb = engine.QPBatch.from_dense(np.zeros((1, n, n)), np.zeros((1, n)), A=np.ones((1, n)), b=np.ones(1),
                                   lb=np.zeros(n), ub=np.full(n, 0.05), device=device)
    qb.batch = B
    qb.P = pan.cov(r_d, t_d, mode=1)
    xty, _ = pan.gram_xy(r_d, t_d)
    qb.q = (-2.0 * xty).contiguous()
    qb.p_scale = torch.full((B,), 2.0, dtype=torch.float64, device=device)
    lr = engine.LowRank(pan, r_d, t_d, mu=None)
    res = engine.solve_lowrank(qb, lr, engine.Settings(rho0_rel=0.5))
    x = res.x.cpu().numpy().copy()
    assert np.all(res.status.cpu().numpy() == 1)
    res_d = engine.solve(qb, engine.Settings(rho0_rel=0.5))
    assert np.all(res_d.status.cpu().numpy() == 1)
    # flat optimal face (see below): rounding differences between the two K^-1 forms move
    # the iterates along it, so the paths agree to the weight tolerance, not to 1e-9
    assert np.abs(x - res_d.x.cpu().numpy()).max() < 1e-5
    for i, e in enumerate(ends):
        X = R[e - T + 1:e + 1]
        P, q = 2 * X.T @ X, -2 * X.T @ y[e - T + 1:e + 1]
        o = solve_qp(P, q, A=np.ones((1, n)), b=np.ones(1), lb=np.zeros(n), ub=np.full(n, 0.05))
        # rank(P) <= T = 120 < n = 600: the minimiser is a face, not a point, so the oracle
        # and the engine may return different optimal x -- compare value and feasibility.
        assert abs((0.5 * x[i] @ P @ x[i] + q @ x[i]) - o.obj) <= 1e-6 * abs(o.obj)
        assert abs(x[i].sum() - 1.0) <= 1e-7
        assert x[i].min() >= -1e-7 and x[i].max() <= 0.05 + 1e-7


@pytest.mark.parametrize("n,T,D,stride,groups_rows", [(300, 120, 40, 1, False), (300, 120, 40, 1, True),
                                                      (1000, 252, 35, 1, False), (200, 60, 24, 5, True)])
def test_grouped_admm_matches_per_date_lowrank(device, n, T, D, stride, groups_rows):
    """pq_admm_lr_grouped (one workgroup per group of sliding windows, MFMA passes over the
    union rows) reaches the same iterates as the per-date low-rank kernel: the same
    iteration counts up to rounding and the same polished weights."""
    ends = list(range(T + 5, T + 5 + D * stride, stride))
    dates, R, y, sec, pan, r_d, t_d, mu = _setup(n, T, ends, D=max(ends) + 1)
    rows, tlen = engine.window_rows(dates, dates[ends], T)
    B = len(ends)
    G = h = None
    if groups_rows:
        G = np.stack([(sec == g).astype(float) for g in range(3)])
        h = np.full(3, 0.3)
    qb = engine.QPBatch.from_dense(np.zeros((1, n, n)), np.zeros((1, n)), A=np.ones((1, n)), b=np.ones(1),
                                   G=G, h=h, lb=np.zeros(n), ub=np.full(n, 0.2), device=device)
    qb.batch = B
    # the bench layout: sliding K1 writing the lower triangle only (upper tiles stay NaN --
    # nothing on the low-rank path may read them)
    Pbuf = torch.full((B, qb.ld, qb.ld), float("nan"), dtype=torch.float64, device=device)
    qb.P = pan.cov(r_d, t_d, mode=0, mu=mu, out=Pbuf, plan=engine.SlidePlan(rows, tlen, device),
                   lower_only=True)
    qb.q = torch.zeros((B, qb.ld), dtype=torch.float64, device=device)
    qb.p_scale = torch.full((B,), 2.0, dtype=torch.float64, device=device)
    lr = engine.LowRank(pan, r_d, t_d, mu=mu, w_scale=1.0 / (t_d.to(torch.float64) - 1.0))
    gp = engine.GroupPlan(rows, tlen, device)
    assert gp.ok and gp.ngroups < B
    ws_g = engine.Workspace(qb)
    assert engine.grouped_applicable(qb, lr, gp, ws_g)
    st0 = engine.Settings(eps_grouped=0.0)   # both paths stop ADMM at eps_abs: same iteration counts
    res_g = engine.solve_lowrank(qb, lr, st0, ws=ws_g, groups=gp)
    xg, itg, stg = res_g.x.cpu().numpy().copy(), res_g.iters.cpu().numpy().copy(), res_g.status.cpu().numpy().copy()
    res_d = engine.solve_lowrank(qb, lr, st0)
    xd, itd = res_d.x.cpu().numpy(), res_d.iters.cpu().numpy()
    assert np.all(stg == 1) and np.all(res_d.status.cpu().numpy() == 1)
    assert np.abs(itg - itd).max() <= 2, (itg, itd)
    assert np.abs(xg - xd).max() < 1e-8
    assert np.abs(xg.sum(1) - 1).max() < 1e-9 and xg.min() > -1e-9 and xg.max() < 0.2 + 1e-9
    for i in (0, B - 1):
        e = ends[i]
        P = 2 * cov_pearson(R[e - T + 1:e + 1])
        o = solve_qp(P, np.zeros(n), G=G, h=h, A=np.ones((1, n)), b=np.ones(1), lb=np.zeros(n),
                     ub=np.full(n, 0.2))
        assert abs(0.5 * xg[i] @ P @ xg[i] - o.obj) <= 1e-6 * abs(o.obj)


@pytest.mark.parametrize("centred,groups_rows,stride", [(True, False, 1), (True, True, 3), (False, True, 1)])
def test_band_gram_capacitance_matches_direct(device, centred, groups_rows, stride):
    """pq_lr_capacitance_band (M from the panel's row band Gram, shared by overlapping
    windows) builds the same capacitance matrices as the per-date MFMA SYRK
    pq_lr_capacitance, and the solve reaches the same optimum."""
    n, T, D = 400, 120, 30
    ends = list(range(T + 5, T + 5 + D * stride, stride))
    dates, R, y, sec, pan, r_d, t_d, mu = _setup(n, T, ends, centred=centred, D=max(ends) + 1)
    B = len(ends)
    G = h = None
    if groups_rows:
        G = np.stack([(sec == g).astype(float) for g in range(3)])
        h = np.full(3, 0.4)
    qb = engine.QPBatch.from_dense(np.zeros((1, n, n)), np.zeros((1, n)), A=np.ones((1, n)), b=np.ones(1),
                                   G=G, h=h, lb=np.zeros(n), ub=np.full(n, 0.1), device=device)
    qb.batch = B
    qb.P = None
    qb.q = torch.zeros((B, qb.ld), dtype=torch.float64, device=device)
    qb.p_scale = torch.full((B,), 2.0, dtype=torch.float64, device=device)
    w = 1.0 / (t_d.to(torch.float64) - 1.0) if centred else None
    lr = engine.LowRank(pan, r_d, t_d, mu=mu, w_scale=w)
    lib = engine._lib.load()
    ws = engine.Workspace(qb, dense=False)
    import ctypes
    P_, S_ = ctypes.byref(qb.c_struct()), ctypes.byref(ws.c_struct())
    L_ = ctypes.byref(lr.c_struct())
    SS = ctypes.byref(engine.Settings().to_c())
    strm = engine._stream()
    engine._lib.check(lib.pq_init_state_lr(L_, P_, S_, None, 0, SS, strm), "init")
    k_ld = engine.round_up(lr.tmax + qb.mg, 64)
    M1 = torch.zeros((B, k_ld, k_ld), dtype=torch.float64, device=device)
    M2 = torch.zeros_like(M1)
    engine._lib.check(lib.pq_lr_capacitance(L_, P_, S_, None, 0, SS, M1.data_ptr(), k_ld, k_ld * k_ld, strm), "direct")
    bd = engine._band_setup(qb, lr, strm)
    assert bd is not None
    engine._lib.check(lib.pq_lr_capacitance_band(L_, P_, S_, None, 0, SS, bd["band"].data_ptr(), bd["ldo"], bd["r0"],
                                                 bd["pc"].data_ptr(), bd["pc"].stride(0), bd["cc"].data_ptr(),
                                                 M2.data_ptr(), k_ld, k_ld * k_ld, strm), "band")
    lower = torch.tril(torch.ones(k_ld, k_ld, dtype=torch.bool, device=device))
    d = ((M1 - M2).abs() * lower).amax().item()
    assert d <= 1e-12 * M1.abs().amax().item(), d
    r1 = engine.solve_lowrank(qb, lr, band=False)
    x1, i1 = r1.x.cpu().numpy().copy(), r1.iters.cpu().numpy().copy()
    r2 = engine.solve_lowrank(qb, lr, band=True)
    assert np.all(r2.status.cpu().numpy() == 1) and np.all(r1.status.cpu().numpy() == 1)
    assert np.abs(r2.iters.cpu().numpy() - i1).max() <= 2
    assert np.abs(r2.x.cpu().numpy() - x1).max() < 1e-8


@pytest.mark.parametrize("n,T,D,stride,groups_rows,centred", [(1000, 252, 40, 1, False, True),
                                                               (300, 120, 40, 2, True, True),
                                                               (400, 100, 30, 1, True, False)])
def test_grouped_fused_matches_unfused(device, n, T, D, stride, groups_rows, centred):
    """The fused grouped ADMM (uniform D: Cg x~ from the band tables, one pass per date)
    follows the unfused kernel's iterates and reaches the same polished weights."""
    ends = list(range(T + 5, T + 5 + D * stride, stride))
    dates, R, y, sec, pan, r_d, t_d, mu = _setup(n, T, ends, centred=centred, D=max(ends) + 1)
    rows, tlen = engine.window_rows(dates, dates[ends], T)
    B = len(ends)
    G = h = None
    if groups_rows:
        G = np.stack([(sec == g).astype(float) for g in range(3)])
        h = np.full(3, 0.35)
    qb = engine.QPBatch.from_dense(np.zeros((1, n, n)), np.zeros((1, n)), A=np.ones((1, n)), b=np.ones(1),
                                   G=G, h=h, lb=np.zeros(n), ub=np.full(n, 0.15), device=device)
    qb.batch = B
    qb.P = None
    qb.q = torch.zeros((B, qb.ld), dtype=torch.float64, device=device)
    qb.p_scale = torch.full((B,), 2.0, dtype=torch.float64, device=device)
    w = 1.0 / (t_d.to(torch.float64) - 1.0) if centred else None
    lr = engine.LowRank(pan, r_d, t_d, mu=mu, w_scale=w)
    gp = engine.GroupPlan(rows, tlen, device)
    st0 = engine.Settings(eps_grouped=0.0)   # both forms stop ADMM at eps_abs: same iteration counts
    r1 = engine.solve_lowrank(qb, lr, st0, groups=gp, fuse=False)
    x1, i1 = r1.x.cpu().numpy().copy(), r1.iters.cpu().numpy().copy()
    assert r1.capacitance == "band"
    r2 = engine.solve_lowrank(qb, lr, st0, groups=gp, fuse=True)
    assert np.all(r1.status.cpu().numpy() == 1) and np.all(r2.status.cpu().numpy() == 1)
    assert np.abs(r2.iters.cpu().numpy() - i1).max() <= 2
    assert np.abs(r2.x.cpu().numpy() - x1).max() < 1e-8


@pytest.mark.parametrize("path", ["window", "dense"])
def test_polish_rejection_resumes_admm_to_tight_eps(device, path):
    """ADMM stops at eps 1e-4 for the polish; a problem whose polish is rejected (forced
    here with a single active-set round) resumes ADMM to eps_retry from its iterate and is
    polished again -- it ends SOLVED at the same optimum as the default settings."""
    n, T, D = 300, 100, 12
    ends = list(range(T + 5, T + 5 + D))
    dates, R, y, sec, pan, r_d, t_d, mu = _setup(n, T, ends, D=max(ends) + 1)
    rows, tlen = engine.window_rows(dates, dates[ends], T)
    qb = engine.QPBatch.from_dense(np.zeros((1, n, n)), np.zeros((1, n)), A=np.ones((1, n)), b=np.ones(1),
                                   lb=np.zeros(n), ub=np.full(n, 0.1), device=device)
    qb.batch = D
    qb.q = torch.zeros((D, qb.ld), dtype=torch.float64, device=device)
    qb.p_scale = torch.full((D,), 2.0, dtype=torch.float64, device=device)
    qb.p_diag = torch.full((D,), 1e-4, dtype=torch.float64, device=device)   # P > 0: a unique optimum
    if path == "dense":
        qb.P = pan.cov(r_d, t_d, mode=0, mu=mu)
        run = lambda st: engine.solve(qb, st)
    else:
        qb.P = None
        lr = engine.LowRank(pan, r_d, t_d, mu=mu, w_scale=1.0 / (t_d.to(torch.float64) - 1.0))
        gp = engine.GroupPlan(rows, tlen, device)
        run = lambda st: engine.solve_lowrank(qb, lr, st, groups=gp)
    ref = run(engine.Settings())
    x0 = ref.x.cpu().numpy().copy()
    assert np.all(ref.status.cpu().numpy() == 1)
    one = run(engine.Settings(polish_rounds=1))
    st = one.status.cpu().numpy()
    assert np.all(st == 1), st
    assert one.iters.cpu().numpy().max() > ref.iters.cpu().numpy().max()   # the retry ran
    assert np.abs(one.x.cpu().numpy() - x0).max() < 1e-8


@pytest.mark.gpu
def test_workspace_bytes_matches_the_allocation(device):
    """pq_workspace_bytes (the C-ABI size query) equals what engine.Workspace allocates."""
    from porqua_amd import _lib
    n, B, T = 1000, 5, 252
    qb = engine.QPBatch.from_dense(np.zeros((1, n, n)), np.zeros((1, n)), A=np.ones((1, n)), b=np.ones(1),
                                   lb=np.zeros(n), ub=np.ones(n), device=device)
    qb.batch = B
    lib = _lib.load()
    for dense in (True, False):
        ws = engine.Workspace(qb, dense=dense)
        ts = [ws.K, ws.Dt, ws.x, ws.Px, ws.z, ws.y, ws.rho, ws.iters, ws.status, ws.info, ws.out, ws.work]
        if not dense:
            lrb = ws.lr_buffers(engine.round_up(T + qb.mg, 64))
            ts += [lrb[k] for k in ("M", "Minv", "Dt", "iters", "status", "info")]
        got = sum(t.numel() * t.element_size() for t in ts)
        assert lib.pq_workspace_bytes(n, B, qb.mg, 0 if dense else 1, T, ws.ldk) == got
