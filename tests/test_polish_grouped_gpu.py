"""The grouped polish pipeline (polish_g.hip: per-round setup / form / LDS solve kernels and
MFMA window passes over each slide group's union rows) against the per-date window polish
it restructures (polish_w.hip, pq_polish_w_batched): same ADMM point in, the same polished
weights, statuses, objective and multipliers out (to rounding), on the shapes the
backtests use -- long-only min-variance at n = 1000 (bench), capped boxes (fixed weights at
an upper bound: the P x_B pass), sector caps (active general rows), uncentred least
squares, free sets beyond the LDS solve (the pipeline's large-free-set solve up to the K
scratch's 256, the per-date kernel beyond).  The grouped
side forms P_FF from one union Gram per polish group where at least three of its dates form
in a round (k_pg_form_grp), so these cases also pin that derivation against the per-date
window products."""
import numpy as np
import pytest
import torch

from porqua_amd import _lib, engine
from porqua_amd.synthetic import factor_panel

pytestmark = pytest.mark.gpu


def _problem(device, n, T, D, ub, ngroups_rows=0, cap=0.3, centred=True, stride=1, seed=None):
    ends = list(range(T + 5, T + 5 + D * stride, stride))
    dates, R, y, sec = factor_panel(max(ends) + 1, n, **({} if seed is None else {"seed": seed}))
    rows, tlen = engine.window_rows(dates, dates[ends], T)
    pan = engine.Panel(R, y, device=device)
    r_d, t_d = pan.rows_to_device(rows, tlen)
    G = h = None
    if ngroups_rows:
        G = np.stack([(sec == g).astype(float) for g in range(ngroups_rows)])
        h = np.full(ngroups_rows, cap)
    qb = engine.QPBatch.from_dense(np.zeros((1, n, n)), np.zeros((1, n)), A=np.ones((1, n)), b=np.ones(1),
                                   G=G, h=h, lb=np.zeros(n), ub=np.full(n, ub), device=device)
    qb.batch = D
    qb.P = None
    qb.p_scale = torch.full((D,), 2.0, dtype=torch.float64, device=device)
    if centred:
        mu = pan.window_means(r_d, t_d)
        qb.q = torch.zeros((D, qb.ld), dtype=torch.float64, device=device)
        lr = engine.LowRank(pan, r_d, t_d, mu=mu, w_scale=1.0 / (t_d.to(torch.float64) - 1.0))
    else:
        xty, _ = pan.gram_xy(r_d, t_d)
        qb.q = (-2.0 * xty).contiguous()
        lr = engine.LowRank(pan, r_d, t_d, mu=None)
    gp = engine.GroupPlan(rows, tlen, device)
    return qb, lr, gp


def _solve(qb, lr, gp, grouped_polish, settings=None, eps_grouped=0.0, polish_fix_rel=0.0, polish_inner=0):
    """(wide rounds off: this file pins the LDS-solve pipeline against the per-date kernel;
    tests/test_polish_wide_gpu.py covers the wide rounds.  The looser ADMM stop before the
    pipeline (Settings.eps_grouped), the pipeline's extra lower-bound classification
    (Settings.polish_fix_rel) and its inner primal steps (Settings.polish_inner) are off unless
    asked for: both sides start from the same ADMM point and take the same active sets.)"""
    import dataclasses
    settings = dataclasses.replace(settings or engine.Settings(), eps_grouped=eps_grouped,
                                   polish_fix_rel=polish_fix_rel, polish_inner=polish_inner)
    ws = engine.Workspace(qb, dense=False)
    assert engine.grouped_applicable(qb, lr, gp, ws)
    res = engine.solve_lowrank(qb, lr, settings, ws=ws, groups=gp, grouped_polish=grouped_polish,
                               wide_polish=False)
    torch.cuda.synchronize()
    rec = ws.pg_record()[:, _lib.PQ_PG_STATE].cpu().numpy().copy() if grouped_polish else None
    return (res.x.cpu().numpy().copy(), res.status.cpu().numpy().copy(), res.obj.cpu().numpy().copy(),
            res.y.cpu().numpy().copy(), res.z_box.cpu().numpy().copy(), res.out.cpu().numpy().copy(), rec)


@pytest.mark.parametrize("case", ["bench", "capped", "sectors", "lsq", "uncentred_q0", "small_T"])
def test_grouped_polish_matches_per_date_polish(device, case):
    if case == "bench":
        qb, lr, gp = _problem(device, 1000, 252, 48, 1.0)
        settings = None
    elif case == "capped":
        qb, lr, gp = _problem(device, 400, 120, 40, 0.05)
        settings = None
    elif case == "sectors":
        qb, lr, gp = _problem(device, 600, 150, 36, 0.2, ngroups_rows=5, cap=0.25, stride=2)
        settings = None
    elif case == "lsq":
        qb, lr, gp = _problem(device, 500, 120, 30, 0.1, centred=False)
        settings = engine.Settings(rho0_rel=0.5)
    elif case == "uncentred_q0":   # uncentred Gram, q = 0 (minimum second moment): sparse free sets
        qb, lr, gp = _problem(device, 600, 150, 40, 1.0, centred=False)   # inside the LDS solve, no mean
        qb.q.zero_()
        settings = None
    else:
        qb, lr, gp = _problem(device, 300, 60, 40, 1.0)
        settings = None
    xa, sa, oa, ya, za, outa, _ = _solve(qb, lr, gp, False, settings)
    xb, sb, ob, yb, zb, outb, rec = _solve(qb, lr, gp, True, settings)
    assert np.array_equal(sa, sb), (sa, sb)
    assert np.all(sb == _lib.PQ_SOLVED)
    # most dates go through the pipeline (the rest fall back to the per-date kernel); the
    # tracking problem's free sets exceed the LDS solve (k > 128), so it all falls back
    if case != "lsq":
        assert (rec == _lib.PQ_PG_DONE).mean() >= 0.8, np.unique(rec, return_counts=True)
    assert np.all((rec == _lib.PQ_PG_DONE) | (rec == _lib.PQ_PG_FALLBACK))
    assert np.abs(xa - xb).max() <= 1e-10, np.abs(xa - xb).max()
    assert np.abs(oa - ob).max() <= 1e-12 * max(1.0, np.abs(oa).max()) + 1e-15
    sc = max(np.abs(ya).max(), np.abs(za).max(), 1e-30)
    assert np.abs(ya - yb).max() <= 1e-8 * sc and np.abs(za - zb).max() <= 1e-8 * sc
    # the same free sets and rounds as the per-date kernel
    assert np.array_equal(outa[:, _lib.PQ_OUT_NFREE], outb[:, _lib.PQ_OUT_NFREE])
    assert np.abs(outa[:, _lib.PQ_OUT_PRIM] - outb[:, _lib.PQ_OUT_PRIM]).max() <= 1e-12


def test_grouped_polish_hands_large_free_sets_to_the_per_date_kernel(device):
    """Free sets beyond the K scratch of the pipeline (k > ldk = 256: the tracking problem holds
    most of its 500 assets strictly inside the box) are FALLBACK problems and still end SOLVED
    with the per-date kernel's answer."""
    qb, lr, gp = _problem(device, 500, 120, 30, 0.1, centred=False)
    st_ = engine.Settings(rho0_rel=0.5)
    xa, sa, oa, *_ = _solve(qb, lr, gp, False, st_)
    xb, sb, ob, _, _, outb, rec = _solve(qb, lr, gp, True, st_)
    assert np.array_equal(sa, sb)
    assert np.abs(xa - xb).max() <= 1e-10
    big = outb[:, _lib.PQ_OUT_NFREE] > 256
    assert big.any()
    assert np.all(rec[big] == _lib.PQ_PG_FALLBACK)


def test_large_free_sets_are_solved_inside_the_pipeline(device):
    """Free sets between the LDS solve and the K scratch (128 < k <= 256: a ridge keeps most of
    400 assets strictly inside the box, as the tracking windows of configs 1/2 do with 160..220
    free assets) go through the grouped large-free-set solve (k_pg_big: P_FF formed from the
    window, MFMA tile Cholesky, Schur complement, proximal refinement) instead of the per-date
    kernel, and give its answers to rounding."""
    qb, lr, gp = _problem(device, 400, 100, 24, 1.0)
    qb.p_diag = torch.full((qb.batch,), 5e-3, dtype=torch.float64, device=device)
    xa, sa, oa, ya, za, outa, _ = _solve(qb, lr, gp, False)
    xb, sb, ob, yb, zb, outb, rec = _solve(qb, lr, gp, True)
    assert np.all(sa == _lib.PQ_SOLVED) and np.array_equal(sa, sb)
    k = outb[:, _lib.PQ_OUT_NFREE]
    assert ((k > 128) & (k <= 256)).mean() >= 0.5, k
    assert np.all(rec == _lib.PQ_PG_DONE), np.unique(rec, return_counts=True)
    assert np.abs(xa - xb).max() <= 1e-10, np.abs(xa - xb).max()
    assert np.abs(oa - ob).max() <= 1e-12 * max(1.0, np.abs(oa).max()) + 1e-15
    sc = max(np.abs(ya).max(), np.abs(za).max(), 1e-30)
    assert np.abs(ya - yb).max() <= 1e-8 * sc and np.abs(za - zb).max() <= 1e-8 * sc
    assert np.array_equal(outa[:, _lib.PQ_OUT_NFREE], k)


def test_large_free_sets_from_the_group_gram(device):
    """Uncentred windows with free sets of 129..256 (config 2's SPTR tracking on the usa-shaped
    panel, 24 consecutive daily dates: about 190 of 494 assets free): the pipeline forms each
    date's P_FF from one Gram of its polish group's union rows over the union of the group's
    free lists minus the date's outside rows (k_pg_form_grp_big + k_pg_form<256>) instead of
    from its whole window, and gives the per-date kernel's answers to rounding."""
    import dataclasses
    from tests.conftest import load_golden
    from porqua_amd.workloads import ReplicationBacktest
    g = load_golden("sptr")
    wl = ReplicationBacktest(g["days"], g["returns"], n_rows=252 + 23, device=device)
    xty, _ = wl.pan.gram_xy(wl.rows_d, wl.tlen_d)
    torch.mul(xty, -2.0, out=wl.qb.q)
    qb, lr, gp = wl.qb, wl.lr, wl.gplan
    xa, sa, oa, ya, za, outa, _ = _solve(qb, lr, gp, False, settings=wl.settings)
    st = dataclasses.replace(wl.settings, eps_grouped=0.0, polish_fix_rel=0.0, polish_inner=0)
    ws = engine.Workspace(qb, dense=False)
    res = engine.solve_lowrank(qb, lr, st, ws=ws, groups=gp, grouped_polish=True, wide_polish=False)
    torch.cuda.synchronize()
    rec = ws.pg_record().cpu().numpy()
    xb, sb, ob, outb = (res.x.cpu().numpy(), res.status.cpu().numpy(), res.obj.cpu().numpy(),
                        res.out.cpu().numpy())
    assert np.all(sa == _lib.PQ_SOLVED) and np.array_equal(sa, sb)
    k = outb[:, _lib.PQ_OUT_NFREE]
    assert ((k > 128) & (k <= 256)).mean() >= 0.5, k
    assert np.all(rec[:, _lib.PQ_PG_STATE] == _lib.PQ_PG_DONE)
    assert (rec[:, 348] > 0).any()   # R_GFORM: some date's last round formed from its group's Gram
    assert np.abs(xa - xb).max() <= 1e-10, np.abs(xa - xb).max()
    assert np.abs(oa - ob).max() <= 1e-12 * max(1.0, np.abs(oa).max()) + 1e-15
    assert np.array_equal(outa[:, _lib.PQ_OUT_NFREE], k)


def test_loose_admm_stop_before_the_pipeline(device):
    """Settings.eps_grouped (centred windows, default 0.5 with at least min_iter_grouped = 7 iterations): the ADMM stops early and the
    pipeline's rounds finish the job -- the same optimum as from the eps_abs point, fewer
    ADMM iterations, every date SOLVED."""
    qb, lr, gp = _problem(device, 1000, 252, 48, 1.0)
    xa, sa, oa, *_ = _solve(qb, lr, gp, True)
    d = engine.Settings()
    assert d.eps_grouped > d.eps_abs
    ws = engine.Workspace(qb, dense=False)
    res = engine.solve_lowrank(qb, lr, None, ws=ws, groups=gp)
    torch.cuda.synchronize()
    assert np.all(res.status.cpu().numpy() == _lib.PQ_SOLVED)
    ob = res.obj.cpu().numpy()
    assert np.max(np.abs(ob - oa) / np.maximum(np.abs(oa), 1e-30)) <= 1e-9
    ws0 = engine.Workspace(qb, dense=False)
    import dataclasses
    engine.solve_lowrank(qb, lr, dataclasses.replace(d, eps_grouped=0.0), ws=ws0, groups=gp)
    torch.cuda.synchronize()
    assert ws.iters.float().mean().item() < ws0.iters.float().mean().item()


def test_loose_admm_stop_resumes_the_hand_offs(device):
    """Dates the pipeline hands to the per-date kernel (a strong ridge keeps every asset
    strictly inside the box: free sets beyond the K scratch, k = n = 800 > 256) resume ADMM to
    eps_abs before that polish, so the answer is the one from the eps_abs point."""
    qb, lr, gp = _problem(device, 800, 100, 24, 1.0)
    qb.p_diag = torch.full((qb.batch,), 5e-2, dtype=torch.float64, device=device)
    xa, sa, *_ = _solve(qb, lr, gp, True)
    xb, sb, _, _, _, outb, rec = _solve(qb, lr, gp, True, eps_grouped=2e-2)
    assert np.all(sa == _lib.PQ_SOLVED) and np.array_equal(sa, sb)
    assert (rec == _lib.PQ_PG_FALLBACK).mean() >= 0.5, np.unique(rec, return_counts=True)
    assert np.abs(xa - xb).max() <= 1e-9, np.abs(xa - xb).max()


@pytest.mark.parametrize("case", ["bench", "capped", "sectors", "small_T"])
def test_fix_rel_classification_same_optimum(device, case):
    """Settings.polish_fix_rel (the default 0.1): small ADMM weights start fixed at the
    lower bound -- a different first active set, the same certified optimum (to the proximal
    refinement's accuracy)."""
    args = {"bench": (1000, 252, 48, 1.0), "capped": (400, 120, 40, 0.05),
            "sectors": (600, 150, 36, 0.2), "small_T": (300, 60, 40, 1.0)}[case]
    kw = dict(ngroups_rows=5, cap=0.25, stride=2) if case == "sectors" else {}
    qb, lr, gp = _problem(device, *args, **kw)
    d = engine.Settings()
    assert d.polish_fix_rel > 0
    xa, sa, oa, *_ = _solve(qb, lr, gp, True)
    xb, sb, ob, _, _, outb, rec = _solve(qb, lr, gp, True, polish_fix_rel=d.polish_fix_rel)
    assert np.all(sa == _lib.PQ_SOLVED) and np.all(sb == _lib.PQ_SOLVED)
    assert (rec == _lib.PQ_PG_DONE).mean() >= 0.8, np.unique(rec, return_counts=True)
    assert np.abs(xa - xb).max() <= 1e-8, np.abs(xa - xb).max()
    assert np.max(np.abs(ob - oa) / np.maximum(np.abs(oa), 1e-30)) <= 1e-12


def test_inner_primal_steps_same_optimum_fewer_rounds(device):
    """Settings.polish_inner (k_pg_solve fixes the free variables its solve leaves outside the
    box and re-solves the reduced system inside the round): the bench shape with the bench's
    settings (loose ADMM stop, first-active-set rule) reaches the same certified optimum as one
    solve per round, in no more rounds on average."""
    qb, lr, gp = _problem(device, 1000, 252, 48, 1.0)
    d = engine.Settings()
    assert d.polish_inner > 0
    runs = {}
    for inner in (0, d.polish_inner):
        runs[inner] = _solve(qb, lr, gp, True, d, eps_grouped=d.eps_grouped, polish_fix_rel=d.polish_fix_rel,
                             polish_inner=inner)
    xa, sa, oa, _, _, outa, reca = runs[0]
    xb, sb, ob, _, _, outb, recb = runs[d.polish_inner]
    assert np.all(sa == _lib.PQ_SOLVED) and np.array_equal(sa, sb)
    assert np.all(recb == _lib.PQ_PG_DONE), np.unique(recb, return_counts=True)
    assert np.abs(xa - xb).max() <= 1e-9, np.abs(xa - xb).max()
    assert np.abs(oa - ob).max() <= 1e-10 * max(1.0, np.abs(oa).max())
    assert np.array_equal(outa[:, _lib.PQ_OUT_NFREE], outb[:, _lib.PQ_OUT_NFREE])
    ra, rb = outa[:, _lib.PQ_OUT_ROUNDS], outb[:, _lib.PQ_OUT_ROUNDS]
    assert rb.mean() <= ra.mean(), (ra.mean(), rb.mean())


def test_vertex_overshoot_is_released(device):
    """The drop-in's mean-variance problem (config-3 panel, q = -mu geometric: nearly linear,
    ~3 free assets per date): a round that fixes two weights past their upper bound of 1 at
    once leaves a vertex whose bound values overshoot the budget; the post releases them
    (k_pg_post) instead of repeating that infeasible active set until the hand-off.  Every date
    stays in the pipeline and matches the per-date polish from the eps_abs point."""
    from porqua_amd.workloads import MinVarianceBacktest
    wl = MinVarianceBacktest(D=4749, device=device)
    n = wl.n
    wl.qb.q[:, :n] = -wl.pan.window_geomeans_grouped(wl.gplan, wl.tlen_d)[:, :n]
    ws = engine.Workspace(wl.qb, dense=False)
    res = engine.solve_lowrank(wl.qb, wl.lr, wl.settings, ws=ws, groups=wl.gplan, sync_free=True, sf_rounds=4)
    torch.cuda.synchronize()
    fb = getattr(ws, "pg_fallback", None)
    assert fb is None or fb.numel() == 0, fb
    sa = res.status.cpu().numpy()
    assert np.all(sa == _lib.PQ_SOLVED)
    oa = res.obj.cpu().numpy().copy()
    ws0 = engine.Workspace(wl.qb, dense=False)
    import dataclasses
    r0 = engine.solve_lowrank(wl.qb, wl.lr, dataclasses.replace(wl.settings, eps_grouped=0.0), ws=ws0,
                              groups=wl.gplan, grouped_polish=False)
    torch.cuda.synchronize()
    o0 = r0.obj.cpu().numpy()
    assert np.all(r0.status.cpu().numpy() == _lib.PQ_SOLVED)
    assert np.max(np.abs(oa - o0) / np.maximum(np.abs(o0), 1e-30)) <= 1e-8


def test_loose_stop_waits_for_min_iter(device):
    """pq_settings.min_iter: the loose ADMM stop before the grouped polish is not taken before
    Settings.min_iter_grouped iterations even when the residuals already pass a very loose eps
    (ADMM's early residuals dip and rise again); the answers stay the certified optimum."""
    import dataclasses
    qb, lr, gp = _problem(device, 1000, 252, 48, 1.0)
    d = engine.Settings()
    assert d.min_iter_grouped >= 1
    xa, sa, oa, *_ = _solve(qb, lr, gp, True)
    ws = engine.Workspace(qb, dense=False)
    res = engine.solve_lowrank(qb, lr, dataclasses.replace(d, eps_grouped=10.0), ws=ws, groups=gp)
    torch.cuda.synchronize()
    it = res.iters.cpu().numpy()
    assert it.min() >= d.min_iter_grouped, it.min()
    assert np.all(res.status.cpu().numpy() == _lib.PQ_SOLVED)
    ob = res.obj.cpu().numpy()
    assert np.max(np.abs(ob - oa) / np.maximum(np.abs(oa), 1e-30)) <= 1e-9
