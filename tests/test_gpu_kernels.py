"""GPU parity of the HIP kernels against the CPU oracle (run on an MI355X: -m gpu)."""
import numpy as np
import pytest
import torch

from oracle.ref_pipeline import cov_pearson, window_rows as oracle_window_rows
from oracle.qp_ipm import solve_qp
from porqua_amd import engine
from porqua_amd.synthetic import factor_panel
from tests.conftest import load_golden

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300)


@pytest.mark.parametrize("n,T,D", [(24, 252, 400), (100, 60, 200), (130, 40, 120)])
def test_cov_and_gram_match_numpy(device, n, T, D):
    dates, R, y, _ = factor_panel(D, n, seed=n)
    reb = dates[T::7][:9]
    rows, tlen = engine.window_rows(dates, reb, T)
    pan = engine.Panel(R, y, device=device)
    r_d, t_d = pan.rows_to_device(rows, tlen)
    S = pan.cov(r_d, t_d, mode=0).cpu().numpy()
    G = pan.cov(r_d, t_d, mode=1).cpu().numpy()
    xty, yty = pan.gram_xy(r_d, t_d)
    xty, yty = xty.cpu().numpy(), yty.cpu().numpy()
    for b, rd in enumerate(reb):
        rr = oracle_window_rows(dates, rd, T)
        assert np.array_equal(rr, rows[b, :tlen[b]])
        X = R[rr]
        assert _rel(S[b, :n, :n], cov_pearson(X)) < 1e-12
        assert _rel(G[b, :n, :n], X.T @ X) < 1e-12
        assert _rel(xty[b, :n], X.T @ y[rr]) < 1e-12
        assert abs(yty[b] - y[rr] @ y[rr]) <= 1e-12 * abs(yty[b])
        assert np.all(S[b, n:, :] == 0) and np.all(S[b, :, n:] == 0)


@pytest.mark.parametrize("n,T,stride,offset", [(24, 252, 1, 0.0), (130, 60, 1, 0.0), (200, 252, 21, 0.0),
                                               (70, 40, 3, 50.0)])
def test_sliding_cov_matches_full_syrk_and_numpy(device, n, T, stride, offset):
    """pq_cov_slide_batched (anchor SYRK + rank-2s updates) == pq_cov_batched == np.cov;
    offset: price-like data with a large common mean (the shift keeps it exact)."""
    D = T + 70 * stride
    dates, R, y, _ = factor_panel(D, n, seed=n + stride)
    R = R + offset
    reb = dates[T - 1::stride][:70]
    rows, tlen = engine.window_rows(dates, reb, T)
    plan = engine.SlidePlan(rows, tlen, device, group=16)
    assert plan.ngroups < len(reb)
    pan = engine.Panel(R, y, device=device)
    r_d, t_d = pan.rows_to_device(rows, tlen)
    for mode in (0, 1):
        full = pan.cov(r_d, t_d, mode=mode).cpu().numpy()
        sl = pan.cov(r_d, t_d, mode=mode, plan=plan).cpu().numpy()
        gs = plan.gstart.cpu().numpy()
        assert np.array_equal(full[gs[:-1]], sl[gs[:-1]])          # anchors: same arithmetic
        lo = torch.full_like(torch.from_numpy(sl), float("nan")).to(device)
        lo = pan.cov(r_d, t_d, mode=mode, plan=plan, out=lo, lower_only=True).cpu().numpy()
        ld = lo.shape[-1]
        tile = np.arange(ld) // 64
        upper = tile[:, None] < tile[None, :]                          # strictly-upper 64x64 tiles
        assert np.array_equal(lo[:, ~upper], sl[:, ~upper]) and np.isnan(lo[:, upper]).all()
        for b in range(len(reb)):
            X = R[rows[b, :tlen[b]]]
            ref = cov_pearson(X) if mode == 0 else X.T @ X
            assert _rel(sl[b, :n, :n], ref) < 1e-12, (mode, b, _rel(sl[b, :n, :n], ref))
            assert np.array_equal(sl[b, :n, :n], sl[b, :n, :n].T)
            assert np.all(sl[b, n:, :] == 0) and np.all(sl[b, :, n:] == 0)


@pytest.mark.parametrize("n", [24, 64, 150, 300])
def test_factor_and_inverse(device, n):
    rng = np.random.default_rng(n)
    B = 3
    M = rng.standard_normal((B, n + 7, n))
    P = np.einsum("bki,bkj->bij", M, M) / n + 0.1 * np.eye(n)
    qb = engine.QPBatch.from_dense(P, np.zeros((B, n)), device=device)
    ws, info = engine.factor_only(qb, invert=False)
    assert int(info.abs().max()) == 0
    L = torch.tril(ws.K).cpu().numpy()[:, :n, :n]
    for b in range(B):
        assert _rel(L[b], np.linalg.cholesky(P[b])) < 1e-12
    ws, info = engine.factor_only(qb, invert=True)
    Ki = ws.K.cpu().numpy()[:, :n, :n]
    for b in range(B):
        assert _rel(Ki[b], np.linalg.inv(P[b])) < 1e-10
    # a non-PD matrix reports info > 0 (the isPD test)
    P[1] = -P[1]
    qb = engine.QPBatch.from_dense(P, np.zeros((B, n)), device=device)
    _, info = engine.factor_only(qb)
    info = info.cpu().numpy()
    assert info[0] == 0 and info[1] == 1 and info[2] == 0


@pytest.mark.parametrize("tag", ["msci_ls", "msci_ls_l2", "msci_ls_log", "msci_mv", "msci_mv_shrink", "msci_qeqw"])
def test_qp_golden_msci(device, tag):
    g = load_golden(tag)
    P, q, A, b, lb, ub = g["P"], g["q"], g["A"], g["b"], g["lb"], g["ub"]
    qb = engine.QPBatch.from_dense(P, q, A=A[0], b=b[0].reshape(-1), lb=lb[0], ub=ub[0], device=device)
    res = engine.solve(qb)
    x = res.x.cpu().numpy()
    st = res.status.cpu().numpy()
    obj = res.obj.cpu().numpy()
    assert np.all(st == 1), (tag, np.unique(st, return_counts=True))
    xg = g["x"]
    og = g["obj"]
    errs = np.abs(x - xg).max(axis=1)
    assert errs.max() < 1e-5, (tag, errs.max(), int(errs.argmax()))
    objd = np.array([0.5 * x[i] @ P[i] @ x[i] + q[i] @ x[i] for i in range(len(x))])
    assert np.allclose(objd, obj, rtol=1e-9, atol=1e-15)
    rel = np.abs(obj - og) / np.maximum(np.abs(og), 1e-12)
    assert rel.max() < 1e-6, (tag, rel.max())
    viol = np.maximum(np.abs(x.sum(1) - 1), np.maximum(lb - x, x - ub).max(1))
    assert viol.max() <= 1e-7


@pytest.mark.parametrize("shrink", [0.1, 0.0])
def test_qp_synthetic_n1000_min_variance(device, shrink):
    n, T = 1000, 252
    dates, R, _, _ = factor_panel(520, n)
    ends = [300, 519]
    Ps = []
    for e in ends:
        S = cov_pearson(R[e - T + 1:e + 1])
        if shrink:
            S = S + shrink * np.mean(np.diag(S)) * np.eye(n)
        Ps.append(2 * S)
    P = np.stack(Ps)
    q = np.zeros((len(ends), n))
    qb = engine.QPBatch.from_dense(P, q, A=np.ones((1, n)), b=np.ones(1), lb=np.zeros(n), ub=np.ones(n), device=device)
    res = engine.solve(qb)
    x = res.x.cpu().numpy()
    assert np.all(res.status.cpu().numpy() == 1)
    for i in range(len(ends)):
        s = solve_qp(P[i], q[i], A=np.ones((1, n)), b=np.ones(1), lb=np.zeros(n), ub=np.ones(n))
        o = 0.5 * x[i] @ P[i] @ x[i]
        assert abs(o - s.obj) <= 1e-6 * abs(s.obj)
        assert np.abs(x[i] - s.x).max() < 1e-5
        assert max(abs(x[i].sum() - 1), -x[i].min(), x[i].max() - 1) <= 1e-7


@pytest.mark.parametrize("n,T,stride,offset", [(1000, 252, 1, 0.0), (130, 60, 3, 0.0), (70, 40, 1, 50.0)])
def test_grouped_window_moments_match_per_date_kernels(device, n, T, stride, offset):
    """pq_window_moments_grouped (one sliding pass per slide group, shifted sums) against
    pq_window_mean + pq_window_sumsq (and numpy); offset: price-like data with a large common
    mean, where unshifted sliding sums would cancel."""
    D = T + 60 * stride
    dates, R, y, _ = factor_panel(D, n, seed=n + stride)
    R = R + offset
    reb = dates[T - 1::stride][:60]
    rows, tlen = engine.window_rows(dates, reb, T)
    gp = engine.GroupPlan(rows, tlen, device)
    assert gp.ok and gp.ngroups < len(reb)
    pan = engine.Panel(R, device=device)
    r_d, t_d = pan.rows_to_device(rows, tlen)
    mu_a = pan.window_means(r_d, t_d)
    dg_a = pan.window_sumsq(r_d, t_d, mu_a)
    mu_b = torch.full_like(mu_a, float("nan"))
    dg_b = torch.full_like(dg_a, float("nan"))
    pan.window_moments_grouped(gp, t_d, mu_b, dg_b)
    mu_a, dg_a, mu_b, dg_b = (v.cpu().numpy()[:, :n] for v in (mu_a, dg_a, mu_b, dg_b))
    scale = np.abs(R).max()
    assert np.abs(mu_a - mu_b).max() <= 1e-14 * scale
    assert np.all(np.abs(dg_a - dg_b) <= 1e-12 * dg_a)
    for b in (0, len(reb) // 2, len(reb) - 1):
        X = R[rows[b, :tlen[b]]]
        assert np.abs(mu_b[b] - X.mean(0)).max() <= 1e-14 * scale
        assert np.all(np.abs(dg_b[b] - ((X - X.mean(0)) ** 2).sum(0)) <= 1e-12 * dg_a[b])


@pytest.mark.parametrize("m,n,B,trans,offset", [(255, 1000, 37, 0, 0), (255, 1000, 37, 1, 0),
                                                 (7, 33, 5, 0, 1), (7, 33, 5, 1, 1), (300, 2000, 3, 1, 0)])
def test_gemv_batched_matches_torch(device, m, n, B, trans, offset):
    """pq_gemv_batched (ipm_l1's U x / U' x) against torch.bmm in FP64: aligned 16-byte and
    odd / unaligned scalar paths (offset shifts the base pointer by one double)."""
    from porqua_amd.ipm_l1 import _gemv
    g = torch.Generator(device="cpu").manual_seed(m * 7 + n)
    big = torch.randn(B * m * n + 1, generator=g, dtype=torch.float64).to(device)
    U = big[offset:offset + B * m * n].view(B, m, n)
    x = torch.randn((B, m if trans else n), generator=g, dtype=torch.float64).to(device)
    got = _gemv(U, x, bool(trans))
    ref = torch.bmm(U.transpose(1, 2) if trans else U, x.unsqueeze(2)).squeeze(2)
    torch.cuda.synchronize()
    assert torch.allclose(got, ref, rtol=1e-13, atol=1e-12), float((got - ref).abs().max())



@pytest.mark.parametrize("stride", [1, 21])
def test_geomean_grouped_matches_per_window(device, stride):
    """pq_window_geomean_grouped (sliding log sums over slide-group windows) against the
    per-window kernel and numpy's (1 + X).prod() ** (1 / T) - 1 (src/mean_estimation.py:39-48),
    daily and monthly rebalancing."""
    n, T = 300, 120
    D = T + 40 * stride + 10
    dates, R, _, _ = factor_panel(D, n, seed=7)
    reb = dates[T + 3::stride][:40]
    rows, tlen = engine.window_rows(dates, reb, T)
    pan = engine.Panel(R, None, device=device)
    r_d, t_d = pan.rows_to_device(rows, tlen)
    gp = engine.GroupPlan(rows, tlen, device)
    assert gp.ok and gp.ngroups < len(reb)
    mg = pan.window_geomeans_grouped(gp, t_d).cpu().numpy()
    mw = pan.window_means(r_d, t_d, geometric=True).cpu().numpy()
    assert _rel(mg[:, :n], mw[:, :n]) <= 1e-12
    for b in range(len(reb)):
        Xw = R[rows[b, :tlen[b]]]
        assert _rel(mg[b, :n], (1.0 + Xw).prod(0) ** (1.0 / tlen[b]) - 1.0) <= 1e-11

@pytest.mark.parametrize("stride", [1, 21])
def test_gram_xy_grouped_matches_per_window(device, stride):
    """pq_gram_xy_grouped (X'y, y'y and diag(X'X) of slide-group windows by entering / leaving
    rows) against numpy per window: daily (stride 1) and monthly (stride 21) rebalancing."""
    n, T = 300, 120
    D = T + 40 * stride + 10
    dates, R, y, _ = factor_panel(D, n, seed=5)
    reb = dates[T + 3::stride][:40]
    rows, tlen = engine.window_rows(dates, reb, T)
    pan = engine.Panel(R, y, device=device)
    _, t_d = pan.rows_to_device(rows, tlen)
    gp = engine.GroupPlan(rows, tlen, device)
    assert gp.ok and gp.ngroups < len(reb)
    dg = torch.zeros((len(reb), 320), dtype=torch.float64, device=device)
    xty, yty = pan.gram_xy_grouped(gp, t_d, dg=dg)
    xty, yty, dg = xty.cpu().numpy(), yty.cpu().numpy(), dg.cpu().numpy()
    for b in range(len(reb)):
        Xw, yw = R[rows[b, :tlen[b]]], y[rows[b, :tlen[b]]]
        assert _rel(xty[b, :n], Xw.T @ yw) <= 1e-12
        assert abs(yty[b] - yw @ yw) <= 1e-13 * (yw @ yw)
        assert _rel(dg[b, :n], (Xw * Xw).sum(0)) <= 1e-12
