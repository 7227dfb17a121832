"""Eigen-form capacitance (engine.EigCap / pq_eigcap_form) for the risk-aversion x date sweep
(BASELINE.json configs[4]; P = 2 lam Sigma_d, src/optimization.py:168-174):

  * kernel: M_b^-1 formed from one eigendecomposition per date equals the inverse of the
    capacitance pq_lr_capacitance builds for the same problem (per-problem rho, scale and
    budget row), also when only a subset of problems is re-formed after a rho change;
  * solve: the sweep with factor='eig' (one eigendecomposition per date) reproduces the
    per-problem Cholesky form (factor='chol') and the oracle optimum, at a small n and with
    the nearly linear risk aversions (lam 0.1 ..) that need their own |q|-aware rho."""
import ctypes

import numpy as np
import pytest
import torch

from oracle.qp_ipm import solve_qp
from oracle.ref_pipeline import cov_pearson
from porqua_amd import _lib, engine
from porqua_amd.sweep import mean_variance_sweep
from porqua_amd.synthetic import factor_panel
from tests.kkt import kkt_residuals

pytestmark = pytest.mark.gpu


def _sweep_batch(pan, rows, tlen, lambdas, dev):
    nd, L, n = len(tlen), len(lambdas), pan.n
    r_d, t_d = pan.rows_to_device(rows, tlen)
    mu = pan.window_means(r_d, t_d)
    rp, tp = pan.rows_to_device(np.repeat(rows, L, axis=0), np.repeat(tlen, L))
    B = nd * L
    qb = engine.QPBatch(n, B, 1, device=dev, P=torch.empty(0, dtype=torch.float64, device=dev))
    qb.P = None
    qb.Cg[0, 0, :n] = 1.0
    qb.lg[0, 0] = qb.ug[0, 0] = 1.0
    qb.lb[0, :n], qb.ub[0, :n] = 0.0, 1.0
    qb.lb[0, n:] = qb.ub[0, n:] = 0.0
    lam_p = torch.from_numpy(np.tile(lambdas, nd)).to(dev)
    qb.p_scale = 2.0 * lam_p
    lr = engine.LowRank(pan, rp, tp, mu=mu.repeat_interleave(L, dim=0).contiguous(),
                        w_scale=1.0 / (tp.to(torch.float64) - 1.0))
    return qb, lr, r_d, t_d, mu


@pytest.mark.parametrize("backend", ["jacobi", "rocsolver"])
def test_eigcap_form_matches_capacitance_inverse(device, backend):
    n, T, nd = 400, 120, 3
    lambdas = np.array([0.1, 1.0, 7.5, 100.0])
    L = len(lambdas)
    dates, R, _, _ = factor_panel(T + 40, n)
    ends = [T - 1, T + 10, T + 39]
    rows, tlen = engine.window_rows(dates, dates[ends], T)
    pan = engine.Panel(R, device=device)
    qb, lr, r_d, t_d, mu = _sweep_batch(pan, rows, tlen, lambdas, device)
    B = nd * L
    k = T + 1
    k_ld = engine.round_up(k, 64)
    ws = engine.Workspace(qb, dense=False)
    g = torch.Generator().manual_seed(7)
    ws.rho.copy_((10.0 ** (torch.rand(B, generator=g, dtype=torch.float64) * 6 - 4)).to(device))
    s = engine.Settings().to_c()
    pb, st, lrs = qb.c_struct(), ws.c_struct(), lr.c_struct()
    lib = _lib.load()
    M = torch.zeros((B, k_ld, k_ld), dtype=torch.float64, device=device)
    _lib.check(lib.pq_lr_capacitance(ctypes.byref(lrs), ctypes.byref(pb), ctypes.byref(st), None, 0,
                                     ctypes.byref(s), M.data_ptr(), k_ld, k_ld * k_ld, engine._stream()), "cap")
    Mf = torch.tril(M) + torch.tril(M, -1).mT
    ref = torch.linalg.inv(Mf)
    pdate = torch.arange(nd, dtype=torch.int32, device=device).repeat_interleave(L)
    eig = engine.EigCap(pan, r_d, t_d, mu, qb, pdate, k_ld, backend=backend)
    Minv = torch.full((B, k_ld, k_ld), np.nan, dtype=torch.float64, device=device)
    eig.form(ctypes.byref(lrs), ctypes.byref(pb), ctypes.byref(st), ctypes.byref(s), Minv, None, 0, engine._stream())
    torch.cuda.synchronize()
    assert bool(torch.isfinite(Minv).all())
    err = ((Minv - ref).abs().amax(dim=(1, 2)) / ref.abs().amax(dim=(1, 2))).cpu().numpy()
    assert err.max() <= 1e-11, err
    # a rho change on a subset re-forms only those problems
    idx = torch.tensor([1, 6, 11], dtype=torch.int32, device=device)
    ws.rho[idx.long()] *= 37.0
    _lib.check(lib.pq_lr_capacitance(ctypes.byref(lrs), ctypes.byref(pb), ctypes.byref(st), None, 0,
                                     ctypes.byref(s), M.data_ptr(), k_ld, k_ld * k_ld, engine._stream()), "cap")
    ref2 = torch.linalg.inv(torch.tril(M) + torch.tril(M, -1).mT)
    before = Minv.clone()
    eig.form(ctypes.byref(lrs), ctypes.byref(pb), ctypes.byref(st), ctypes.byref(s), Minv, idx, 3, engine._stream())
    torch.cuda.synchronize()
    changed = torch.zeros(B, dtype=torch.bool, device=device)
    changed[idx.long()] = True
    err2 = ((Minv - ref2).abs().amax(dim=(1, 2)) / ref2.abs().amax(dim=(1, 2)))
    assert float(err2[changed].max()) <= 1e-11
    assert bool((Minv[~changed] == before[~changed]).all())


def test_sweep_eig_matches_chol_and_oracle(device):
    n, T = 1000, 252
    lambdas = np.logspace(-1, 2, 8)
    ends = [260, 281, 302]
    dates, R, _, _ = factor_panel(max(ends) + 1, n)
    rows, tlen = engine.window_rows(dates, dates[ends], T)
    pan = engine.Panel(R, device=device)
    res_e, meta_e = mean_variance_sweep(pan, rows, tlen, lambdas, factor="eig")
    res_c, meta_c = mean_variance_sweep(pan, rows, tlen, lambdas, factor="chol")
    assert meta_e["factor"] == "eig" and meta_e["factorizations"] == len(ends)
    assert res_e.capacitance == "eig"
    st = res_e.status.cpu().numpy()
    assert np.all(st == _lib.PQ_SOLVED), st
    xe, xc = res_e.x.cpu().numpy(), res_c.x.cpu().numpy()
    assert np.abs(xe - xc).max() <= 1e-6
    ye, zb = res_e.y.cpu().numpy(), res_e.z_box.cpu().numpy()
    L = len(lambdas)
    for d, e in enumerate(ends):
        W = R[e - T + 1:e + 1]
        S = cov_pearson(W)
        mu = np.exp(np.mean(np.log1p(W), axis=0)) - 1.0
        for j in (0, 3, 7):
            p = d * L + j
            P = 2 * lambdas[j] * S
            k = kkt_residuals(P, -mu, xe[p], A=np.ones((1, n)), b=np.ones(1), lb=np.zeros(n), ub=np.ones(n),
                              y=ye[p], z_box=zb[p])
            assert max(k.values()) <= 1e-7, (lambdas[j], k)
            o = solve_qp(P, -mu, A=np.ones((1, n)), b=np.ones(1), lb=np.zeros(n), ub=np.ones(n))
            obj = 0.5 * xe[p] @ P @ xe[p] - mu @ xe[p]
            assert abs(obj - o.obj) <= 1e-6 * abs(o.obj), (e, lambdas[j], obj, o.obj)
            assert np.abs(xe[p] - o.x).max() <= 1e-5, (e, lambdas[j])
