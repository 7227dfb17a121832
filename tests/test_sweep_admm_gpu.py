"""The risk-aversion sweep's ADMM kernel (admm_sweep.hip, engine.SweepPlan) against the
grouped kernel it replaces (k_admm_grp's fused form):

  * iterates: after a fixed number of iterations (max_iter) x, z, y and the general rows agree
    to rounding -- same updates, same rhs, only the summation order of the window passes
    differs;
  * stops: with the sweep's loose ADMM stop the iteration counts and statuses agree, and the
    polished answers are the same optimum;
  * ragged shapes: n not a multiple of the 256-asset chunk, dates with 40 and 70 risk
    aversions (groups of 40, and 64 + 6), and a group partly solved before the call.
The optima themselves are pinned against the oracle at the config-5 shape by
tests/test_large_n_gpu.py and tests/test_full_configs_gpu.py (src/optimization.py:168-174)."""
import numpy as np
import pytest
import torch

from porqua_amd import _lib, engine
from porqua_amd.sweep import SWEEP_SETTINGS, MeanVarianceSweep
from porqua_amd.synthetic import factor_panel

pytestmark = pytest.mark.gpu


def _sweep(n, dates, lambdas, settings, device, use_kernel, per_date=False):
    T, stride = 252, 21
    d_all, R, _, _ = factor_panel(T - 1 + stride * dates, n)
    ends = np.arange(T - 1, T - 1 + stride * dates, stride)
    rows, tlen = engine.window_rows(d_all, d_all[ends], T)
    pan = engine.Panel(R, device=device)
    sw = MeanVarianceSweep(pan, rows, tlen, lambdas, settings=settings, factor="chol")
    if not use_kernel:
        sw.sp = None
    if per_date:   # no groups at all: pq_admm_lr_batched, one workgroup per problem
        sw.sp = sw.gp = None
    res, meta = sw.solve()
    torch.cuda.synchronize()
    return sw, res


def _state(sw, res):
    ws = sw.ws
    return (res.x.cpu().numpy().copy(), ws.z.cpu().numpy().copy(), ws.y.cpu().numpy().copy(),
            res.iters.cpu().numpy().copy(), res.status.cpu().numpy().copy())


@pytest.mark.parametrize("n,L", [(700, 40), (520, 70)])
def test_sweep_kernel_iterates_match_grouped_kernel(device, n, L):
    """Fixed iteration budget, no polish: the sweep kernel's iterates agree with the grouped
    kernel's as closely as the grouped kernel's agree with the per-problem kernel's
    (pq_admm_lr_batched) -- three summation orders of the same iteration, whose rounding the
    capacitance solve amplifies (cond(M_b) grows with the risk aversion)."""
    lambdas = np.logspace(-1, 2, L)
    st = engine.Settings.from_params({**SWEEP_SETTINGS, "polish": 0, "max_iter": 9, "eps_grouped": 0.0,
                                    "eps_abs": 1e-12, "eps_rel": 1e-12})
    sw_a, ra = _sweep(n, 3, lambdas, st, device, True)
    sw_b, rb = _sweep(n, 3, lambdas, st, device, False)
    sw_c, rc = _sweep(n, 3, lambdas, st, device, False, per_date=True)
    assert sw_a.sp is not None and sw_a.sp.ngroups == 3 * ((L + 63) // 64)
    xa, za, ya, ia, sa = _state(sw_a, ra)
    xb, zb, yb, ib, sb = _state(sw_b, rb)
    xc, zc, yc, _, _ = _state(sw_c, rc)
    assert np.array_equal(ia, ib) and np.array_equal(sa, sb), (np.unique(ia), np.unique(ib))
    assert np.all(sa == _lib.PQ_MAX_ITER)
    for a, b, c in ((xa, xb, xc), (za, zb, zc), (ya, yb, yc)):
        sc = np.maximum(np.abs(b).max(1), 1e-300)
        d_new = np.abs(a - b).max(1) / sc                  # per problem, relative
        d_ref = np.abs(b - c).max(1) / sc
        assert d_new.max() <= 10.0 * d_ref.max() + 1e-14, (d_new.max(), d_ref.max())
        assert np.median(d_new) <= 10.0 * np.median(d_ref) + 1e-14, (np.median(d_new), np.median(d_ref))
        assert d_new.max() <= 1e-6, d_new.max()


def test_sweep_kernel_solves_like_grouped_kernel(device):
    """The sweep's own settings (loose stop, grouped polish): same iteration counts up to a
    stop decided within rounding, same certified optima."""
    lambdas = np.logspace(-1, 2, 64)
    st = engine.Settings.from_params(SWEEP_SETTINGS)
    sw_a, ra = _sweep(900, 4, lambdas, st, device, True)
    sw_b, rb = _sweep(900, 4, lambdas, st, device, False)
    xa, _, _, ia, sa = _state(sw_a, ra)
    xb, _, _, ib, sb = _state(sw_b, rb)
    assert np.all(sa == _lib.PQ_SOLVED) and np.all(sb == _lib.PQ_SOLVED)
    assert np.mean(ia == ib) >= 0.95, (ia, ib)
    assert np.abs(xa - xb).max() <= 1e-7, np.abs(xa - xb).max()


def test_sweep_kernel_skips_solved_problems(device):
    """Problems already solved when the kernel starts keep their state (the polish hand-back
    resumes ADMM for a subset)."""
    lambdas = np.logspace(-1, 2, 48)
    st = engine.Settings.from_params({**SWEEP_SETTINGS, "polish": 0, "max_iter": 6, "eps_grouped": 0.0,
                                    "eps_abs": 1e-12, "eps_rel": 1e-12})
    T, stride, n = 252, 21, 600
    d_all, R, _, _ = factor_panel(T - 1 + stride * 2, n)
    ends = np.arange(T - 1, T - 1 + stride * 2, stride)
    rows, tlen = engine.window_rows(d_all, d_all[ends], T)
    pan = engine.Panel(R, device=device)
    sw = MeanVarianceSweep(pan, rows, tlen, lambdas, settings=st, factor="chol")
    res, _ = sw.solve()
    torch.cuda.synchronize()
    ws = sw.ws
    x0 = res.x.clone()
    it0 = res.iters.clone()
    # mark every other problem solved, resume the rest through the kernel for 6 more iterations
    done = torch.zeros_like(ws.status, dtype=torch.bool)
    done[::2] = True
    ws.status[done] = _lib.PQ_SOLVED
    ws.status[~done] = _lib.PQ_UNSOLVED
    lib = _lib.load()
    qb, lr = sw.qb, sw.lr
    s = st.to_c()
    s.max_iter = 12
    M = ws.lr_buffers(256)
    bd = engine._band_setup(qb, lr, engine._stream(), w_min=0)
    scr = sw.sp.buffer(qb, lib)
    pb, stc, lrs = qb.c_struct(), ws.c_struct(), lr.c_struct()
    import ctypes
    _lib.check(lib.pq_admm_lr_sweep(ctypes.byref(lrs), ctypes.byref(pb), ctypes.byref(stc), M["Minv"].data_ptr(), 256,
                                    256 * 256, sw.sp.gdates.data_ptr(), sw.sp.ngroups, ctypes.byref(s), 6,
                                    bd["pc"].data_ptr(), bd["pc"].stride(0), bd["r0"], bd["cc"].data_ptr(), 1,
                                    scr.data_ptr(), scr.numel(), engine._stream()), "pq_admm_lr_sweep")
    torch.cuda.synchronize()
    assert torch.equal(res.x[done], x0[done])
    assert torch.equal(ws.iters[done], it0[done])
    assert bool((ws.iters[~done] == it0[~done] + 6).all())
    assert bool((res.x[~done] - x0[~done]).abs().amax() > 0)


def test_sweep_kernel_adaptive_rho_matches_grouped_kernel(device):
    """Adaptive rho inside the sweep kernel: the rho requests (NEED_REFACTOR), the engine's
    refactorisation and the resumed iterations agree with the grouped kernel's."""
    lambdas = np.logspace(-1, 2, 24)
    st = engine.Settings.from_params({**SWEEP_SETTINGS, "polish": 0, "max_iter": 14, "eps_grouped": 0.0,
                                      "eps_abs": 1e-12, "eps_rel": 1e-12, "adapt_interval": 4,
                                      "adapt_tol": 1.5})
    sw_a, ra = _sweep(600, 2, lambdas, st, device, True)
    sw_b, rb = _sweep(600, 2, lambdas, st, device, False)
    assert ra.refactors > 0 and ra.refactors == rb.refactors, (ra.refactors, rb.refactors)
    xa, _, _, ia, sa = _state(sw_a, ra)
    xb, _, _, ib, sb = _state(sw_b, rb)
    assert np.array_equal(ia, ib) and np.array_equal(sa, sb)
    # the requested rho is a ratio of residual maxima, which carry the iterates' rounding
    # differences (up to ~1e-7 relative after a few iterations, the first test above)
    rho_a, rho_b = sw_a.ws.rho.cpu().numpy(), sw_b.ws.rho.cpu().numpy()
    assert np.abs(rho_a / rho_b - 1.0).max() <= 1e-5, np.abs(rho_a / rho_b - 1.0).max()
    sc = np.maximum(np.abs(xb).max(1), 1e-300)
    assert (np.abs(xa - xb).max(1) / sc).max() <= 1e-6
