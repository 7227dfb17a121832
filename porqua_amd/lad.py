"""LAD (least absolute deviation) tracking as a batched LP on the device.

The reference's ``LAD.model_qpsolvers`` (src/optimization.py:296-345) hands qpsolvers a QP
with P = 0: variables [w; u; v] (n + 2T), equality rows [budget; X I -I] = [b; y], box on w,
u, v >= 0, objective 1'u + 1'v.  That LP has T + 1 general rows, beyond what the ADMM
engine keeps in LDS, and ADMM converges slowly on LPs anyway, so it is solved here by a
batched Mehrotra predictor-corrector interior-point method for

    min c'x   s.t.  A x = b,  l <= x <= h   (infinite bounds allowed)

Each iteration eliminates u, v, the slacks and the T window rows exactly and forms the
w-space normal matrix H = diag(z/s) + X' diag(1/(theta_u + theta_v)) X (n x n) for every
window at once (one batched GEMM).  K2 (``pq_factor_batched``, the engine's FP64-MFMA
blocked Cholesky, invert = 2) factors and inverts it; the predictor and the corrector
reuse the inverse, refined against the unshifted H, and the few budget / group rows
border it through a small Schur system.  Inequality rows G x <= h get slack columns.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib, engine

F64 = torch.float64
_REFINE = 2
_INACCURATE = 1e-6


# window-form (Woodbury) normal equations when T < n; False forces the dense n x n H
WOODBURY = True


def round_up64(v: int) -> int:
    return (int(v) + 63) // 64 * 64


class LPResult:
    """x: the best iterate by the merit max(rel. primal residual, rel. dual residual, rel.
    gap); status PQ_SOLVED (merit < tol), PQ_SOLVED_INACCURATE (< 1e-6) or PQ_MAX_ITER."""

    def __init__(self, x, lam, status, iters, obj, merit):
        self.x, self.lam, self.status, self.iters, self.obj, self.merit = x, lam, status, iters, obj, merit

    @property
    def found(self):
        return (self.status == _lib.PQ_SOLVED) | (self.status == _lib.PQ_SOLVED_INACCURATE)


class LADProblem:
    """The reference's LP (src/optimization.py:301-336) for a batch of windows, kept in
    structured form: variables x = [w (n); u (T); v (T); s (mi)], rows
    [C w + [0; s] = d  (C = [A; G], the budget / equality rows first);  X w + u - v = y].
    The reference's dense A_tilde = [[A, 0, 0], [X, I, -I]] and G_tilde = [G, 0, 0] are the
    same rows (G written with slacks).  X (B, T, n) and y (B, T) are device tensors."""

    def __init__(self, X, y, A=None, b=None, G=None, h=None, lb=None, ub=None):
        B, T, n = X.shape
        dev = X.device
        self.X, self.y, self.B, self.T, self.n, self.dev = X, y, B, T, n, dev
        rows, rhs = [], []
        self.me = 0 if A is None else np.atleast_2d(A).shape[0]
        self.mi = 0 if G is None else np.atleast_2d(G).shape[0]
        if self.me:
            rows.append(np.atleast_2d(np.asarray(A, dtype=np.float64)))
            rhs.append(np.asarray(b, dtype=np.float64).reshape(-1))
        if self.mi:
            rows.append(np.atleast_2d(np.asarray(G, dtype=np.float64)))
            rhs.append(np.asarray(h, dtype=np.float64).reshape(-1))
        self.mc = self.me + self.mi
        self.C = torch.as_tensor(np.vstack(rows) if rows else np.zeros((0, n)), dtype=F64, device=dev)
        d = torch.as_tensor(np.concatenate(rhs) if rhs else np.zeros(0), dtype=F64, device=dev)
        self.b = torch.cat([d.expand(B, self.mc), y], 1)          # (B, mc + T)
        N = n + 2 * T + self.mi
        self.N, self.m = N, self.mc + T
        self.c = torch.zeros(N, dtype=F64, device=dev)
        self.c[n:n + 2 * T] = 1.0
        self.lo = torch.zeros(N, dtype=F64, device=dev)
        self.hi = torch.full((N,), np.inf, dtype=F64, device=dev)
        self.lo[:n] = -np.inf if lb is None else torch.as_tensor(np.asarray(lb, dtype=np.float64), device=dev)
        self.hi[:n] = np.inf if ub is None else torch.as_tensor(np.asarray(ub, dtype=np.float64), device=dev)

    def split(self, x):
        n, T = self.n, self.T
        return x[:, :n], x[:, n:n + T], x[:, n + T:n + 2 * T], x[:, n + 2 * T:]

    def A(self, x):
        w, u, v, s = self.split(x)
        rc = w @ self.C.T
        if self.mi:
            rc = rc + torch.cat([torch.zeros_like(rc[:, :self.me]), s], 1)
        rt = _gemv(self.X, w) + u - v
        return torch.cat([rc, rt], 1)

    def At(self, lam):
        lc, lt = lam[:, :self.mc], lam[:, self.mc:]
        gw = lc @ self.C + _gemv(self.X, lt, True)
        return torch.cat([gw, lt, -lt, lc[:, self.me:]], 1)


def _gemv(U, x, trans: bool = False):
    """U[b] x[b] (trans: U[b]' x[b]) for U (B, m, n) with unit column stride and x (B, n) or
    (B, m): the HBM-bound HIP kernel pq_gemv_batched, one read of U per product (a batched
    GEMM with a single right-hand side ran at ~1 TB/s and dominated the IPM iterations)."""
    B, m, n = U.shape
    if U.stride(2) != 1:
        U = U.contiguous()
    x = x.contiguous()
    assert x.shape == (B, m if trans else n), (tuple(x.shape), tuple(U.shape), trans)
    y = torch.empty((B, n if trans else m), dtype=torch.float64, device=U.device)
    lib = _lib.load()
    stream = engine._stream()
    for s in range(0, B, 65535):   # grid.y limit
        c = min(B, s + 65535) - s
        _lib.check(lib.pq_gemv_batched(U[s:].data_ptr(), U.stride(1), U.stride(0), m, n, c, int(trans),
                                       x[s:].data_ptr(), x.stride(0), y[s:].data_ptr(), y.stride(0), stream),
                   "pq_gemv_batched")
    return y


def _mv(M, V, S=None):
    """M V, or S - M V, for M (B, n, n) with unit column stride and V (B, n, k): the HIP
    kernel pq_lad_mv_batched for k <= 4 (one pass over M), a batched GEMM otherwise."""
    B, n, k = V.shape
    if k > 4:   # several passes over M, four right-hand sides each
        parts = [_mv(M, V[:, :, c:c + 4], None if S is None else S[:, :, c:c + 4]) for c in range(0, k, 4)]
        return torch.cat(parts, 2)
    assert M.stride(2) == 1 and M.shape[1] == n and M.shape[2] == n
    V = V.contiguous()
    S = None if S is None else S.contiguous()
    out = torch.empty_like(V)
    lib = _lib.load()
    _lib.check(lib.pq_lad_mv_batched(M.data_ptr(), M.stride(1), M.stride(0), n, B, V.data_ptr(), V.stride(0), k,
                                     None if S is None else S.data_ptr(), 0 if S is None else S.stride(0),
                                     out.data_ptr(), out.stride(0), engine._stream()), "pq_lad_mv_batched")
    return out


class _NormalFactor:
    """H = diag(1/theta_w) + X' diag(1/(theta_u + theta_v)) X per window (n x n), factored
    and inverted on K2 (pq_factor_batched, invert = 2: Cholesky, trtri, lauum)."""

    LARGE = 1024   # beyond: K2L (pq_factor_large, many workgroups per matrix)

    def __init__(self, B, m, dev):
        self.m = m
        self.qb = engine.QPBatch(m, B, 0, device=dev, has_box=False)
        self.ws = engine.Workspace(self.qb)
        self.scratch = (torch.empty((B, self.qb.ld, self.qb.ld), dtype=F64, device=dev)
                        if m > self.LARGE else None)
        self.s = engine.Settings(sigma=0.0).to_c()
        self.pb = self.qb.c_struct()
        self.st = self.ws.c_struct()
        lib = _lib.load()
        _lib.check(lib.pq_init_state(ctypes.byref(self.pb), ctypes.byref(self.st), None, 0,
                                     ctypes.byref(self.s), engine._stream()), "pq_init_state (LP)")

    def factor(self, H, shift, retries: int = 3):
        """Factor H + diag(shift) and overwrite the K2 scratch with its inverse (invert = 2).
        A problem whose Cholesky breaks down (K2 ``info`` != 0: its inverse is NOT formed)
        is refactored with a 1e4x larger shift, up to ``retries`` times.  Returns a bool
        tensor of the problems that still failed -- the caller must freeze those (their
        Hinv is garbage but finite)."""
        m, lib = self.m, _lib.load()
        P = self.qb.P
        shift = shift.clone() if torch.is_tensor(shift) else torch.full(H.shape[:2], float(shift), dtype=F64,
                                                                           device=H.device)
        for attempt in range(retries + 1):
            P[:, :m, :m].copy_(H)
            P.diagonal(dim1=1, dim2=2)[:, :m].add_(shift)
            if self.scratch is not None:
                _lib.check(lib.pq_factor_large(ctypes.byref(self.pb), ctypes.byref(self.st), None, 0,
                                               ctypes.byref(self.s), 2, self.scratch.data_ptr(),
                                               self.scratch.stride(0), engine._stream()), "pq_factor_large")
            else:
                _lib.check(lib.pq_factor_batched(ctypes.byref(self.pb), ctypes.byref(self.st), None, 0,
                                                 ctypes.byref(self.s), 2, engine._stream()), "pq_factor_batched (LP)")
            bad = self.ws.info != 0
            if attempt == retries or not bool(bad.any()):     # host sync: one small flag
                break
            scale = H.diagonal(dim1=1, dim2=2).abs().amax(1, keepdim=True).clamp(min=1e-300)
            shift = torch.where(bad[:, None], shift * 1e4 + 1e-12 * scale, shift)
        self.Hinv = self.ws.K[:, :m, :m]
        return bad

    def solve_mat(self, R):
        """(H + diag(shift))^-1 R for R (B x n x k)."""
        return _mv(self.Hinv, R)


def lad_ipm_batched(pr: LADProblem, tol: float = 1e-9, max_iter: int = 80, trace=None) -> LPResult:
    """Mehrotra predictor-corrector IPM for min c'x, A x = b, lo <= x <= hi on the LAD
    structure, batched over windows; converged problems are frozen.

    Newton directions: with T < n (every backtest window here) from the LP's m-space normal
    equations (A Theta A') dlam = r, (mc + T) x (mc + T), formed by the weighted-SYRK kernel
    pq_wgram_batched and factored on K2 (porqua_amd/woodbury.py); otherwise from the w-space
    normal equations (the Koenker / Portnoy form of LAD interior-point methods): u, v, s and
    the T window rows are eliminated exactly, which leaves H dw - C' dlam_C = f (n x n, K2
    Cholesky) bordered by the few rows of C."""
    B, m, N, n, T = pr.B, pr.m, pr.N, pr.n, pr.T
    dev = pr.dev
    c, lo, hi, b = pr.c, pr.lo, pr.hi, pr.b
    FL = torch.isfinite(lo).to(F64).expand(B, N)
    FH = torch.isfinite(hi).to(F64).expand(B, N)
    lo_ = torch.where(torch.isfinite(lo), lo, torch.zeros_like(lo))
    hi_ = torch.where(torch.isfinite(hi), hi, torch.zeros_like(hi))
    span = (hi_ - lo_).clamp(min=0)
    x0 = torch.full((N,), 1.0, dtype=F64, device=dev)
    both = torch.isfinite(lo) & torch.isfinite(hi)
    x0 = torch.where(both, lo_ + 0.5 * span, x0)
    x0 = torch.where(torch.isfinite(lo) & ~torch.isfinite(hi), lo_ + 1.0, x0)
    x0 = torch.where(~torch.isfinite(lo) & torch.isfinite(hi), hi_ - 1.0, x0)
    x = x0.expand(B, N).clone()
    lam = torch.zeros((B, m), dtype=F64, device=dev)
    zl = FL.clone()
    zh = FH.clone()
    mc, me, X, C = pr.mc, pr.me, pr.X, pr.C
    # window shorter than the universe (the backtest configurations, T = 252 < n): the LP's
    # m-space normal equations M = [C; X] diag(theta_w) [C; X]' + diag(0, theta_s, theta_u +
    # theta_v), (mc + T) x (mc + T), on the weighted-SYRK kernel; the w-space n x n H otherwise
    nm = None
    nfac = None
    if WOODBURY and T < n and round_up64(mc + T) <= 1024:
        from .woodbury import NormalM
        nm = NormalM(torch.cat([C.expand(B, mc, n), X], 1).contiguous() if mc else X.contiguous())
    else:
        nfac = _NormalFactor(B, n, dev)
    ncomp = (FL + FH).sum(1).clamp(min=1)
    bn = 1.0 + b.abs().amax(1)
    cn = 1.0 + c.abs().amax()
    done = torch.zeros(B, dtype=torch.bool, device=dev)
    iters = torch.zeros(B, dtype=torch.int32, device=dev)
    best_x = x.clone()
    best_merit = torch.full((B,), np.inf, dtype=F64, device=dev)
    best_it = torch.zeros(B, dtype=torch.int64, device=dev)

    for it in range(max_iter):
        sl = torch.where(FL > 0, (x - lo_).clamp(min=1e-200), torch.ones_like(x))
        sh = torch.where(FH > 0, (hi_ - x).clamp(min=1e-200), torch.ones_like(x))
        rp = b - pr.A(x)
        rd = c - pr.At(lam) - zl + zh
        pobj = (c * x).sum(1)
        dobj = (b * lam).sum(1) + (lo_ * zl * FL).sum(1) - (hi_ * zh * FH).sum(1)
        mu = ((sl * zl * FL).sum(1) + (sh * zh * FH).sum(1)) / ncomp
        merit = torch.maximum(torch.maximum(rp.abs().amax(1) / bn, rd.abs().amax(1) / cn),
                              (pobj - dobj).abs() / (1.0 + pobj.abs()))
        merit = torch.where(torch.isnan(merit), torch.full_like(merit, np.inf), merit)
        better = (merit < best_merit) & ~done
        best_x = torch.where(better[:, None], x, best_x)
        best_it = torch.where(better, torch.full_like(best_it, it), best_it)
        best_merit = torch.where(better, merit, best_merit)
        # converged, or stalled (the normal matrix has run out of accuracy): keep the best iterate
        done = done | (merit < tol) | ((it - best_it > 6) & (best_merit < _INACCURATE))
        done = done | ~torch.isfinite(x).all(1)             # broke down: keep the best iterate
        if trace is not None:
            trace.append((it, float(mu.max()), float((rp.abs().amax(1) / bn).max()),
                          float((rd.abs().amax(1) / cn).max()), float(((pobj - dobj).abs() / (1.0 + pobj.abs())).max())))
        if bool(done.all()):
            break
        iters += (~done).to(torch.int32)
        Dg = (FL * zl / sl + FH * zh / sh).clamp(1e-12, 1e24)
        Dg = torch.where(done[:, None], torch.ones_like(Dg), Dg)     # frozen: any PD system
        th = 1.0 / Dg
        th_w, th_u, th_v, th_s = pr.split(th)
        e_inv = torch.where(done[:, None], torch.ones_like(th_u), 1.0 / (th_u + th_v))
        if nm is not None:
            dM = torch.cat([torch.zeros((B, me), dtype=F64, device=dev), th_s, th_u + th_v], 1)
            failed = nm.factor(th_w, dM)
        else:
            H = torch.bmm(X.transpose(1, 2), X * e_inv.unsqueeze(2))
            H.diagonal(dim1=1, dim2=2).add_(Dg[:, :n])
            # factor a slightly shifted H (rank-deficient X'E^-1 X at degenerate vertices); the
            # refinement step in hsolve is taken against the unshifted H
            failed = nfac.factor(H, 1e-12 * H.diagonal(dim1=1, dim2=2))
        if bool(failed.any()):               # K2 broke down even shifted: freeze at the best iterate
            done = done | failed
            if bool(done.all()):
                break

        def hsolve(R, refine=_REFINE):       # H^-1 R (R: B x n x k), refined against H
            Y = nfac.solve_mat(R)
            for _ in range(refine):
                Y = Y + nfac.solve_mat(_mv(H, Y, R))
            return Y

        if mc and nm is None:
            HiC = hsolve(C.T.expand(B, n, mc).contiguous())          # H^-1 C'
            S = C @ HiC                                              # C H^-1 C' (B, mc, mc)
            theta_S = torch.cat([torch.zeros((B, me), dtype=F64, device=dev), th_s], 1)
            S = S + torch.diag_embed(theta_S)
            S = S + torch.diag_embed(1e-14 * S.diagonal(dim1=1, dim2=2).abs())

        def bordered(f, g):                  # [H -C'; C Theta_S] [dw; dlc] = [f; g]
            Hf = hsolve(f.unsqueeze(2)).squeeze(2)
            dlc = torch.linalg.solve(S, g - Hf @ C.T)
            return Hf + torch.bmm(HiC, dlc.unsqueeze(2)).squeeze(2), dlc

        def direction(rl, rh):
            if nm is not None:
                return direction_m(rl, rh)
            rx = rd - rl / sl + rh / sh              # D dx - A' dlam = -rx,  A dx = rp
            rx_w, rx_u, rx_v, rx_s = pr.split(rx)
            r_c, r_t = rp[:, :mc], rp[:, mc:]
            g_t = r_t + th_u * rx_u - th_v * rx_v
            f = -rx_w + _gemv(X, g_t * e_inv, True)
            if mc:
                g_c = r_c.clone()
                if pr.mi:
                    g_c[:, me:] += th_s * rx_s
                dw, dlc = bordered(f, g_c)
                for _ in range(2):     # refine against [H -C'; C Theta_S]
                    e1 = f - (_mv(H, dw.unsqueeze(2)).squeeze(2) - dlc @ C)
                    e2 = g_c - (dw @ C.T + theta_S * dlc)
                    cw, cl = bordered(e1, e2)
                    dw, dlc = dw + cw, dlc + cl
            else:
                dlc = torch.zeros((B, 0), dtype=F64, device=dev)
                dw = hsolve(f.unsqueeze(2)).squeeze(2)
            dlt = (g_t - _gemv(X, dw)) * e_inv
            du = th_u * (dlt - rx_u)
            dv = th_v * (-dlt - rx_v)
            ds = th_s * (dlc[:, me:] - rx_s)
            dx = torch.cat([dw, du, dv, ds], 1)
            dl = torch.cat([dlc, dlt], 1)
            dzl = FL * (rl - zl * dx) / sl
            dzh = FH * (rh + zh * dx) / sh
            return dx, dl, dzl, dzh

        def direction_m(rl, rh):
            # D dx - A' dlam = -rx, A dx = rp  =>  (A Theta A') dlam = rp + A Theta rx,
            # dx = Theta (A' dlam - rx)
            rx = rd - rl / sl + rh / sh
            dl = nm.solve(rp + pr.A(th * rx), refine=_REFINE)
            dx = th * (pr.At(dl) - rx)
            dzl = FL * (rl - zl * dx) / sl
            dzh = FH * (rh + zh * dx) / sh
            return dx, dl, dzl, dzh

        def steps(dx, dzl, dzh):
            inf = torch.full_like(dx, np.inf)
            ap = torch.minimum(torch.where((FL > 0) & (dx < 0), -sl / dx, inf),
                               torch.where((FH > 0) & (dx > 0), sh / dx, inf)).amin(1)
            ad = torch.minimum(torch.where(dzl < 0, -zl / dzl, inf), torch.where(dzh < 0, -zh / dzh, inf)).amin(1)
            return ap.clamp(max=1.0), ad.clamp(max=1.0)

        dx, dl, dzl, dzh = direction(-sl * zl * FL, -sh * zh * FH)
        ap, ad = steps(dx, dzl, dzh)
        mu_aff = (((sl + ap[:, None] * dx) * (zl + ad[:, None] * dzl) * FL).sum(1)
                  + ((sh - ap[:, None] * dx) * (zh + ad[:, None] * dzh) * FH).sum(1)) / ncomp
        sig = (mu_aff / mu).clamp(0, 1) ** 3
        smu = (sig * mu)[:, None]
        rl = FL * (smu - sl * zl - dx * dzl)
        rh = FH * (smu - sh * zh + dx * dzh)
        dx, dl, dzl, dzh = direction(rl, rh)
        ap, ad = steps(dx, dzl, dzh)
        act = ~done[:, None]
        ap = (0.995 * ap)[:, None]
        ad = (0.995 * ad)[:, None]
        x = torch.where(act, x + ap * dx, x)
        lam = torch.where(act, lam + ad * dl, lam)
        zl = torch.where(act, zl + ad * dzl, zl)
        zh = torch.where(act, zh + ad * dzh, zh)
    status = torch.full_like(iters, _lib.PQ_MAX_ITER)
    status = torch.where(best_merit < _INACCURATE, torch.full_like(iters, _lib.PQ_SOLVED_INACCURATE), status)
    status = torch.where(best_merit < tol, torch.full_like(iters, _lib.PQ_SOLVED), status)
    return LPResult(best_x, lam, status, iters, (c * best_x).sum(1), best_merit)
