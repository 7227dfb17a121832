"""Dense QPs with many general rows, or more than 1024 assets, on the device: a batched
primal-dual IPM.

The ADMM engine (K2-K4) keeps at most 64 general rows in LDS.  The reference's linearised
l1 forms can exceed that: with both a turnover term and a leverage constraint,
``linearize_turnover_*`` adds 2n (+1) rows and ``linearize_leverage_constraint`` n
equality rows (src/qp_problems.py:40-118), which the single-term signed split
(porqua_amd/l1split.py) does not cover.  Those problems are solved here:

    min 0.5 x'Px + q'x   s.t.  A x = b,  G x <= h,  lb <= x <= ub

Mehrotra predictor-corrector on the same machinery as the LAD LP (porqua_amd/lad.py):
slacks of G are eliminated exactly, leaving H = P + diag(z/s) + G' diag(z_G/s_G) G (N x N,
one batched GEMM), factored and inverted on K2 (``pq_factor_batched``, invert = 2), applied
by ``pq_lad_mv_batched`` with refinement, and bordered by the equality rows through a
small Schur system.  Beyond 1024 variables (the per-QP drop-in at thousands of assets,
src/qp_problems.py:184-216) the normal matrix is factored and inverted on K2L
(``pq_factor_large``: many workgroups per matrix) instead of K2.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib
from .lad import LPResult, _mv, _NormalFactor, _INACCURATE

F64 = torch.float64


def qp_ipm_batched(P, q, A=None, b=None, G=None, h=None, lb=None, ub=None, tol: float = 1e-9,
                   max_iter: int = 80) -> LPResult:
    """P (B, N, N), q (B, N) device tensors; A (me, N), b (B, me), G (mi, N), h (B, mi) device
    tensors or None (rows shared by the batch); lb, ub (N,) device tensors or None."""
    B, N = q.shape
    dev = q.device
    me = 0 if A is None else A.shape[0]
    mi = 0 if G is None else G.shape[0]
    lo = torch.full((N,), -np.inf, dtype=F64, device=dev) if lb is None else lb
    hi = torch.full((N,), np.inf, dtype=F64, device=dev) if ub is None else ub
    FL = torch.isfinite(lo).to(F64).expand(B, N)
    FH = torch.isfinite(hi).to(F64).expand(B, N)
    lo_ = torch.where(torch.isfinite(lo), lo, torch.zeros_like(lo))
    hi_ = torch.where(torch.isfinite(hi), hi, torch.zeros_like(hi))
    both = torch.isfinite(lo) & torch.isfinite(hi)
    x0 = torch.zeros(N, dtype=F64, device=dev)
    x0 = torch.where(both, 0.5 * (lo_ + hi_), x0)
    x0 = torch.where(torch.isfinite(lo) & ~torch.isfinite(hi), lo_ + 1.0, x0)
    x0 = torch.where(~torch.isfinite(lo) & torch.isfinite(hi), hi_ - 1.0, x0)
    x = x0.expand(B, N).clone()
    zl, zh = FL.clone(), FH.clone()
    # G slacks s = h - G x > 0 and their multipliers zs
    s = (h - x @ G.T).clamp(min=1.0) if mi else torch.zeros((B, 0), dtype=F64, device=dev)
    zs = torch.ones_like(s)
    ya = torch.zeros((B, me), dtype=F64, device=dev)     # equality multipliers
    nfac = _NormalFactor(B, N, dev)
    ncomp = (FL + FH).sum(1) + mi
    ncomp = ncomp.clamp(min=1)
    rhs = torch.cat([b if me else torch.zeros((B, 0), dtype=F64, device=dev),
                     h if mi else torch.zeros((B, 0), dtype=F64, device=dev)], 1)
    bn = 1.0 + (rhs.abs().amax(1) if me + mi else torch.zeros(B, dtype=F64, device=dev))
    qn = 1.0 + q.abs().amax(1)
    done = torch.zeros(B, dtype=torch.bool, device=dev)
    iters = torch.zeros(B, dtype=torch.int32, device=dev)
    best_x = x.clone()
    best_ya = ya.clone()
    best_zs = zs.clone()
    best_zb = zh - zl
    best_merit = torch.full((B,), np.inf, dtype=F64, device=dev)
    best_it = torch.zeros(B, dtype=torch.int64, device=dev)

    def Px_of(v):
        return _mv(P, v.unsqueeze(2)).squeeze(2)

    for it in range(max_iter):
        sl = torch.where(FL > 0, (x - lo_).clamp(min=1e-200), torch.ones_like(x))
        sh = torch.where(FH > 0, (hi_ - x).clamp(min=1e-200), torch.ones_like(x))
        Px = Px_of(x)
        # stationarity: P x + q - A'ya + G'zs - zl + zh = 0
        rd = -(Px + q) + (ya @ A if me else 0.0) - (zs @ G if mi else 0.0) + zl - zh
        ra = (b - x @ A.T) if me else torch.zeros((B, 0), dtype=F64, device=dev)
        rg = (h - x @ G.T - s) if mi else torch.zeros((B, 0), dtype=F64, device=dev)
        pobj = 0.5 * (x * Px).sum(1) + (q * x).sum(1)
        gap = ((sl * zl * FL).sum(1) + (sh * zh * FH).sum(1) + (s * zs).sum(1))
        mu = gap / ncomp
        rp_n = torch.cat([ra.abs(), rg.abs()], 1).amax(1) if me + mi else torch.zeros(B, dtype=F64, device=dev)
        merit = torch.maximum(torch.maximum(rp_n / bn, rd.abs().amax(1) / qn), gap / (1.0 + pobj.abs()))
        merit = torch.where(torch.isnan(merit), torch.full_like(merit, np.inf), merit)
        better = (merit < best_merit) & ~done
        best_x = torch.where(better[:, None], x, best_x)
        best_ya = torch.where(better[:, None], ya, best_ya)
        best_zs = torch.where(better[:, None], zs, best_zs)
        best_zb = torch.where(better[:, None], zh - zl, best_zb)
        best_it = torch.where(better, torch.full_like(best_it, it), best_it)
        best_merit = torch.where(better, merit, best_merit)
        done = done | (merit < tol) | ((it - best_it > 6) & (best_merit < _INACCURATE))
        done = done | ~torch.isfinite(x).all(1)
        if bool(done.all()):
            break
        iters += (~done).to(torch.int32)
        Dg = (FL * zl / sl + FH * zh / sh)
        eg = zs / s                                            # G-row weights
        Dg = torch.where(done[:, None], torch.ones_like(Dg), Dg)
        eg = torch.where(done[:, None], torch.ones_like(eg), eg)
        H = P.clone()
        if mi:
            H = H + torch.matmul(G.T * eg.unsqueeze(1), G)
        H.diagonal(dim1=1, dim2=2).add_(Dg)
        failed = nfac.factor(H, 1e-12 * H.diagonal(dim1=1, dim2=2).abs() + 1e-300)
        if bool(failed.any()):               # K2 broke down even shifted: freeze at the best iterate
            done = done | failed
            if bool(done.all()):
                break

        def hsolve(R, refine=2):
            Y = nfac.solve_mat(R)
            for _ in range(refine):
                Y = Y + nfac.solve_mat(_mv(H, Y, R))
            return Y

        if me:
            HiA = hsolve(A.T.expand(B, N, me).contiguous())   # H^-1 A'
            S = A @ HiA
            S = S + torch.diag_embed(1e-14 * S.diagonal(dim1=1, dim2=2).abs())

        def bordered(f, g):                  # [H A'; A 0] [dx; -dya] = [f; g]
            Hf = hsolve(f.unsqueeze(2)).squeeze(2)
            if not me:
                return Hf, torch.zeros((B, 0), dtype=F64, device=dev)
            dya = torch.linalg.solve(S, g - Hf @ A.T)
            return Hf + torch.bmm(HiA, dya.unsqueeze(2)).squeeze(2), dya

        def direction(rl, rh, rs):
            # bounds: zl dx + sl dzl = rl, -zh dx + sh dzh = rh; G rows: zs ds + s dzs = rs,
            # G dx + ds = rg, stationarity (P + ...) dx - A'dya + G'dzs - dzl + dzh = rd
            dzs_part = (rs - zs * rg) / s                    # dzs = eg G dx + dzs_part
            f = rd + FL * rl / sl - FH * rh / sh
            if mi:
                f = f - dzs_part @ G
            dx, dya = bordered(f, ra)
            for _ in range(2):
                Hdx = _mv(H, dx.unsqueeze(2)).squeeze(2)
                e1 = f - (Hdx - (dya @ A if me else 0.0))
                e2 = (ra - dx @ A.T) if me else ra
                cx, cy = bordered(e1, e2)
                dx, dya = dx + cx, dya + cy
            dzl = FL * (rl - zl * dx) / sl
            dzh = FH * (rh + zh * dx) / sh
            if mi:
                gdx = dx @ G.T
                ds = rg - gdx
                dzs = eg * gdx + dzs_part
            else:
                ds = dzs = s
            return dx, dya, dzl, dzh, ds, dzs

        def steps(dx, dzl, dzh, ds, dzs):
            inf = torch.full_like(dx, np.inf)
            ap = torch.minimum(torch.where((FL > 0) & (dx < 0), -sl / dx, inf),
                               torch.where((FH > 0) & (dx > 0), sh / dx, inf)).amin(1)
            ad = torch.minimum(torch.where(dzl < 0, -zl / dzl, inf), torch.where(dzh < 0, -zh / dzh, inf)).amin(1)
            if mi:
                infs = torch.full_like(s, np.inf)
                ap = torch.minimum(ap, torch.where(ds < 0, -s / ds, infs).amin(1))
                ad = torch.minimum(ad, torch.where(dzs < 0, -zs / dzs, infs).amin(1))
            a = torch.minimum(ap, ad).clamp(max=1.0)          # one step (QP: primal and dual coupled)
            return a

        dx, dya, dzl, dzh, ds, dzs = direction(-sl * zl * FL, -sh * zh * FH, -s * zs)
        a = steps(dx, dzl, dzh, ds, dzs)[:, None]
        mu_aff = (((sl + a * dx) * (zl + a * dzl) * FL).sum(1) + ((sh - a * dx) * (zh + a * dzh) * FH).sum(1)
                  + ((s + a * ds) * (zs + a * dzs)).sum(1)) / ncomp
        sig = (mu_aff / mu).clamp(0, 1) ** 3
        smu = (sig * mu)[:, None]
        rl = FL * (smu - sl * zl - dx * dzl)
        rh = FH * (smu - sh * zh + dx * dzh)
        rs = smu - s * zs - ds * dzs
        dx, dya, dzl, dzh, ds, dzs = direction(rl, rh, rs)
        a = (0.995 * steps(dx, dzl, dzh, ds, dzs))[:, None]
        act = ~done[:, None]
        x = torch.where(act, x + a * dx, x)
        ya = torch.where(act, ya + a * dya, ya)
        zl = torch.where(act, zl + a * dzl, zl)
        zh = torch.where(act, zh + a * dzh, zh)
        if mi:
            s = torch.where(act, s + a * ds, s)
            zs = torch.where(act, zs + a * dzs, zs)
    status = torch.full_like(iters, _lib.PQ_MAX_ITER)
    status = torch.where(best_merit < _INACCURATE, torch.full_like(iters, _lib.PQ_SOLVED_INACCURATE), status)
    status = torch.where(best_merit < tol, torch.full_like(iters, _lib.PQ_SOLVED), status)
    Pb = _mv(P, best_x.unsqueeze(2)).squeeze(2)
    res = LPResult(best_x, best_ya, status, iters, 0.5 * (best_x * Pb).sum(1) + (q * best_x).sum(1), best_merit)
    # multipliers at the returned iterate in qpsolvers' signs (P x + q + A'y + G'z + z_box = 0):
    # y = -ya, z = zs (>= 0), z_box = zh - zl (upper bounds positive, lower negative)
    res.z = best_zs if mi else None
    res.z_box = best_zb
    res.Px = Pb
    return res


def active_set_polish(P, q, A, b, G, h, lb, ub, x, y, z, zb, rounds: int = 8):
    """Exact solve on the active set detected at an interior-point answer, for ONE problem
    (device tensors; y, z, zb in qpsolvers' signs: P x + q + A'y + G'z + z_box = 0).  The
    interior-point iterate stops at merit ~1e-9 with its weights accurate to ~1e-4 near
    degenerate faces; the reduced system [P_FF C_F'; C_F 0] on the free set F and the active
    rows C = [A; G_act] (P_FF factored and inverted on K2 / K2L, the rows bordered by a small
    Schur system, one step of iterative refinement) gives the optimum to rounding.  A short
    primal-dual active-set loop corrects the classification (the oracle's refinement,
    oracle/qp_ipm.py).  Returns (x, y, z, z_box, ok); ok False (P_FF not PD: the optimal
    face is not a point, or no consistent active set within ``rounds``) leaves the caller's
    iterate in place."""
    dev = q.device
    n = q.numel()
    me = 0 if A is None else A.shape[0]
    mi = 0 if G is None else G.shape[0]
    sc = float(max(P.abs().max().item(), q.abs().max().item(), 1e-300))
    Ps, qs = P / sc, q / sc
    inf = torch.full((n,), np.inf, dtype=F64, device=dev)
    lo = -inf if lb is None else lb
    up = inf if ub is None else ub
    at_lo = torch.isfinite(lo) & ((x - lo) < -zb)
    at_up = torch.isfinite(up) & ((up - x) < zb) & ~at_lo
    act = ((h - G @ x) < z) if mi else torch.zeros(0, dtype=torch.bool, device=dev)
    tol = 1e-12 * (1.0 + float(qs.abs().max().item()))
    for _ in range(rounds):
        fixed = at_lo | at_up
        xb = torch.where(at_lo, lo, torch.where(at_up, up, torch.zeros_like(x)))
        F = torch.nonzero(~fixed).flatten()
        nF = int(F.numel())
        C = torch.cat([A if me else torch.zeros((0, n), dtype=F64, device=dev),
                       G[act] if mi else torch.zeros((0, n), dtype=F64, device=dev)])
        d = torch.cat([b if me else torch.zeros(0, dtype=F64, device=dev),
                       h[act] if mi else torch.zeros(0, dtype=F64, device=dev)])
        m = C.shape[0]
        if nF == 0:
            return x, y, z, zb, False
        PFF = Ps[F][:, F].contiguous()
        rF = -(qs + Ps @ xb)[F]
        dF = d - C @ xb
        CF = C[:, F].contiguous()
        fac = _NormalFactor(1, nF, dev)
        if bool(fac.factor(PFF[None], 0.0, retries=0).any()):
            return x, y, z, zb, False
        HiC = fac.solve_mat(CF.T[None].contiguous())[0] if m else None
        if m:
            # Schur complement of the active rows, S = C_F P_FF^-1 C_F' (m x m, m <= a few
            # dozen; SPD, singular when active rows are linearly dependent).  Its pseudo-inverse
            # from a symmetric eigendecomposition on the device (eigenvalues below 1e-12 of the
            # largest dropped) gives the minimum-norm multipliers: a dependent row's share is
            # split evenly instead of scaled by 1 / shift (the former shifted Cholesky left x
            # right -- HiC annihilates that part -- but y / z arbitrarily large)
            S = 0.5 * (CF @ HiC + (CF @ HiC).T)
            ev, V = torch.linalg.eigh(S)
            keep = ev > 1e-12 * ev.abs().max().clamp(min=1e-300)
            Sp = (V * torch.where(keep, 1.0 / torch.where(keep, ev, torch.ones_like(ev)), torch.zeros_like(ev))) @ V.T

        def solve(f, g):
            hf = fac.solve_mat(f[None, :, None].contiguous())[0, :, 0]
            if not m:
                return hf, torch.zeros(0, dtype=F64, device=dev)
            r = CF @ hf - g
            lam = Sp @ r
            lam = lam + Sp @ (r - S @ lam)   # one refinement step
            return hf - HiC @ lam, lam

        xF, lam = solve(rF, dF)
        e1 = rF - (PFF @ xF + (CF.T @ lam if m else 0.0))
        e2 = dF - CF @ xF if m else dF
        cx, cl = solve(e1, e2)
        xF, lam = xF + cx, lam + cl
        xn = xb.clone()
        xn[F] = xF
        g = Ps @ xn + qs + (C.T @ lam if m else 0.0)
        zbn = torch.where(fixed, -g, torch.zeros_like(g))
        viol_lo = ~fixed & (xn < lo - 1e-13)
        viol_up = ~fixed & (xn > up + 1e-13)
        bad_lo = at_lo & (zbn > tol)
        bad_up = at_up & (zbn < -tol)
        zG = torch.zeros(mi, dtype=F64, device=dev)
        if mi:
            zG[act] = lam[me:]
            viol_G = ~act & ((G @ xn - h) > 1e-13)
            bad_G = act & (zG < -tol)
        else:
            viol_G = bad_G = torch.zeros(0, dtype=torch.bool, device=dev)
        flags = torch.stack([v.any() for v in (viol_lo, viol_up, bad_lo, bad_up)] +
                            ([viol_G.any(), bad_G.any()] if mi else []))
        if not bool(flags.any()):
            return xn, lam[:me] * sc, zG * sc, zbn * sc, True
        at_lo = (at_lo & ~bad_lo) | viol_lo
        at_up = (at_up & ~bad_up) | viol_up
        if mi:
            act = (act & ~bad_G) | viol_G
    return x, y, z, zb, False
