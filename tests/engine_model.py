"""numpy model of the engine's batched-QP algorithm (test infrastructure).

This is NOT the reference algorithm (that is ``oracle.qp_ipm``).  It restates, step by
step and for one problem, what the HIP kernels in ``porqua_amd/csrc`` compute
(Ruiz scaling, OSQP-style ADMM with an explicit K^-1, adaptive rho, active-set polish),
so GPU results can be compared with it iteration for iteration when debugging, and so
algorithm parameters can be tuned on the CPU.
"""
from __future__ import annotations

import numpy as np

INF = 1e30


def ruiz(P, q, C, iters=10, clip=(1e-4, 1e4)):
    n = P.shape[0]
    m = C.shape[0]
    D = np.ones(n)
    E = np.ones(m)
    Ps, qs, Cs = P.copy(), q.copy(), C.copy()
    for _ in range(iters):
        cn = np.maximum(np.max(np.abs(Ps), axis=0), np.max(np.abs(Cs), axis=0) if m else 0)
        rn = np.max(np.abs(Cs), axis=1) if m else np.zeros(0)
        cn = np.where(cn < clip[0], 1.0, np.minimum(cn, clip[1]))
        rn = np.where(rn < clip[0], 1.0, np.minimum(rn, clip[1]))
        dd = 1 / np.sqrt(cn)
        ee = 1 / np.sqrt(rn)
        Ps = dd[:, None] * Ps * dd[None, :]
        qs = dd * qs
        Cs = ee[:, None] * Cs * dd[None, :]
        D *= dd
        E *= ee
    cnorm = np.mean(np.max(np.abs(Ps), axis=0))
    c = 1 / max(cnorm, np.max(np.abs(qs)), clip[0])
    c = min(c, clip[1])
    return D, E, c, Ps * c, qs * c, Cs


def admm(P, q, C, l, u, rho=0.1, sigma=1e-6, alpha=1.6, eps_abs=1e-5, eps_rel=1e-5,
         max_iter=4000, scaling=10, adapt_interval=25, adapt_tol=5.0, verbose=False):
    n = P.shape[0]
    m = C.shape[0]
    D, E, c, Ps, qs, Cs = ruiz(P, q, C, scaling) if scaling else (
        np.ones(n), np.ones(m), 1.0, P.copy(), q.copy(), C.copy())
    ls = np.where(l <= -INF, -INF, l * E)
    us = np.where(u >= INF, INF, u * E)
    eq = (us - ls) < 1e-4 * 1  # OSQP RHO_TOL

    def rho_vec(r):
        rv = np.full(m, r)
        rv[eq] = 1e3 * r
        rv[(ls <= -INF) & (us >= INF)] = 1e-6
        return rv

    rv = rho_vec(rho)
    K = Ps + sigma * np.eye(n) + Cs.T @ (rv[:, None] * Cs)
    Kinv = np.linalg.inv(K)
    x = np.zeros(n); z = np.zeros(m); y = np.zeros(m); Px = np.zeros(n)
    nref = 0
    it = 0
    status = "max_iter"
    for it in range(1, max_iter + 1):
        rhs = sigma * x - qs + Cs.T @ (rv * z - y)
        xt = Kinv @ rhs
        zt = Cs @ xt
        Pxt = rhs - sigma * xt - Cs.T @ (rv * zt)
        x_new = alpha * xt + (1 - alpha) * x
        zh = alpha * zt + (1 - alpha) * z
        z_new = np.clip(zh + y / rv, ls, us)
        y = y + rv * (zh - z_new)
        Px = alpha * Pxt + (1 - alpha) * Px
        x, z = x_new, z_new
        Cx = Cs @ x
        Cty = Cs.T @ y
        rp = np.max(np.abs((Cx - z) / E), initial=0)
        rd = np.max(np.abs((Px + qs + Cty) / D)) / c
        ep = eps_abs + eps_rel * max(np.max(np.abs(Cx / E), initial=0), np.max(np.abs(z / E), initial=0))
        ed = eps_abs + eps_rel / c * max(np.max(np.abs(Px / D)), np.max(np.abs(Cty / D)),
                                         np.max(np.abs(qs / D)))
        if rp <= ep and rd <= ed:
            status = "solved"
            break
        if adapt_interval and it % adapt_interval == 0:
            rps = np.max(np.abs(Cx - z), initial=0) / (max(np.max(np.abs(Cx), initial=0), np.max(np.abs(z), initial=0)) + 1e-30)
            rds = np.max(np.abs(Px + qs + Cty)) / (max(np.max(np.abs(Px)), np.max(np.abs(Cty)), np.max(np.abs(qs))) + 1e-30)
            rn = np.clip(rho * np.sqrt(rps / (rds + 1e-30)), 1e-6, 1e6)
            if rn > rho * adapt_tol or rn < rho / adapt_tol:
                rho = rn
                rv = rho_vec(rho)
                K = Ps + sigma * np.eye(n) + Cs.T @ (rv[:, None] * Cs)
                Kinv = np.linalg.inv(K)
                nref += 1
    # unscale
    xu = D * x
    yu = E * y / c
    zu = z / E
    return dict(x=xu, y=yu, z=zu, iters=it, status=status, refactors=nref, rho=rho)


def polish(P, q, C, l, u, x, y, z, delta=1e-9, rounds=10, refine=8, dual_tol=1e-7):
    """Active-set polish: box rows eliminated, active general rows as equalities.

    The reduced KKT is solved by proximal iterative refinement started at the ADMM point
    (x_F, y_act): exact where the system is nonsingular, and staying at the ADMM
    multipliers along degenerate directions (e.g. every variable fixed at a bound)."""
    n = P.shape[0]
    m = C.shape[0]
    mg = m - n
    lo, up = l[mg:], u[mg:]
    yb = y[mg:]
    zb = z[mg:]
    at_lo = (lo > -INF) & (zb - lo < -yb)
    at_up = (up < INF) & (up - zb < yb) & ~at_lo
    Cg, lg, ug = C[:mg], l[:mg], u[:mg]
    yg, zg = y[:mg], z[:mg]
    act_lo = (lg > -INF) & (zg - lg < -yg)
    act_up = (ug < INF) & (ug - zg < yg)
    act = act_lo | act_up | (np.abs(ug - lg) < 1e-12)
    xn = x.copy()
    lam = yg.copy()
    zbox = np.zeros(n)
    for r in range(rounds):
        fixed = at_lo | at_up
        xb = np.where(at_lo, lo, np.where(at_up, up, 0.0))
        F = np.flatnonzero(~fixed)
        B = np.flatnonzero(fixed)
        rhs_row = np.where(act_lo & ~act_up, lg, ug)
        Ca = Cg[act]
        da = rhs_row[act]
        rF = -q[F] - P[np.ix_(F, B)] @ xb[B]
        dF = da - Ca[:, B] @ xb[B]
        CF = Ca[:, F]
        k = len(F)
        ma = CF.shape[0]
        M = np.zeros((k + ma, k + ma))
        M[:k, :k] = P[np.ix_(F, F)]
        M[:k, k:] = CF.T
        M[k:, :k] = CF
        Mreg = M.copy()
        Mreg[:k, :k] += delta * np.eye(k)
        Mreg[k:, k:] -= delta * np.eye(ma)
        rhs = np.concatenate([rF, dF])
        sol = np.concatenate([xn[F], lam[act]])
        for _ in range(refine):
            sol = sol + np.linalg.solve(Mreg, rhs - M @ sol)
        xn = xb.copy(); xn[F] = sol[:k]
        lam = np.zeros(mg); lam[act] = sol[k:]
        g = P @ xn + q + Cg.T @ lam
        zbox = np.where(fixed, -g, 0.0)
        viol_lo = ~fixed & (xn < lo - 1e-12)
        viol_up = ~fixed & (xn > up + 1e-12)
        bad_lo = at_lo & (zbox > dual_tol)
        bad_up = at_up & (zbox < -dual_tol)
        if not (viol_lo.any() or viol_up.any() or bad_lo.any() or bad_up.any()):
            return xn, lam, zbox, r + 1, True
        at_lo = (at_lo & ~bad_lo) | viol_lo
        at_up = (at_up & ~bad_up) | viol_up
    return xn, lam, zbox, rounds, False
