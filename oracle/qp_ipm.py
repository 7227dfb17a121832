"""Dense primal-dual interior-point QP solver (TEST INFRASTRUCTURE ONLY).

The reference solves each rebalance date's QP through the third-party ``qpsolvers``
package (``src/qp_problems.py:184-216``; default backend ``cvxopt``,
``src/optimization.py:45``).  Neither ``qpsolvers`` (unpinned; the API used implies
>= 3.x) nor any backend is present in the reference tree or in this image, so this
module restates the published algorithm of cvxopt's ``coneqp`` for the nonnegative
orthant: a Mehrotra predictor-corrector primal-dual path-following method on

    min 0.5 x'Px + q'x   s.t.  Gx <= h,  Ax = b,  lb <= x <= ub

followed by an active-set refinement (an exact equality-constrained solve on the
detected active set) so that golden optima are accurate to ~1e-12 when P is PD on the
active face.  The returned ``OracleSolution`` exposes the qpsolvers ``Solution``
fields the reference reads (``found``, ``x``, ``obj``, ``y``, ``z``, ``z_box``) and the
residual definitions of ``example/compare_solver.ipynb:212-216``.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np
import scipy.linalg as sla


@dataclass
class OracleSolution:
    P: np.ndarray
    q: np.ndarray
    G: np.ndarray | None
    h: np.ndarray | None
    A: np.ndarray | None
    b: np.ndarray | None
    lb: np.ndarray | None
    ub: np.ndarray | None
    x: np.ndarray | None = None
    y: np.ndarray | None = None
    z: np.ndarray | None = None
    z_box: np.ndarray | None = None
    found: bool = False
    iterations: int = 0
    extras: dict = field(default_factory=dict)

    @property
    def obj(self):
        if self.x is None:
            return None
        return float(0.5 * self.x @ self.P @ self.x + self.q @ self.x)

    def primal_residual(self) -> float:
        """max(||Ax-b||inf, [Gx-h]+, [lb-x]+, [x-ub]+)  (compare_solver.ipynb:212-214)."""
        x = self.x
        r = 0.0
        if self.A is not None:
            r = max(r, float(np.max(np.abs(self.A @ x - self.b), initial=0.0)))
        if self.G is not None:
            r = max(r, float(np.max(np.maximum(self.G @ x - self.h, 0.0), initial=0.0)))
        if self.lb is not None:
            r = max(r, float(np.max(np.maximum(self.lb - x, 0.0), initial=0.0)))
        if self.ub is not None:
            r = max(r, float(np.max(np.maximum(x - self.ub, 0.0), initial=0.0)))
        return r

    def dual_residual(self) -> float:
        """||Px + q + A'y + G'z + z_box||inf  (compare_solver.ipynb:215-216)."""
        g = self.P @ self.x + self.q
        if self.A is not None:
            g = g + self.A.T @ self.y
        if self.G is not None:
            g = g + self.G.T @ self.z
        if self.z_box is not None:
            g = g + self.z_box
        return float(np.max(np.abs(g)))

    def duality_gap(self) -> float:
        """|x'Px + q'x + b'y + h'z + lb'min(z_box,0) + ub'max(z_box,0)| (qpsolvers semantics)."""
        x = self.x
        gap = x @ self.P @ x + self.q @ x
        if self.A is not None:
            gap += self.b @ self.y
        if self.G is not None:
            gap += self.h @ self.z
        if self.z_box is not None:
            if self.lb is not None:
                fin = np.isfinite(self.lb)
                gap += self.lb[fin] @ np.minimum(self.z_box, 0.0)[fin]
            if self.ub is not None:
                fin = np.isfinite(self.ub)
                gap += self.ub[fin] @ np.maximum(self.z_box, 0.0)[fin]
        return float(abs(gap))


def _as2d(M, n):
    if M is None:
        return None
    M = np.asarray(M, dtype=np.float64)
    return M.reshape(-1, n)


class SingularKKT(Exception):
    """The (1,1) block is not numerically positive definite (Cholesky breakdown)."""


def _chol(M):
    try:
        c = sla.cho_factor(M, lower=True, check_finite=False)
    except sla.LinAlgError:
        raise SingularKKT from None
    if not np.all(np.isfinite(c[0].diagonal())) or np.min(c[0].diagonal()) <= 0.0:
        raise SingularKKT
    return c


class _KKT:
    """Factor of [H + reg I, A'; A, -(D + reg I)] for repeated solves: the Cholesky of
    H + reg I and the Schur complement S = A (H + reg I)^-1 A' + D + reg I of the bordered
    rows -- cvxopt's 'chol2' KKT solver family.  Each solve takes one step of iterative
    refinement on the full system.  The multipliers of linearly dependent rows are not unique:
    S is solved in the minimum-norm sense.  When the Cholesky breaks down and ``shift`` is set,
    it is retried on H + 1e-14 max|diag H| I (an inexact Newton direction, harmless to a
    path-following method whose residuals are recomputed from the iterate every iteration);
    ``shift=False`` raises SingularKKT instead (exact solves only)."""

    def __init__(self, H, A, reg=0.0, shift=True, D=None):
        n = H.shape[0]
        self.H, self.A, self.reg = H, A, reg
        self.me = me = 0 if A is None else A.shape[0]
        self.n = n
        if n == 0:
            return
        M = H + reg * np.eye(n) if reg else H
        try:
            self.c = _chol(M)
        except SingularKKT:
            if not shift:
                raise
            M = M + 1e-14 * max(float(np.max(np.abs(np.diag(H)))), 1e-300) * np.eye(n)
            self.c = _chol(M)
        Dv = np.zeros(me) if D is None else np.asarray(D, dtype=np.float64)
        self.Dv = Dv + reg if reg else Dv
        if me:
            self.HiA = sla.cho_solve(self.c, A.T, check_finite=False)
            self.S = A @ self.HiA + np.diag(self.Dv)

    def _solve1(self, f, g):
        hf = sla.cho_solve(self.c, f, check_finite=False)
        if not self.me:
            return hf, np.zeros(0)
        dy = np.linalg.lstsq(self.S, self.A @ hf - g, rcond=1e-13)[0]
        return hf - self.HiA @ dy, dy

    def solve(self, r1, r2):
        if self.n == 0:   # every variable fixed: no primal unknowns, the multipliers stay undetermined (0)
            return np.zeros(0), np.zeros(self.me)
        A, me = self.A, self.me
        x, y = self._solve1(r1, r2)
        e1 = r1 - (self.H @ x + self.reg * x + (A.T @ y if me else 0.0))
        e2 = (r2 - (A @ x - self.Dv * y)) if me else np.zeros(0)
        cx, cy = self._solve1(e1, e2)
        return x + cx, (y + cy if me else np.zeros(0))


def _kkt_solve_indefinite(H, A, r1, r2):
    """[H A'; A 0] [x; y] = [r1; r2] by LAPACK's symmetric-indefinite solver (sysv), raising
    (LinAlgError / LinAlgWarning) instead of returning an ill-conditioned answer."""
    import warnings
    n, me = H.shape[0], A.shape[0]
    K = np.zeros((n + me, n + me))
    K[:n, :n] = H
    K[:n, n:] = A.T
    K[n:, :n] = A
    with warnings.catch_warnings():
        warnings.simplefilter("error", sla.LinAlgWarning)
        sol = sla.solve(K, np.concatenate([r1, r2]), assume_a="sym")
    if not np.all(np.isfinite(sol)):
        raise sla.LinAlgError("non-finite KKT solution")
    return sol[:n], sol[n:]


def _kkt_solve_lstsq(H, A, r1, r2):
    """Minimum-norm least-squares solution of [H A'; A 0] [x; y] = [r1; r2] (SVD-based)."""
    n, me = H.shape[0], A.shape[0]
    K = np.zeros((n + me, n + me))
    K[:n, :n] = H
    K[:n, n:] = A.T
    K[n:, :n] = A
    sol = np.linalg.lstsq(K, np.concatenate([r1, r2]), rcond=None)[0]
    return sol[:n], sol[n:]


def _kkt_solve(H, A, r1, r2, reg=0.0, shift=True, D=None):
    """One solve with a fresh _KKT factor."""
    return _KKT(H, A, reg=reg, shift=shift, D=D).solve(r1, r2)


def solve_qp(P, q, G=None, h=None, A=None, b=None, lb=None, ub=None,
             tol=1e-12, max_iter=200, refine=True) -> OracleSolution:
    """Solve with the objective scaled to unit magnitude (tolerances are then relative),
    and report x / duals of the original problem."""
    P = np.asarray(P, dtype=np.float64)
    q = np.asarray(q, dtype=np.float64).reshape(-1)
    s = max(float(np.max(np.abs(P), initial=0.0)), float(np.max(np.abs(q), initial=0.0)))
    s = 1.0 if s == 0.0 or not np.isfinite(s) else 1.0 / s
    sol = _solve_qp_scaled(P * s, q * s, G, h, A, b, lb, ub, tol, max_iter, refine)
    out = OracleSolution(np.asarray(P, dtype=np.float64), q, sol.G, sol.h, sol.A, sol.b,
                         sol.lb, sol.ub)
    out.x, out.found, out.iterations, out.extras = sol.x, sol.found, sol.iterations, sol.extras
    out.y = None if sol.y is None else sol.y / s
    out.z = None if sol.z is None else sol.z / s
    out.z_box = None if sol.z_box is None else sol.z_box / s
    out.extras["kkt_primal"] = out.primal_residual()
    out.extras["kkt_dual"] = out.dual_residual()
    return out


def _solve_qp_scaled(P, q, G, h, A, b, lb, ub, tol, max_iter, refine) -> OracleSolution:
    P = np.asarray(P, dtype=np.float64)
    n = P.shape[0]
    P = 0.5 * (P + P.T)
    q = np.asarray(q, dtype=np.float64).reshape(n)
    G = _as2d(G, n)
    A = _as2d(A, n)
    h = None if h is None else np.asarray(h, dtype=np.float64).reshape(-1)
    b = None if b is None else np.asarray(b, dtype=np.float64).reshape(-1)
    lb = None if lb is None else np.asarray(lb, dtype=np.float64).reshape(n)
    ub = None if ub is None else np.asarray(ub, dtype=np.float64).reshape(n)
    sol = OracleSolution(P, q, G, h, A, b, lb, ub)

    # stacked inequalities  Gh x <= hh  :  [G; -I_L; I_U]
    Lidx = np.flatnonzero(np.isfinite(lb)) if lb is not None else np.zeros(0, int)
    Uidx = np.flatnonzero(np.isfinite(ub)) if ub is not None else np.zeros(0, int)
    mi = 0 if G is None else G.shape[0]
    rows = [G] if G is not None else []
    hs = [h] if G is not None else []
    if len(Lidx):
        E = np.zeros((len(Lidx), n)); E[np.arange(len(Lidx)), Lidx] = -1.0
        rows.append(E); hs.append(-lb[Lidx])
    if len(Uidx):
        E = np.zeros((len(Uidx), n)); E[np.arange(len(Uidx)), Uidx] = 1.0
        rows.append(E); hs.append(ub[Uidx])
    Gh = np.vstack(rows) if rows else np.zeros((0, n))
    hh = np.concatenate(hs) if hs else np.zeros(0)
    m = Gh.shape[0]
    me = 0 if A is None else A.shape[0]
    bb = np.zeros(0) if b is None else b

    # initial point (coneqp style): [P A' Gh'; A 0 0; Gh 0 -I] [x;y;z] = [-q; b; hh]
    H0 = P + Gh.T @ Gh
    x, y = _kkt_solve(H0, A, -q + Gh.T @ hh, bb, reg=1e-12)
    s = hh - Gh @ x
    z = -s.copy()
    if m:
        a = -np.min(s)
        if a >= -1e-8:
            s = s + 1 + a
        a = -np.min(z)
        if a >= -1e-8:
            z = z + 1 + a
    nq = 1 + np.max(np.abs(q))
    nb = 1 + (np.max(np.abs(bb)) if me else 0.0)
    nh = 1 + (np.max(np.abs(hh)) if m else 0.0)
    it = 0
    best = (np.inf, None)
    stall = 0
    for it in range(1, max_iter + 1):
        rd = P @ x + q + (A.T @ y if me else 0.0) + Gh.T @ z
        rp = (A @ x - bb) if me else np.zeros(0)
        ri = Gh @ x + s - hh
        mu = (s @ z) / m if m else 0.0
        pres = max(np.max(np.abs(rp), initial=0.0) / nb, np.max(np.abs(ri), initial=0.0) / nh)
        dres = np.max(np.abs(rd)) / nq
        gapr = mu * m / (1 + abs(0.5 * x @ P @ x + q @ x))
        if pres < tol and dres < tol and gapr < tol:
            break
        merit = max(pres, dres, gapr)
        if merit < 0.5 * best[0]:
            best = (merit, (x.copy(), y.copy(), s.copy(), z.copy()))
            stall = 0
        else:
            stall += 1
            if stall >= 8:  # numerical floor reached: keep the best iterate
                x, y, s, z = best[1]
                break
        w = z / s if m else np.zeros(0)
        # Newton system, box rows (unit rows of Gh) folded into H as a diagonal.  The general
        # rows G are folded too (H + G'diag(w_G)G, as coneqp's chol2 does) unless that
        # Cholesky breaks down: an active row's weight z/s reaches ~1e23 and leaves a rank-mi
        # spike FP64 cannot resolve; then they stay bordered, C = [A; G], D = [0; s_G/z_G],
        # where the spike is the harmless entry s/z ~ 1e-23.
        Hd = P.copy()
        dg = np.zeros(n)
        np.add.at(dg, Lidx, w[mi:mi + len(Lidx)])
        np.add.at(dg, Uidx, w[mi + len(Lidx):])
        Hd[np.diag_indices(n)] += dg
        kkt, bordered = None, False
        if mi:
            try:
                kkt = _KKT(Hd + (G.T * w[:mi]) @ G, A if me else None, shift=False)
            except SingularKKT:
                C = np.vstack([A if me else np.zeros((0, n)), G])
                kkt = _KKT(Hd, C, D=np.concatenate([np.zeros(me), s[:mi] / z[:mi]]))
                bordered = True
        else:
            kkt = _KKT(Hd, A if me else None)

        def newton(rc):
            # ds = -ri - Gh dx ; dz = (-rc - z ds) / s   (all rows); box rows eliminated:
            #   H dx + A'dy + G'dz_G = -rd - E'((-rc_b + z_b ri_b)/s_b),  A dx = -rp,
            # and the general rows either folded (dz_G = ((-rc_G + z_G ri_G) + z_G G dx)/s_G)
            # or bordered:  G dx - (s_G/z_G) dz_G = -(-rc_G + z_G ri_G)/z_G
            vb = (-rc[mi:] + z[mi:] * ri[mi:]) / s[mi:]
            r1 = -rd - Gh[mi:].T @ vb if m > mi else -rd
            vg = (-rc[:mi] + z[:mi] * ri[:mi])
            if bordered:
                dx, dl = kkt.solve(r1, np.concatenate([-rp, -vg / z[:mi]]))
                dy = dl[:me]
            else:
                if mi:
                    r1 = r1 - G.T @ (vg / s[:mi])
                dx, dy = kkt.solve(r1, -rp)
            ds = -ri - Gh @ dx
            dz = (-rc - z * ds) / s if m else np.zeros(0)
            return dx, dy, ds, dz

        def max_step(v, dv):
            neg = dv < 0
            if not np.any(neg):
                return 1.0
            return min(1.0, float(np.min(-v[neg] / dv[neg])))

        if m:
            dx_a, dy_a, ds_a, dz_a = newton(s * z)
            a_aff = min(max_step(s, ds_a), max_step(z, dz_a))
            mu_aff = ((s + a_aff * ds_a) @ (z + a_aff * dz_a)) / m
            sigma = (mu_aff / mu) ** 3 if mu > 0 else 0.0
            rc = s * z + ds_a * dz_a - sigma * mu
            dx, dy, ds, dz = newton(rc)
            a = min(1.0, 0.99 * min(max_step(s, ds), max_step(z, dz)))
        else:
            dx, dy, ds, dz = newton(np.zeros(0))
            a = 1.0
        x = x + a * dx
        y = y + a * dy if me else y
        s = s + a * ds
        z = z + a * dz
        if m:
            s = np.maximum(s, 1e-300)
            z = np.maximum(z, 1e-300)

    zG = z[:mi] if mi else (np.zeros(0) if G is not None else None)
    zbox = np.zeros(n)
    if len(Lidx):
        zbox[Lidx] -= z[mi:mi + len(Lidx)]
    if len(Uidx):
        zbox[Uidx] += z[mi + len(Lidx):]
    sol.x, sol.y, sol.z = x, (y if me else (np.zeros(0) if A is not None else None)), zG
    sol.z_box = zbox if (lb is not None or ub is not None) else None
    sol.iterations = it
    sol.found = bool(np.all(np.isfinite(x)))
    if refine and sol.found:
        _refine_active_set(sol)
    sol.extras["kkt_primal"] = sol.primal_residual()
    sol.extras["kkt_dual"] = sol.dual_residual()
    return sol


def _refine_active_set(sol: OracleSolution, max_rounds: int = 30):
    """Exact solve on the detected active set (a short primal-dual active-set loop started
    from the IPM classification); kept only if it improves the KKT residuals."""
    P, q, G, h, A, b, lb, ub = sol.P, sol.q, sol.G, sol.h, sol.A, sol.b, sol.lb, sol.ub
    n = P.shape[0]
    x = sol.x
    lo = np.full(n, -np.inf) if lb is None else lb
    up = np.full(n, np.inf) if ub is None else ub
    zbox = np.zeros(n) if sol.z_box is None else sol.z_box
    at_lo = np.isfinite(lo) & (x - lo < -zbox)
    at_up = np.isfinite(up) & (up - x < zbox) & ~at_lo
    mi = 0 if G is None else G.shape[0]
    act_G = np.zeros(mi, bool)
    if mi:
        act_G = (h - G @ x) < sol.z
    me = 0 if A is None else A.shape[0]
    best = None
    for _ in range(max_rounds):
        fixed = at_lo | at_up
        xb = np.where(at_lo, lo, np.where(at_up, up, 0.0))
        F = np.flatnonzero(~fixed)
        Bi = np.flatnonzero(fixed)
        rowsC, rhsC = [], []
        if me:
            rowsC.append(A); rhsC.append(b)
        if act_G.any():
            rowsC.append(G[act_G]); rhsC.append(h[act_G])
        C = np.vstack(rowsC) if rowsC else np.zeros((0, n))
        d = np.concatenate(rhsC) if rhsC else np.zeros(0)
        rF = -q[F] - (P[np.ix_(F, Bi)] @ xb[Bi] if len(Bi) else 0.0)
        dF = d - (C[:, Bi] @ xb[Bi] if len(Bi) else 0.0)
        try:   # exact solves only
            xF, lam = _kkt_solve(P[np.ix_(F, F)], C[:, F] if C.shape[0] else None, rF, dF, shift=False)
        except SingularKKT:
            # P_FF singular: the bordered system can still be nonsingular when the active rows
            # pin the null directions down (e.g. the auxiliary variables of the l1
            # linearisations, P = 0 on them); solved by a symmetric-indefinite factorisation.
            # If that is singular too, the optimal face is not a point (e.g. x+ and x- of the
            # leverage split both positive for an asset): the minimum-norm least-squares
            # solution of the consistent system is one exact point of the face.  Either way
            # the candidate is kept only if it improves the KKT residuals (below).
            try:
                xF, lam = _kkt_solve_indefinite(P[np.ix_(F, F)], C[:, F], rF, dF)
            except (sla.LinAlgError, sla.LinAlgWarning, ValueError):
                xF, lam = _kkt_solve_lstsq(P[np.ix_(F, F)], C[:, F], rF, dF)
        xn = xb.copy()
        xn[F] = xF
        y = lam[:me] if me else None
        zG = np.zeros(mi)
        if act_G.any():
            zG[act_G] = lam[me:]
        g = P @ xn + q
        if me:
            g = g + A.T @ y
        if mi:
            g = g + G.T @ zG
        zb = np.where(fixed, -g, 0.0)
        tol = 1e-12 * (1 + np.max(np.abs(q)))
        viol_lo = (~fixed) & (xn < lo - 1e-13)
        viol_up = (~fixed) & (xn > up + 1e-13)
        bad_lo = at_lo & (zb > tol)
        bad_up = at_up & (zb < -tol)
        viol_G = (~act_G) & ((G @ xn - h) > 1e-13) if mi else np.zeros(0, bool)
        bad_G = act_G & (zG < -tol) if mi else np.zeros(0, bool)
        if not (viol_lo.any() or viol_up.any() or bad_lo.any() or bad_up.any()
                or viol_G.any() or bad_G.any()):
            best = (xn, y, zG, zb)
            break
        # add the worst primal violators, release wrong-sign duals
        at_lo = (at_lo & ~bad_lo) | viol_lo
        at_up = (at_up & ~bad_up) | viol_up
        if mi:
            act_G = (act_G & ~bad_G) | viol_G
    if best is None:
        sol.extras["refined"] = False
        return
    cand = OracleSolution(P, q, G, h, A, b, lb, ub)
    cand.x, cand.y = best[0], (best[1] if A is not None else None)
    cand.z = best[2] if G is not None else None
    cand.z_box = best[3] if sol.z_box is not None else None
    old = max(sol.primal_residual(), sol.dual_residual())
    new = max(cand.primal_residual(), cand.dual_residual())
    if np.all(np.isfinite(cand.x)) and new <= max(old, 1e-12):
        sol.x, sol.y, sol.z, sol.z_box = cand.x, cand.y, cand.z, cand.z_box
        sol.extras["refined"] = True
    else:
        sol.extras["refined"] = False
