"""Turnover (cost or budget) and leverage together, batched over rebalance dates.

``model_qpsolvers`` (src/optimization.py:125-142) linearises a turnover term around x0 and a
leverage budget with extra variables and rows (src/qp_problems.py:40-157): d >= |x - x0|
(2n rows + the budget row, or a cost c'd) and x = x- - x+ with 1'(x+ + x-) <= L (n equality
rows).  The ADMM engine covers one such term as a signed split (porqua_amd/l1split.py); both
together are solved here by a batched primal-dual interior-point method on the same optimum
written with per-asset blocks:

    min 1/2 |t|^2 + 1/2 x' diag(pd) x + q'x + c 1'(u + v)
    s.t.  U_W x - t = 0                  (T' window rows: P = U_W'U_W + diag(pd))
          A x = b,  G x + s_g = h         (budget / group rows of Constraints.to_GhAb)
          1'(u + v) + s_t = tau           (turnover budget; absent for the cost form)
          1'(p + m) + s_L = L             (leverage budget)
          x - u + v = x0,  x - p + m = 0  (per asset)
          lb <= x <= ub;  u, v, p, m, s >= 0

(u - v = x - x0 and p - m = x are the signed parts; every optimum is complementary, so the
x-optimum is the reference's.)  U_W is the window in window form (sqrt(p_scale w_scale) Xc,
T' = T < n) or any square root of a dense P (T' = n).

Newton systems are reduced exactly to the k x k coupling system, k = T' + me + mi + 1 or 2:
the per-asset 5 x 5 block (x, u, v, p, m) with its two local rows is eliminated through the
null space of those rows, N = [n1 = (1,1,0,1,0), n2 = (0,1,1,0,0), n3 = (0,0,0,1,1)], whose
3 x 3 matrix N'HN and every entry of K = (CN)(N'HN)^-1(CN)' have closed forms that are sums
of positive terms (no cancellation however the barrier weights spread).  The coupling
matrix is  S = [U diag(K_xx) U' + diag(d_U), U K_xt, U K_xL; ...; sum K_tt + th_t, ...],
its U-block formed by the hand-written FP64-MFMA weighted SYRK (pq_wgram_batched), bordered
by two GEMVs, factored + inverted on K2 and refined against the exact S.  Per iteration:
2 k^2 n flop (T = 252, n = 1000: 1.3e8) instead of the (3n)^3 / 3 of the reference's
linearised normal matrix.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np
import torch

from . import _lib, engine
from .lad import LPResult, _INACCURATE, _gemv, _mv, _NormalFactor

F64 = torch.float64


@dataclass
class L1Terms:
    """The linearisations model_qpsolvers applies (src/optimization.py:125-142): a turnover
    term around x0 -- cost c 1'd in the objective (``cost``) or the budget 1'd <= tau
    (``to_budget``) -- and a leverage budget 1'|x| <= ``lev_budget``."""
    x0: np.ndarray
    cost: float = 0.0
    to_budget: float | None = None
    lev_budget: float = np.inf


def block_k(dx, du, dv, dp, dm):
    """Closed forms of the per-asset elimination (all sums of positive terms):
    det(N'HN) and K = (CN) (N'HN)^-1 (CN)' on the coupling types (x-rows, turnover row,
    leverage row), CN = [[1,0,0],[1,2,0],[1,0,2]].  Returns (det, cof, K) with cof the
    cofactors (c11, c12, c13, c22, c23, c33) of N'HN = [[dx+du+dp, du, dp], [du, du+dv, 0],
    [dp, 0, dp+dm]]."""
    # G and K are homogeneous of degree -1 in the weights: evaluate them on the weights
    # divided by their per-asset maximum (no overflow of the triple products however large
    # a barrier weight grows) and scale back
    sc = torch.maximum(torch.maximum(torch.maximum(dx, du), torch.maximum(dv, dp)), dm)
    dx, du, dv, dp, dm = dx / sc, du / sc, dv / sc, dp / sc, dm / sc
    suv, spm = du + dv, dp + dm
    det = (suv * (dx * dp + dx * dm + dp * dm) + spm * du * dv) * sc
    c11 = suv * spm
    c12 = -du * spm
    c13 = -dp * suv
    c22 = (dx + du) * spm + dp * dm
    c23 = du * dp
    c33 = (dx + dp) * suv + du * dv
    K = {"xx": c11 / det,
         "xt": spm * (dv - du) / det,
         "xL": suv * (dm - dp) / det,
         "tt": (spm * (4 * dx + du + dv) + 4 * dp * dm) / det,
         "LL": (suv * (4 * dx + dp + dm) + 4 * du * dv) / det,
         "tL": (dv - du) * (dm - dp) / det}
    return det, (c11, c12, c13, c22, c23, c33), K


def block_solve(det, cof, a1, a2, a3):
    """(N'HN)^-1 a per asset."""
    c11, c12, c13, c22, c23, c33 = cof
    return ((c11 * a1 + c12 * a2 + c13 * a3) / det,
            (c12 * a1 + c22 * a2 + c23 * a3) / det,
            (c13 * a1 + c23 * a2 + c33 * a3) / det)


class _Coupling:
    """S for a batch (see the module docstring), factored on K2; ``solve`` refines against
    the exact S applied in structured form."""

    def __init__(self, U, budget: bool):
        self.U = U
        self.B, self.k0, self.n = U.shape
        self.budget = budget
        self.nb = 2 if budget else 1
        self.k = self.k0 + self.nb
        self.nf = _NormalFactor(self.B, self.k, U.device)
        self.k_ld = self.nf.qb.ld

    def factor(self, det, cof, K, dU, th_st, th_sL):
        self.det, self.cof, self.dU, self.th_st, self.th_sL = det, cof, dU, th_st, th_sL
        B, k0, n, U = self.B, self.k0, self.n, self.U
        P = self.nf.qb.P
        lib = _lib.load()
        stream = engine._stream()
        kxx = K["xx"].contiguous()
        dUc = dU.contiguous()
        for s in range(0, B, 65535):
            c = min(B, s + 65535) - s
            Us = U[s:s + c]
            _lib.check(lib.pq_wgram_batched(Us.data_ptr(), Us.stride(1), Us.stride(0), k0, n, c,
                                            kxx[s:].data_ptr(), kxx.stride(0), None, 0, dUc[s:].data_ptr(),
                                            dUc.stride(0), P[s:].data_ptr(), self.k_ld, P.stride(0), stream),
                       "pq_wgram_batched (l1 coupling)")
        r = k0
        if self.budget:
            P[:, r, :k0] = _gemv(U, K["xt"])
            P[:, r, r] = K["tt"].sum(1) + th_st
            r += 1
        P[:, r, :k0] = _gemv(U, K["xL"])
        if self.budget:
            P[:, r, r - 1] = K["tL"].sum(1)
        P[:, r, r] = K["LL"].sum(1) + th_sL
        nf = self.nf
        _lib.check(lib.pq_factor_batched(ctypes.byref(nf.pb), ctypes.byref(nf.st), None, 0,
                                         ctypes.byref(nf.s), 2, stream), "pq_factor_batched (l1 coupling)")
        # a breakdown (rounding, barrier weights spread over ~1e24) is refactored with a
        # growing diagonal shift, like the LAD / Woodbury normal matrices (lad._NormalFactor,
        # woodbury.NormalM): the shifted inverse is only the preconditioner of ``solve``,
        # which refines against the exact S, so the direction stays exact
        bad = nf.ws.info != 0
        kk = torch.arange(self.k, device=P.device)
        for attempt in range(3):
            if not bool(bad.any()):          # host sync: one small flag
                break
            idx = torch.nonzero(bad).flatten()
            d = P[idx[:, None], kk[None, :], kk[None, :]]
            P[idx[:, None], kk[None, :], kk[None, :]] = d + (1e-12 * 1e4 ** attempt) * d.abs().amax(1, keepdim=True).clamp(min=1e-300)
            idx32 = idx.to(torch.int32).contiguous()
            _lib.check(lib.pq_factor_batched(ctypes.byref(nf.pb), ctypes.byref(nf.st), idx32.data_ptr(),
                                             int(idx32.numel()), ctypes.byref(nf.s), 2, stream),
                       "pq_factor_batched (l1 coupling, shifted)")
            bad[idx] = nf.ws.info[idx] != 0
        self.Minv = nf.ws.K[:, :self.k, :self.k]
        return bad

    def split(self, y):
        k0 = self.k0
        yU = y[:, :k0]
        yt = y[:, k0] if self.budget else None
        yL = y[:, self.k - 1]
        return yU, yt, yL

    def nu(self, yU, yt, yL):
        """(CN)' y per asset: (U'y_U + y_t + y_L, 2 y_t, 2 y_L)."""
        n1 = _gemv(self.U, yU, True) + yL[:, None]
        n2 = torch.zeros_like(n1)
        if yt is not None:
            n1 = n1 + yt[:, None]
            n2 = (2.0 * yt)[:, None].expand_as(n1)
        n3 = (2.0 * yL)[:, None].expand_as(n1)
        return n1, n2, n3

    def apply(self, y):
        yU, yt, yL = self.split(y)
        w1, w2, w3 = block_solve(self.det, self.cof, *self.nu(yU, yt, yL))
        out = [_gemv(self.U, w1) + self.dU * yU]
        if self.budget:
            out.append(((w1 + 2 * w2).sum(1) + self.th_st * yt)[:, None])
        out.append(((w1 + 2 * w3).sum(1) + self.th_sL * yL)[:, None])
        return torch.cat(out, 1)

    def solve(self, g, refine: int = 2):
        Y = _mv(self.Minv, g.unsqueeze(2).contiguous()).squeeze(2)
        for _ in range(refine):
            Y = Y + _mv(self.Minv, (g - self.apply(Y)).unsqueeze(2).contiguous()).squeeze(2)
        return Y


def l1_ipm_batched(UW, pd, q, terms: L1Terms, A=None, b=None, G=None, h=None, lb=None, ub=None,
                   tol: float = 1e-12, max_iter: int = 100, trace=None) -> LPResult:
    """UW (B, T', n) device rows with P = UW'UW + diag(pd) (pd (B,) or None), q (B, n);
    A (me, n), b (me,), G (mi, n), h (mi,) shared host arrays or None; lb, ub (n,) or None.
    Returns an LPResult whose x is the weight vector (B, n) and obj the reference model's
    objective 1/2 x'Px + q'x + c 1'|x - x0|."""
    B, Tp, n = UW.shape
    dev = UW.device
    T = lambda v: torch.as_tensor(np.asarray(v, dtype=np.float64), device=dev)   # noqa: E731
    me = 0 if A is None else np.atleast_2d(A).shape[0]
    mi = 0 if G is None else np.atleast_2d(G).shape[0]
    rows = [UW]
    if me:
        rows.append(T(np.atleast_2d(A)).expand(B, me, n))
    if mi:
        rows.append(T(np.atleast_2d(G)).expand(B, mi, n))
    U = torch.cat(rows, 1).contiguous()
    k0 = Tp + me + mi
    bA = T(np.asarray(b).reshape(-1)) if me else None
    hG = T(np.asarray(h).reshape(-1)) if mi else None
    budget = terms.to_budget is not None
    tau = float(terms.to_budget) if budget else 0.0
    Lb = float(terms.lev_budget)
    c = float(terms.cost or 0.0)
    x0 = T(terms.x0).expand(B, n)
    pd = torch.zeros(B, dtype=F64, device=dev) if pd is None else pd
    lo = T(lb) if lb is not None else torch.full((n,), -np.inf, dtype=F64, device=dev)
    hi = T(ub) if ub is not None else torch.full((n,), np.inf, dtype=F64, device=dev)
    FL = torch.isfinite(lo).to(F64).expand(B, n)
    FH = torch.isfinite(hi).to(F64).expand(B, n)
    lo_ = torch.where(torch.isfinite(lo), lo, torch.zeros_like(lo))
    hi_ = torch.where(torch.isfinite(hi), hi, torch.zeros_like(hi))
    zeros = lambda *s: torch.zeros(s, dtype=F64, device=dev)   # noqa: E731
    ones = lambda *s: torch.ones(s, dtype=F64, device=dev)     # noqa: E731

    # ---- starting point: x mid-box, signed parts of x - x0 and x shifted into the interior
    xs = torch.where(torch.isfinite(lo) & torch.isfinite(hi), 0.5 * (lo_ + hi_),
                     torch.where(torch.isfinite(lo), lo_ + 1.0, torch.where(torch.isfinite(hi), hi_ - 1.0,
                                                                             torch.zeros_like(lo))))
    z = {"x": xs.expand(B, n).clone()}
    z["u"] = (z["x"] - x0).clamp(min=0) + 0.1
    z["v"] = (x0 - z["x"]).clamp(min=0) + 0.1
    z["p"] = z["x"].clamp(min=0) + 0.1
    z["m"] = (-z["x"]).clamp(min=0) + 0.1
    z["t"] = _gemv(UW, z["x"])
    z["sg"] = (hG - z["x"] @ T(np.atleast_2d(G)).T).clamp(min=0.1) if mi else zeros(B, 0)
    z["st"] = ones(B) if budget else zeros(B)
    z["sL"] = ones(B)
    lam = {"U": zeros(B, k0), "t": zeros(B), "L": zeros(B), "l1": zeros(B, n), "l2": zeros(B, n)}
    # bound multipliers: x (lower / upper, masked), the rest lower (>= 0)
    du = {"xl": FL.clone(), "xh": FH.clone(), "u": ones(B, n), "v": ones(B, n), "p": ones(B, n),
          "m": ones(B, n), "sg": ones(B, mi), "st": ones(B) if budget else zeros(B), "sL": ones(B)}
    low_vars = ("u", "v", "p", "m", "sg", "st", "sL")
    ncomp = (FL + FH).sum(1) + 4 * n + mi + (1 if budget else 0) + 1
    Gm = T(np.atleast_2d(G)) if mi else None
    Am = T(np.atleast_2d(A)) if me else None
    coup = _Coupling(U, budget)
    bn = 1.0 + max([abs(tau), abs(Lb)] + ([float(bA.abs().max())] if me else [])
                   + ([float(hG.abs().max())] if mi else []) + [float(np.abs(terms.x0).max())])
    qn = 1.0 + q.abs().amax(1) + c

    done = torch.zeros(B, dtype=torch.bool, device=dev)
    iters = torch.zeros(B, dtype=torch.int32, device=dev)
    best_x = z["x"].clone()
    best_merit = torch.full((B,), np.inf, dtype=F64, device=dev)
    best_it = torch.zeros(B, dtype=torch.int64, device=dev)

    def residuals(z, lam, du):
        Ux = _gemv(U, z["x"])                 # [UW x; A x; G x]
        rp = {"W": z["t"] - Ux[:, :Tp], "l1": x0 - (z["x"] - z["u"] + z["v"]), "l2": -(z["x"] - z["p"] + z["m"]),
              "L": Lb - (z["p"] + z["m"]).sum(1) - z["sL"]}
        rp["A"] = (bA - Ux[:, Tp:Tp + me]) if me else zeros(B, 0)
        rp["G"] = (hG - Ux[:, Tp + me:] - z["sg"]) if mi else zeros(B, 0)
        rp["t"] = (tau - (z["u"] + z["v"]).sum(1) - z["st"]) if budget else zeros(B)
        ATl = _gemv(U, lam["U"], True) + lam["l1"] + lam["l2"]
        lt = lam["t"] if budget else zeros(B)
        rd = {"x": pd[:, None] * z["x"] + q - ATl - du["xl"] + du["xh"],
              "u": c - lt[:, None] + lam["l1"] - du["u"], "v": c - lt[:, None] - lam["l1"] - du["v"],
              "p": -lam["L"][:, None] + lam["l2"] - du["p"], "m": -lam["L"][:, None] - lam["l2"] - du["m"],
              "t": z["t"] + lam["U"][:, :Tp], "sg": -lam["U"][:, Tp + me:] - du["sg"],
              "st": (-lt - du["st"]) if budget else zeros(B), "sL": -lam["L"] - du["sL"]}
        return rp, rd

    for it in range(max_iter):
        sl = {"x": torch.where(FL > 0, (z["x"] - lo_).clamp(min=1e-200), ones(B, n))}
        sh = torch.where(FH > 0, (hi_ - z["x"]).clamp(min=1e-200), ones(B, n))
        for k in low_vars:
            sl[k] = z[k].clamp(min=1e-200)
        rp, rd = residuals(z, lam, du)
        xPx = (z["t"] ** 2).sum(1) + pd * (z["x"] ** 2).sum(1)
        pobj = 0.5 * xPx + (q * z["x"]).sum(1) + c * (z["u"] + z["v"]).sum(1)
        gap = (sl["x"] * du["xl"] * FL).sum(1) + (sh * du["xh"] * FH).sum(1)
        for k in low_vars:
            g_k = sl[k] * du[k]
            gap = gap + (g_k.sum(1) if g_k.dim() == 2 else g_k)
        if not budget:
            gap = gap - sl["st"] * du["st"]
        mu = gap / ncomp
        rpn = torch.stack([v.abs().amax(1) if v.dim() == 2 and v.shape[1] else
                           (v.abs() if v.dim() == 1 else zeros(B)) for v in rp.values()], 1).amax(1)
        rdn = torch.stack([v.abs().amax(1) if v.dim() == 2 and v.shape[1] else
                           (v.abs() if v.dim() == 1 else zeros(B)) for v in rd.values()], 1).amax(1)
        merit = torch.maximum(torch.maximum(rpn / bn, rdn / qn), gap / (1.0 + pobj.abs()))
        merit = torch.where(torch.isnan(merit), torch.full_like(merit, np.inf), merit)
        if trace is not None:
            trace.append((it, float((rpn / bn).max()), float((rdn / qn).max()),
                          float((gap / (1.0 + pobj.abs())).max()),
                          {k: float(v.abs().max()) if v.numel() else 0.0 for k, v in rd.items()},
                          {k: float(v.abs().max()) if v.numel() else 0.0 for k, v in rp.items()}))
        better = (merit < best_merit) & ~done
        best_x = torch.where(better[:, None], z["x"], best_x)
        best_it = torch.where(better, torch.full_like(best_it, it), best_it)
        best_merit = torch.where(better, merit, best_merit)
        done = done | (merit < tol) | ((it - best_it > 8) & (best_merit < _INACCURATE))
        done = done | ~torch.isfinite(z["x"]).all(1)
        if bool(done.all()):
            break
        iters += (~done).to(torch.int32)
        act = ~done
        # barrier weights; frozen problems get any well-posed system
        D = {"x": (FL * du["xl"] / sl["x"] + FH * du["xh"] / sh)}
        for k in low_vars:
            D[k] = du[k] / sl[k]
        dx = (pd[:, None] + D["x"]).clamp(min=1e-14)
        dlt = {k: torch.where(act.view(-1, *([1] * (D[k].dim() - 1))), D[k], torch.ones_like(D[k])).clamp(min=1e-14)
               for k in ("u", "v", "p", "m", "sg", "st", "sL")}
        dx = torch.where(act[:, None], dx, torch.ones_like(dx))
        th_t = ones(B, Tp)                                # t: Q = 1, unbounded
        th_sg = 1.0 / dlt["sg"]
        th_st = (1.0 / dlt["st"]) if budget else zeros(B)
        th_sL = 1.0 / dlt["sL"]
        det, cof, K = block_k(dx, dlt["u"], dlt["v"], dlt["p"], dlt["m"])
        dU = torch.cat([th_t, zeros(B, me), th_sg], 1)
        failed = coup.factor(det, cof, K, dU, th_st, th_sL)
        if bool(failed.any()):
            done = done | failed
            if bool(done.all()):
                break

        def direction(rl, rh):
            # rl: lower-bound complementarity rhs per variable, rh: x's upper-bound rhs
            rx = {"x": rd["x"] - FL * rl["x"] / sl["x"] + FH * rh / sh}
            for k in low_vars:
                rx[k] = rd[k] - rl[k] / sl[k]
            rx["t"] = rd["t"]
            a1 = rx["x"] + rx["u"] + rx["p"]
            a2 = rx["u"] + rx["v"] + dlt["v"] * rp["l1"]
            a3 = rx["p"] + rx["m"] + dlt["m"] * rp["l2"]
            ga1, ga2, ga3 = block_solve(det, cof, a1, a2, a3)
            Uga = _gemv(U, ga1)
            gU = torch.cat([rp["W"], rp["A"], rp["G"]], 1) + Uga
            gU[:, :Tp] -= th_t * rx["t"]
            if mi:
                gU[:, Tp + me:] += th_sg * rx["sg"]
            g = [gU]
            if budget:
                g.append((rp["t"] - rp["l1"].sum(1) + (ga1 + 2 * ga2).sum(1) + th_st * rx["st"])[:, None])
            g.append((rp["L"] - rp["l2"].sum(1) + (ga1 + 2 * ga3).sum(1) + th_sL * rx["sL"])[:, None])
            dl = coup.solve(torch.cat(g, 1))
            dlU, dlt_, dlL = coup.split(dl)
            n1, n2, n3 = coup.nu(dlU, dlt_, dlL)
            w1, w2, w3 = block_solve(det, cof, n1, n2, n3)
            w1, w2, w3 = w1 - ga1, w2 - ga2, w3 - ga3
            # the per-asset step two ways: null space (above: local rows exact, the error of a
            # component ~ eps / (softest mode) -- large against a stiff weight) and range space
            # (each component theta_j (E'dl_l + C'dl_c - rx)_j: its H row exact, error ~ eps
            # theta_j -- large for a soft weight).  Each component takes the form that is
            # accurate for it: range space where its weight exceeds the block's geometric mean.
            lt2 = dlt_[:, None] if budget else 0.0
            yv = {"x": _gemv(U, dlU, True) - rx["x"],
                  "u": lt2 - rx["u"], "v": lt2 - rx["v"], "p": dlL[:, None] - rx["p"], "m": dlL[:, None] - rx["m"]}
            th = {"x": 1.0 / dx, "u": 1.0 / dlt["u"], "v": 1.0 / dlt["v"], "p": 1.0 / dlt["p"], "m": 1.0 / dlt["m"]}
            r1 = rp["l1"] - (th["x"] * yv["x"] - th["u"] * yv["u"] + th["v"] * yv["v"])
            r2 = rp["l2"] - (th["x"] * yv["x"] - th["p"] * yv["p"] + th["m"] * yv["m"])
            s11, s22, s12 = th["x"] + th["u"] + th["v"], th["x"] + th["p"] + th["m"], th["x"]
            dl_ = th["x"] * (th["u"] + th["v"] + th["p"] + th["m"]) + (th["u"] + th["v"]) * (th["p"] + th["m"])
            l1r = (s22 * r1 - s12 * r2) / dl_
            l2r = (s11 * r2 - s12 * r1) / dl_
            zr = {"x": th["x"] * (l1r + l2r + yv["x"]), "u": th["u"] * (yv["u"] - l1r), "v": th["v"] * (yv["v"] + l1r),
                  "p": th["p"] * (yv["p"] - l2r), "m": th["m"] * (yv["m"] + l2r)}
            zn = {"x": w1, "u": w1 + w2, "v": w2 + rp["l1"], "p": w1 + w3, "m": w3 + rp["l2"]}
            dmin = torch.minimum(torch.minimum(torch.minimum(dx, dlt["u"]), torch.minimum(dlt["v"], dlt["p"])), dlt["m"])
            dmax = torch.maximum(torch.maximum(torch.maximum(dx, dlt["u"]), torch.maximum(dlt["v"], dlt["p"])), dlt["m"])
            gm = (dmin * dmax).sqrt()
            dw = {"x": dx, "u": dlt["u"], "v": dlt["v"], "p": dlt["p"], "m": dlt["m"]}
            pick = {k: torch.where(dw[k] > gm, zr[k], zn[k]) for k in zn}
            dz = {"x": pick["x"], "u": pick["u"], "v": pick["v"], "p": pick["p"], "m": pick["m"],
                  "t": th_t * (-dlU[:, :Tp] - rx["t"]),
                  "sg": th_sg * (dlU[:, Tp + me:] - rx["sg"]),
                  "st": th_st * (dlt_ - rx["st"]) if budget else zeros(B),
                  "sL": th_sL * (dlL - rx["sL"])}
            dlam = {"U": dlU, "t": dlt_ if budget else zeros(B), "L": dlL, "l1": l1r, "l2": l2r}
            if trace is not None:   # Newton-row residuals of the direction (diagnostics)
                lt2 = dlt_[:, None] if budget else 0.0
                ru = dlt["u"] * dz["u"] - (lt2 - dlam["l1"]) + rx["u"]
                rv = dlt["v"] * dz["v"] - (lt2 + dlam["l1"]) + rx["v"]
                ATd = _gemv(U, dlU, True) + dlam["l1"] + dlam["l2"]
                rxx = dx * dz["x"] - ATd + rx["x"]
                trace.append(("newton", float(ru.abs().max()), float(rv.abs().max()), float(rxx.abs().max()),
                              float(dlt["u"].max()), float(dlt["v"].max())))
            ddu = {"xl": FL * (rl["x"] - du["xl"] * dz["x"]) / sl["x"], "xh": FH * (rh + du["xh"] * dz["x"]) / sh}
            for k in low_vars:
                ddu[k] = (rl[k] - du[k] * dz[k]) / sl[k]
            return dz, dlam, ddu

        def step(dz, ddu):
            inf = float("inf")

            def ratio(s, d, mask=None):
                r = torch.where(d < 0, -s / d, torch.full_like(d, inf))
                if mask is not None:
                    r = torch.where(mask > 0, r, torch.full_like(r, inf))
                return r.amin(1) if r.dim() == 2 and r.shape[1] else (r if r.dim() == 1 else torch.full((B,), inf,
                                                                                                   dtype=F64, device=dev))
            a = torch.minimum(ratio(sl["x"], dz["x"], FL), ratio(sh, -dz["x"], FH))
            for k in low_vars:
                if k == "st" and not budget:
                    continue
                a = torch.minimum(a, ratio(sl[k], dz[k]))
            for k, v in ddu.items():
                if k == "st" and not budget:
                    continue
                base = du[k]
                a = torch.minimum(a, ratio(base, v, FL if k == "xl" else FH if k == "xh" else None))
            return a.clamp(max=1.0)

        rl0 = {"x": -sl["x"] * du["xl"] * FL}
        for k in low_vars:
            rl0[k] = -sl[k] * du[k]
        rh0 = -sh * du["xh"] * FH
        dz, dlam, ddu = direction(rl0, rh0)
        a = step(dz, ddu)
        # Mehrotra centring
        aff = ((sl["x"] + a[:, None] * dz["x"]) * (du["xl"] + a[:, None] * ddu["xl"]) * FL).sum(1) \
            + ((sh - a[:, None] * dz["x"]) * (du["xh"] + a[:, None] * ddu["xh"]) * FH).sum(1)
        for k in low_vars:
            if k == "st" and not budget:
                continue
            ak = a[:, None] if sl[k].dim() == 2 else a
            g_k = (sl[k] + ak * dz[k]) * (du[k] + ak * ddu[k])
            aff = aff + (g_k.sum(1) if g_k.dim() == 2 else g_k)
        sig = ((aff / ncomp) / mu.clamp(min=1e-300)).clamp(0, 1) ** 3
        smu = sig * mu
        rl = {"x": FL * (smu[:, None] - sl["x"] * du["xl"] - dz["x"] * ddu["xl"])}
        for k in low_vars:
            sm = smu[:, None] if sl[k].dim() == 2 else smu
            rl[k] = sm - sl[k] * du[k] - dz[k] * ddu[k]
        if not budget:
            rl["st"] = zeros(B)
        rh = FH * (smu[:, None] - sh * du["xh"] + dz["x"] * ddu["xh"])
        dz, dlam, ddu = direction(rl, rh)
        a = 0.995 * step(dz, ddu)

        def upd(d, dd):
            for k in dd:
                if d[k].numel() == 0:
                    continue
                ak = a.view(-1, *([1] * (d[k].dim() - 1)))
                m = act.view(-1, *([1] * (d[k].dim() - 1)))
                d[k] = torch.where(m, d[k] + ak * dd[k], d[k])
        upd(z, dz)
        upd(lam, dlam)
        upd(du, ddu)
        if not budget:
            z["st"] = zeros(B)
            du["st"] = zeros(B)
    status = torch.full_like(iters, _lib.PQ_MAX_ITER)
    status = torch.where(best_merit < _INACCURATE, torch.full_like(iters, _lib.PQ_SOLVED_INACCURATE), status)
    status = torch.where(best_merit < tol, torch.full_like(iters, _lib.PQ_SOLVED), status)
    Px = _gemv(UW, _gemv(UW, best_x), True) + pd[:, None] * best_x
    obj = 0.5 * (best_x * Px).sum(1) + (q * best_x).sum(1) + c * (best_x - x0).abs().sum(1)
    return LPResult(best_x, lam["U"], status, iters, obj, best_merit)


def terms_from_model(constraints, params, universe) -> L1Terms | None:
    """The terms model_qpsolvers applies (src/optimization.py:125-142) when a turnover term
    and a leverage budget come together (l1split.term_from_model's "unsupported" case):
    transaction_cost not None -> the cost form (and, when it is 0 and a turnover constraint
    exists, the budget as well -- `not 0` is True); otherwise the turnover budget."""
    tocon = constraints.l1.get("turnover")
    levcon = constraints.l1.get("leverage")
    x0 = tocon["x0"] if tocon is not None and tocon.get("x0") is not None else params.get("x0")
    if x0 is None or levcon is None:
        return None
    x_init = np.array([x0.get(a, 0) for a in universe], dtype=np.float64)
    tc = params.get("transaction_cost")
    cost = float(tc) if tc is not None else 0.0
    budget = float(tocon["rhs"]) if (tocon and not tc) else None
    if tc is None and budget is None:
        return None
    return L1Terms(x0=x_init, cost=cost, to_budget=budget, lev_budget=float(levcon["rhs"]))


def window_rows(stage, scale, pdiag, Pm, n):
    """(UW, pd) with P_eff = UW'UW + diag(pd) for the dates of a backtest chunk: the centred
    (or uncentred) window rows scaled by sqrt(p_scale w_scale) on the window path, or the
    eigen-square-root of the dense P (rocSOLVER syevd) when T >= n."""
    B = stage.batch
    dev = stage.device
    lr = stage.lowrank
    scale = torch.ones(B, dtype=F64, device=dev) if scale is None else scale
    pd = torch.zeros(B, dtype=F64, device=dev) if pdiag is None else pdiag
    if lr is not None:
        rows = lr.rows.to(torch.int64)
        Tm = rows.shape[1]
        X = lr.panel.R[rows.clamp(min=0)][:, :, :n]
        if lr.mu is not None:
            X = X - lr.mu[:, None, :n]
        mask = torch.arange(Tm, device=dev)[None, :] < lr.tlen.to(torch.int64)[:, None]
        s = scale * (lr.w_scale if lr.w_scale is not None else 1.0)
        UW = (X * mask[:, :, None]) * s.clamp(min=0).sqrt()[:, None, None]
        return UW.contiguous(), pd
    P = Pm[:, :n, :n]
    P = torch.tril(P) + torch.tril(P, -1).transpose(1, 2)
    ev, V = torch.linalg.eigh(scale[:, None, None] * P)
    UW = (V * ev.clamp(min=0).sqrt()[:, None, :]).transpose(1, 2)
    return UW.contiguous(), pd
