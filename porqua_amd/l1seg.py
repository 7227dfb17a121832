"""Turnover and leverage together as a segment split on the ADMM
engine, instead of the reference's 3n + 2 linearised variables and 4n + 2 rows.

The reference linearises a turnover term around x0 (cost c 1'd or budget 1'd <= tau, d >=
|x - x0|) and a leverage budget 1'|x| <= L with auxiliary variables and rows
(``linearize_turnover_*`` / ``linearize_leverage_constraint``, src/qp_problems.py:40-157,
driven from ``model_qpsolvers``, src/optimization.py:125-142).  Both |x_i - x0_i| and |x_i|
are piecewise linear in x_i with breakpoints {0, x0_i}, so with a_i = min(0, x0_i),
b_i = max(0, x0_i) and lb_i <= a_i, b_i <= ub_i, asset i's range splits into three segments

    x_i = lb_i + s1_i + s2_i + s3_i,   0 <= s1_i <= a_i - lb_i,  0 <= s2_i <= b_i - a_i,
                                       0 <= s3_i <= ub_i - b_i,

on which both functions are linear: |x_i - x0_i| = |lb_i - x0_i| + t_i's, |x_i| = |lb_i| +
l_i's with slopes -1 on s1, +-1 on s2 (the sign of x0_i) and +1 on s3.  For any x the
in-order filling (earlier segments full before a later one grows) reproduces both
functions exactly, and any other filling of the same x gives a LARGER value (the slopes
increase along the segments: convexity), so the problem in s

    min 0.5 s' S'P S s + (S'(P lb + q) + c t)' s
    s.t.  A S s = b - A lb,  G S s <= h - G lb,  t's <= tau - 1'|lb - x0|,  l's <= L - 1'|lb|,
          segment boxes

has the reference problem's optimal x (x = lb + S s) and optimal value.  Three n-blocks of
variables, two more general rows, box bounds -- the engine's window path takes it over the
panel [R, R, R] (S'P S = c (Xc S)'(Xc S), Xc S = [Xc, Xc, Xc]).  A ridge p_diag I of P
(linear shrinkage, l2 penalty) becomes p_diag S'S, which is not diagonal: those problems keep
the per-asset-block IPM (porqua_amd/ipm_l1.py).
"""
from __future__ import annotations

import numpy as np


def segment_data(x0, lb, ub, cost=0.0, to_budget=None, lev_budget=np.inf):
    """Host data of the split: segment boxes (3n), turnover / leverage slopes (3n each), the
    constants 1'|lb - x0| and 1'|lb|; None when the box does not contain 0 and x0."""
    x0 = np.asarray(x0, dtype=np.float64).reshape(-1)
    lb = np.asarray(lb, dtype=np.float64).reshape(-1)
    ub = np.asarray(ub, dtype=np.float64).reshape(-1)
    a, b = np.minimum(0.0, x0), np.maximum(0.0, x0)
    tol = 1e-12 * (1.0 + np.abs(x0))
    if np.any(lb > a + tol) or np.any(ub < b - tol) or not np.all(np.isfinite(lb)) or not np.all(np.isfinite(ub)):
        return None
    lb = np.minimum(lb, a)
    ub = np.maximum(ub, b)
    pos = x0 > 0.0
    ones = np.ones_like(x0)
    return {"lo": np.zeros(3 * x0.size),
            "hi": np.concatenate([a - lb, b - a, ub - b]),
            # turnover slopes: below x0 -1, above +1; the middle segment [a, b] lies below x0
            # when x0 = b > 0, above it when x0 = a < 0
            "t": np.concatenate([-ones, np.where(pos, -1.0, 1.0), ones]),
            # leverage slopes: below 0 -1, above +1; the middle segment lies above 0 when x0 > 0
            "l": np.concatenate([-ones, np.where(pos, 1.0, -1.0), ones]),
            "t0": float(np.abs(lb - x0).sum()), "l0": float(np.abs(lb).sum()),
            "lb": lb, "cost": float(cost), "to_budget": to_budget, "lev_budget": float(lev_budget)}


def _rows(sd, n, A, b, G, h):
    """General rows of the split: [A A A] = b - A lb, [G G G] <= h - G lb, then the unit-norm
    turnover / leverage budget rows (skipped when infinite).  Returns (A3, b3, G3, h3)."""
    lb = sd["lb"]
    A3 = b3 = G3 = h3 = None
    if A is not None:
        A = np.asarray(A, dtype=np.float64).reshape(-1, n)
        A3 = np.hstack([A, A, A])
        b3 = np.asarray(b, dtype=np.float64).reshape(-1) - A @ lb
    rows, rhs = [], []
    if G is not None:
        G = np.asarray(G, dtype=np.float64).reshape(-1, n)
        rows.append(np.hstack([G, G, G]))
        rhs.append(np.asarray(h, dtype=np.float64).reshape(-1) - G @ lb)
    r = 1.0 / np.sqrt(3 * n)   # unit-norm rows (ADMM's rho is per row, like the unit box rows)
    if sd["to_budget"] is not None and np.isfinite(sd["to_budget"]):
        rows.append(sd["t"][None, :] * r)
        rhs.append(np.array([(sd["to_budget"] - sd["t0"]) * r]))
    if np.isfinite(sd["lev_budget"]):
        rows.append(sd["l"][None, :] * r)
        rhs.append(np.array([(sd["lev_budget"] - sd["l0"]) * r]))
    if rows:
        G3, h3 = np.vstack(rows), np.concatenate(rhs)
    return A3, b3, G3, h3


def segment_problem(base: dict, sd: dict) -> dict:
    """Dense split of one problem (P, q, A, b, G, h of the problem before the linearisation);
    returns P3, q3, A3, b3, G3, h3, lb3, ub3 and the objective constant."""
    P = np.asarray(base["P"], dtype=np.float64)
    q = np.asarray(base["q"], dtype=np.float64).reshape(-1)
    n = q.size
    lb = sd["lb"]
    S = np.hstack([np.eye(n)] * 3)
    g = P @ lb + q
    q3 = S.T @ g + sd["cost"] * sd["t"]
    A3, b3, G3, h3 = _rows(sd, n, base.get("A"), base.get("b"), base.get("G"), base.get("h"))
    return {"P": S.T @ P @ S, "q": q3, "A": A3, "b": b3, "G": G3, "h": h3, "lb": sd["lo"], "ub": sd["hi"],
            "constant": 0.5 * float(lb @ P @ lb) + float(q @ lb) + sd["cost"] * sd["t0"]}


def merge(s, n: int, lb) -> np.ndarray:
    """x = lb + s1 + s2 + s3."""
    s = np.asarray(s, dtype=np.float64)
    return np.asarray(lb, dtype=np.float64) + s[:n] + s[n:2 * n] + s[2 * n:3 * n]


def segment_batch(qb, lowrank, sd: dict, seg_panel, A, b, G, h):
    """Device form of segment_problem for a batch of dates sharing the constraints (the
    batched backtest) on the window path: ``qb`` / ``lowrank`` hold the original problems
    (P_eff = p_scale w_scale Xc'Xc, p_diag zero -- the caller checks), ``seg_panel`` is the
    panel [R, R, R].  Returns (qb3, lowrank3, const[B])."""
    import torch
    from . import engine
    F64 = torch.float64
    B, n, dev = qb.batch, qb.n, qb.device
    lb = torch.as_tensor(sd["lb"], dtype=F64, device=dev)
    ps = qb.p_scale if qb.p_scale is not None else torch.ones(B, dtype=F64, device=dev)
    q = qb.q[:, :n]
    R = lowrank.panel.R
    rows = lowrank.rows.to(torch.int64)
    T = rows.shape[1]
    mask = torch.arange(T, device=dev)[None, :] < lowrank.tlen.to(torch.int64)[:, None]
    # P lb through the window: u = Xc lb per date, P lb = c Xc' u (one scatter + panel GEMM)
    u = torch.where(mask, (R @ lb)[rows.clamp(min=0)], torch.zeros((), dtype=F64, device=dev))
    if lowrank.mu is not None:
        u = torch.where(mask, u - (lowrank.mu[:, :n] @ lb)[:, None], torch.zeros((), dtype=F64, device=dev))
    xtu = torch.empty((B, n), dtype=F64, device=dev)
    ch = max(1, int(2e8 // (8 * R.shape[0])))
    for s in range(0, B, ch):
        e = min(B, s + ch)
        Sm = torch.zeros((e - s, R.shape[0]), dtype=F64, device=dev)
        Sm.scatter_add_(1, rows[s:e].clamp(min=0), u[s:e])
        xtu[s:e] = Sm @ R
    if lowrank.mu is not None:
        xtu -= lowrank.mu[:, :n] * u.sum(1)[:, None]
    wsc = lowrank.w_scale if lowrank.w_scale is not None else torch.ones(B, dtype=F64, device=dev)
    plb = (ps * wsc)[:, None] * xtu
    g = plb + q
    const = 0.5 * ps * wsc * (u * u).sum(1) + q @ lb + sd["cost"] * sd["t0"]
    A3, b3, G3, h3 = _rows(sd, n, A, b, G, h)
    qb3 = engine.QPBatch.from_dense(None, None, n=3 * n, A=A3, b=b3, G=G3, h=h3, lb=sd["lo"], ub=sd["hi"],
                                    device=dev)
    qb3.batch = B
    q3 = torch.zeros((B, qb3.ld), dtype=F64, device=dev)
    tc = torch.as_tensor(sd["t"] * sd["cost"], dtype=F64, device=dev)
    for k in range(3):
        q3[:, k * n:(k + 1) * n] = g + tc[None, k * n:(k + 1) * n]
    qb3.q = q3
    qb3.P = None
    qb3.p_scale = ps
    qb3.p_diag = None
    mu3 = None if lowrank.mu is None else torch.cat([lowrank.mu[:, :n]] * 3, 1).contiguous()
    lr3 = engine.LowRank(seg_panel, lowrank.rows, lowrank.tlen, mu=mu3, w_scale=lowrank.w_scale)
    return qb3, lr3, const


def merge_batch(x3, n: int, lb):
    """x = lb + s1 + s2 + s3 for every date (x3: B x >= 3n device tensor)."""
    import torch
    lbt = torch.as_tensor(lb, dtype=x3.dtype, device=x3.device)
    return lbt[None, :] + x3[:, :n] + x3[:, n:2 * n] + x3[:, 2 * n:3 * n]
