"""l1 terms of the QP as a signed split instead of the reference's
2n + 1 linearised rows.

The reference turns a turnover term around x0 into auxiliary variables d >= |x - x0| with
2n inequality rows (``linearize_turnover_objective`` / ``linearize_turnover_constraint``,
src/qp_problems.py:40-77, 120-157), which is far beyond the engine's 64 general rows once
n > 31.  Here the same problem is solved in the variables w = [u; v] with
x = x0 + u - v, u, v >= 0:

    min 0.5 w' [P -P; -P P] w + [g0 + c; -g0 + c]' w        g0 = P x0 + q
    s.t.  [A -A] w = b - A x0,   [G -G] w <= h - G x0,   (turnover)  1'u + 1'v <= tau,
          0 <= u <= ub - x0,   0 <= v <= x0 - lb

(c = transaction cost, 0 for the constraint form).  Every optimum of the reference's
problem maps to one of this problem with complementary u, v (|x - x0| = u + v), and back:
x = x0 + u - v, d = |x - x0|.  The l1 rows become box bounds plus at most one general row,
so the problem keeps the engine's dense / window structure (the window of [P -P; -P P] is
[Xc, -Xc]).  Requires a box with lb <= x0 <= ub, which the long-only and long-short boxes
of the builders give for any feasible x0.
"""
from __future__ import annotations

import numpy as np


class L1Split:
    """One recorded l1 term: kind 'cost' (transaction_cost * sum|x - x0| in the objective)
    or 'budget' (sum|x - x0| <= tau).  The leverage constraint sum|x| <= L is the budget
    form around x0 = 0.  ``layout`` is the reference's variable vector: 'd' = [x; d]
    (turnover, src/qp_problems.py:40-77, 120-157), 'pm' = [x; x+; x-] (leverage, :79-118)."""

    def __init__(self, kind: str, x0, value: float, layout: str = "d"):
        if kind not in ("cost", "budget"):
            raise ValueError("L1Split: kind must be 'cost' or 'budget'")
        if layout not in ("d", "pm"):
            raise ValueError("L1Split: layout must be 'd' or 'pm'")
        self.kind = kind
        self.x0 = np.asarray(x0, dtype=np.float64).reshape(-1)
        self.value = float(value)
        self.layout = layout


def split_problem(base: dict, term: L1Split) -> dict:
    """The split QP of ``base`` (P, q, G, h, A, b, lb, ub of the problem *before* the l1
    linearisation) and ``term``; returns the same keys plus the objective constant."""
    P = np.asarray(base["P"], dtype=np.float64)
    q = np.asarray(base["q"], dtype=np.float64).reshape(-1)
    n = q.size
    x0 = term.x0
    if x0.size != n:
        raise ValueError(f"l1 split: x0 has {x0.size} entries, the problem {n}")
    lb, ub = base.get("lb"), base.get("ub")
    if lb is None or ub is None:
        raise NotImplementedError("l1 split: needs box bounds (lb <= x0 <= ub)")
    lb = np.asarray(lb, dtype=np.float64).reshape(-1)
    ub = np.asarray(ub, dtype=np.float64).reshape(-1)
    scale = 1.0 + np.abs(x0)
    if np.any(x0 < lb - 1e-12 * scale) or np.any(x0 > ub + 1e-12 * scale):
        raise NotImplementedError("l1 split: x0 lies outside the box")
    g0 = P @ x0 + q
    c = term.value if term.kind == "cost" else 0.0
    out = {"P": np.block([[P, -P], [-P, P]]), "q": np.concatenate([g0 + c, -g0 + c]),
           "lb": np.zeros(2 * n),
           "ub": np.concatenate([np.maximum(ub - x0, 0.0), np.maximum(x0 - lb, 0.0)]),
           "constant": 0.5 * float(x0 @ P @ x0) + float(q @ x0)}
    A, b = base.get("A"), base.get("b")
    if A is not None:
        A = np.asarray(A, dtype=np.float64).reshape(-1, n)
        out["A"] = np.hstack([A, -A])
        out["b"] = np.asarray(b, dtype=np.float64).reshape(-1) - A @ x0
    else:
        out["A"] = out["b"] = None
    G, h = base.get("G"), base.get("h")
    rows, rhs = [], []
    if G is not None:
        G = np.asarray(G, dtype=np.float64).reshape(-1, n)
        rows.append(np.hstack([G, -G]))
        rhs.append(np.asarray(h, dtype=np.float64).reshape(-1) - G @ x0)
    if term.kind == "budget" and np.isfinite(term.value):
        # 1'u + 1'v <= tau, scaled to a unit-norm row (the same constraint; ADMM's rho for a
        # row of 2n ones would be off by sqrt(2n) against the unit box rows)
        r = 1.0 / np.sqrt(2 * n)
        rows.append(np.full((1, 2 * n), r))
        rhs.append(np.array([term.value * r]))
    out["G"] = np.vstack(rows) if rows else None
    out["h"] = np.concatenate(rhs) if rows else None
    return out


def merge_solution(w: np.ndarray, term: L1Split) -> tuple[np.ndarray, np.ndarray]:
    """(x, aux) of the reference's variable vector from the split solution w: aux = d =
    |x - x0| (layout 'd') or the reference's [x+; x-] blocks (layout 'pm'), ordered so that
    the linearised rows x + x+ - x- = 0 hold."""
    n = term.x0.size
    x = term.x0 + w[:n] - w[n:2 * n]
    if term.layout == "pm":
        # linearize_leverage_constraint writes x + x+ - x- = 0 (src/qp_problems.py:79-118),
        # i.e. x = x- - x+: its first auxiliary block holds the negative part
        return x, np.concatenate([np.maximum(-x, 0.0), np.maximum(x, 0.0)])
    return x, np.abs(x - term.x0)


# ADMM over-relaxation for the split problems: measured on config 3 with a transaction cost
# (tools/bench_l1.py) alpha 1.8 takes 26 iterations against 118 at OSQP's 1.6 (budget form:
# 177 vs 190), while the plain problems are fastest at 1.6 -- so only split solves use it,
# and only when the caller did not set alpha
SPLIT_ALPHA = 1.8
# initial rho of the budget (turnover / leverage constraint) splits, relative to mean diag P:
# measured on config 3 + turnover budget 0.5 (tools/bench_l1.py, profiles/r02h_bench_l1.log)
# 4 -> 168 mean / 1093 max ADMM iterations, 5.6k QPs/s; 16 -> 35 / 397, 12.9k; 32 -> 25 / 537,
# 9.6k (the grouped kernel runs each slide group to its slowest date, so the tail decides)
SPLIT_BUDGET_RHO0_REL = 16.0


def split_settings(settings, params, kind: str = "cost"):
    """Settings for a split solve: ``settings`` with alpha = SPLIT_ALPHA (and, for a budget
    term, rho0_rel = SPLIT_BUDGET_RHO0_REL) unless ``params`` sets them."""
    import dataclasses
    params = params or {}
    upd = {}
    if not any(k in params for k in ("alpha", "admm_alpha")):
        upd["alpha"] = SPLIT_ALPHA
    if kind == "budget" and not any(k in params for k in ("rho0_rel", "admm_rho0_rel")):
        upd["rho0_rel"] = SPLIT_BUDGET_RHO0_REL
    return dataclasses.replace(settings, **upd) if upd else settings


def term_from_model(constraints, params, universe):
    """The l1 term model_qpsolvers would linearise (src/optimization.py:125-142): None,
    an L1Split, or "unsupported" (leverage, which the split does not cover)."""
    term = None
    tocon = constraints.l1.get("turnover")
    x0 = tocon["x0"] if tocon is not None and tocon.get("x0") is not None else params.get("x0")
    if x0 is not None:
        x_init = np.array([x0.get(a, 0) for a in universe], dtype=np.float64)
        tc = params.get("transaction_cost")
        if tc is not None and tocon and not tc:
            # INTENTIONAL DIFFERENCE from the reference: with transaction_cost == 0 it applies
            # BOTH linearisations (tc is not None, and `not 0` is True,
            # src/optimization.py:131-137); the second one sizes its rows for the already
            # extended 2N variables (src/qp_problems.py:40-59), leaving G with m + 6N + 1 rows
            # against h with m + 4N + 1 entries, which qpsolvers rejects -- the reference has
            # no answer here.  The engine solves the intended problem: the turnover budget
            # with a zero cost (the budget form)
            term = L1Split("budget", x_init, tocon["rhs"])
        elif tc is not None:
            term = L1Split("cost", x_init, tc)
        elif tocon:
            term = L1Split("budget", x_init, tocon["rhs"])
    levcon = constraints.l1.get("leverage")
    if levcon is not None:
        if term is not None:
            return "unsupported"      # turnover and leverage together: linearised rows
        term = L1Split("budget", np.zeros(len(universe)), levcon["rhs"], layout="pm")
    return term


def split_batch(qb, lowrank, term: L1Split, split_panel, A, b, G, h, lb, ub):
    """Device form of split_problem for a batch of dates sharing the constraints (the
    batched backtest).  ``qb`` holds the original problems (dense P in qb.P when
    ``lowrank`` is None, else P_eff = p_scale w_scale Xc'Xc + p_diag I in window form);
    ``split_panel`` is the panel [R, -R].  Returns (qb2, lowrank2 or None, const[B]) with
    the original objective = split objective + const.

    Window form: [P -P; -P P] = p_scale w_scale [Xc, -Xc]'[Xc, -Xc] + p_diag [I -I; -I I];
    the p_diag block is replaced by p_diag I_2n, which only adds p_diag (u'u + v'v -
    (u - v)'(u - v)) = 2 p_diag u'v >= 0 -- zero at every complementary point, and every
    optimum is complementary (lowering u_i and v_i together keeps x and every constraint
    and lowers the objective), so the optimum is unchanged."""
    import torch
    from . import engine
    F64 = torch.float64
    B, n, dev = qb.batch, qb.n, qb.device
    x0 = torch.as_tensor(term.x0, dtype=F64, device=dev)
    ps = qb.p_scale if qb.p_scale is not None else torch.ones(B, dtype=F64, device=dev)
    pd = qb.p_diag if qb.p_diag is not None else torch.zeros(B, dtype=F64, device=dev)
    q = qb.q[:, :n]
    if lowrank is not None:
        R = lowrank.panel.R
        rows = lowrank.rows.to(torch.int64)
        T = rows.shape[1]
        mask = torch.arange(T, device=dev)[None, :] < lowrank.tlen.to(torch.int64)[:, None]
        u = torch.where(mask, (R @ x0)[rows.clamp(min=0)], torch.zeros((), dtype=F64, device=dev))
        if lowrank.mu is not None:
            u = torch.where(mask, u - (lowrank.mu[:, :n] @ x0)[:, None], torch.zeros((), dtype=F64, device=dev))
        xtu = torch.empty((B, n), dtype=F64, device=dev)
        ch = max(1, int(2e8 // (8 * R.shape[0])))        # S chunk <= 200 MB
        for s in range(0, B, ch):
            e = min(B, s + ch)
            S = torch.zeros((e - s, R.shape[0]), dtype=F64, device=dev)
            S.scatter_add_(1, rows[s:e].clamp(min=0), u[s:e])
            xtu[s:e] = S @ R
        if lowrank.mu is not None:
            xtu -= lowrank.mu[:, :n] * u.sum(1)[:, None]
        ws = lowrank.w_scale if lowrank.w_scale is not None else torch.ones(B, dtype=F64, device=dev)
        px0 = (ps * ws)[:, None] * xtu + pd[:, None] * x0[None, :]
        xpx = ps * ws * (u * u).sum(1) + pd * (x0 @ x0)
    else:
        P = ps[:, None, None] * qb.P[:, :n, :n] + pd[:, None, None] * torch.eye(n, dtype=F64, device=dev)
        px0 = P @ x0
        xpx = px0 @ x0
    g0 = px0 + q
    const = 0.5 * xpx + q @ x0
    base = dict(P=np.zeros((n, n)), q=np.zeros(n), A=A, b=b, G=G, h=h, lb=lb, ub=ub)
    sp = split_problem(base, term)
    qb2 = engine.QPBatch.from_dense(None, None, n=2 * n, A=sp["A"], b=sp["b"], G=sp["G"], h=sp["h"], lb=sp["lb"],
                                    ub=sp["ub"], device=dev)
    qb2.batch = B
    c = term.value if term.kind == "cost" else 0.0
    q2 = torch.zeros((B, qb2.ld), dtype=F64, device=dev)
    q2[:, :n] = g0 + c
    q2[:, n:2 * n] = -g0 + c
    qb2.q = q2
    lr2 = None
    if lowrank is not None:
        qb2.P = None
        qb2.p_scale = ps
        qb2.p_diag = pd
        mu2 = None if lowrank.mu is None else torch.cat([lowrank.mu[:, :n], -lowrank.mu[:, :n]], 1).contiguous()
        lr2 = engine.LowRank(split_panel, lowrank.rows, lowrank.tlen, mu=mu2, w_scale=lowrank.w_scale)
    else:
        P2 = torch.zeros((B, qb2.ld, qb2.ld), dtype=F64, device=dev)
        P2[:, :n, :n] = P
        P2[:, :n, n:2 * n] = -P
        P2[:, n:2 * n, :n] = -P
        P2[:, n:2 * n, n:2 * n] = P
        qb2.P = P2
        qb2.p_scale = qb2.p_diag = None
    return qb2, lr2, const


def merge_batch(x2, term: L1Split):
    """x = x0 + u - v for every date (x2: B x >= 2n device tensor)."""
    import torch
    n = term.x0.size
    x0 = torch.as_tensor(term.x0, dtype=x2.dtype, device=x2.device)
    return x0[None, :] + x2[:, :n] - x2[:, n:2 * n]
