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
    or 'budget' (sum|x - x0| <= tau)."""

    def __init__(self, kind: str, x0, value: float):
        if kind not in ("cost", "budget"):
            raise ValueError("L1Split: kind must be 'cost' or 'budget'")
        self.kind = kind
        self.x0 = np.asarray(x0, dtype=np.float64).reshape(-1)
        self.value = float(value)


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
        rows.append(np.ones((1, 2 * n)))
        rhs.append(np.array([term.value]))
    out["G"] = np.vstack(rows) if rows else None
    out["h"] = np.concatenate(rhs) if rows else None
    return out


def merge_solution(w: np.ndarray, term: L1Split) -> tuple[np.ndarray, np.ndarray]:
    """(x, d) of the reference's variable vector [x; d] from the split solution w."""
    n = term.x0.size
    x = term.x0 + w[:n] - w[n:2 * n]
    return x, np.abs(x - term.x0)
