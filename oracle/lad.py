"""LAD oracle -- TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

* ``lad_lp`` restates the reference's LP construction of ``LAD.set_objective`` /
  ``LAD.model_qpsolvers`` (src/optimization.py:271-345): levels log((1 + X).cumprod()) when
  use_level / use_log, variables [w; u; v], rows [A; X I -I] = [b; y], G padded with zeros,
  lb / ub padded with 0 / inf, q = [0; 1; 1], P = 0.
* ``solve_lp`` solves it with scipy's HiGHS (dual simplex / IPM with crossover) at tight
  tolerances.  The reference hands the LP to the third-party qpsolvers (absent here, see
  oracle/__init__.py); an LP's optimal value is unique, so the parity tests compare values
  and feasibility, and weights only where the optimum is unique.
"""
from __future__ import annotations

import numpy as np
from scipy.optimize import linprog


def levels(X, use_level=True, use_log=True):
    """src/optimization.py:276-282."""
    X = np.asarray(X, dtype=np.float64)
    if use_level:
        X = np.cumprod(1 + X, axis=0)
        if use_log:
            X = np.log(X)
    return X


def lad_lp(X, y, A=None, b=None, G=None, h=None, lb=None, ub=None):
    """src/optimization.py:296-336 (the leverage branch, :325-343, raises in the reference)."""
    X = np.asarray(X, dtype=np.float64)
    y = np.asarray(y, dtype=np.float64).reshape(-1)
    T, N = X.shape
    meq = 0 if A is None else (1 if np.ndim(A) == 1 else np.shape(A)[0])
    A_t = np.zeros((T, N + 2 * T)) if A is None else np.pad(np.atleast_2d(A), [(0, T), (0, 2 * T)])
    A_t[meq:T + meq, :N] = X
    A_t[meq:T + meq, N:N + T] = np.eye(T)
    A_t[meq:T + meq, N + T:] = -np.eye(T)
    b_t = y if b is None else np.append(b, y)
    G_t = None if G is None else np.pad(np.atleast_2d(G), [(0, 0), (0, 2 * T)])
    lb_t = np.pad(np.full(N, -np.inf) if lb is None else np.asarray(lb, dtype=np.float64), (0, 2 * T))
    ub_t = np.pad(np.full(N, np.inf) if ub is None else np.asarray(ub, dtype=np.float64), (0, 2 * T),
                  constant_values=np.inf)
    q = np.append(np.zeros(N), np.ones(2 * T))
    return q, A_t, b_t, G_t, h, lb_t, ub_t


def solve_lp(q, A, b, lb, ub, G=None, h=None):
    bounds = [(None if not np.isfinite(lo) else lo, None if not np.isfinite(hi) else hi)
              for lo, hi in zip(lb, ub)]
    res = linprog(q, A_ub=G, b_ub=h, A_eq=A, b_eq=b, bounds=bounds, method="highs",
                  options={"primal_feasibility_tolerance": 1e-10, "dual_feasibility_tolerance": 1e-10})
    assert res.status == 0, res.message
    return res
