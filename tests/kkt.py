"""KKT optimality certificate of a QP solution (test helper; no solver involved).

For the convex QP  min 0.5 x'Px + q'x  s.t. A x = b, G x <= h, lb <= x <= ub  a point x
with multipliers (y_eq, y_g >= 0, z_box: <= 0 at lb, >= 0 at ub) is optimal iff it is
feasible, stationary (P x + q + A'y_eq + G'y_g + z_box = 0) and complementary.  The
certificate is size-independent, so it checks the engine where the dense oracle IPM
(oracle/qp_ipm.py) is too slow (n = 5000).

All dual-side residuals are RELATIVE (OSQP's normalisation): divided by
max(||P x||inf, ||q||inf, ||A'y + G'y_g||inf, ||z_box||inf), the largest term of the
stationarity sum, so a 1e-7 bar means 1e-7 of the problem's own gradient scale whatever
the units of P and q (daily-return covariances are O(1e-4)).  The primal violation stays
absolute (the BASELINE.json bar: violation <= 1e-7)."""
import numpy as np


def kkt_residuals(P, q, x, A=None, b=None, G=None, h=None, lb=None, ub=None, y=None, z_box=None):
    """Returns dict(stat, prim, dual, comp), each relative to the problem scale."""
    n = len(x)
    me = 0 if A is None else np.atleast_2d(A).shape[0]
    y = np.zeros(0) if y is None else np.asarray(y)
    ye, yg = y[:me], y[me:]
    Px = P @ x
    aty = np.zeros(n)
    if me:
        aty = aty + np.atleast_2d(A).T @ ye
    if G is not None and len(yg):
        aty = aty + np.atleast_2d(G).T @ yg
    zb = np.zeros(n) if z_box is None else np.asarray(z_box)
    sc = max(float(np.abs(Px).max()), float(np.abs(q).max(initial=0.0)), float(np.abs(aty).max()),
             float(np.abs(zb).max()), np.finfo(float).tiny)
    stat = float(np.abs(Px + q + aty + zb).max()) / sc
    prim = 0.0
    if me:
        prim = max(prim, float(np.abs(np.atleast_2d(A) @ x - np.asarray(b).reshape(-1)).max()))
    if G is not None:
        prim = max(prim, float(np.maximum(np.atleast_2d(G) @ x - h, 0).max(initial=0.0)))
    if lb is not None:
        prim = max(prim, float(np.maximum(lb - x, 0).max()))
    if ub is not None:
        prim = max(prim, float(np.maximum(x - ub, 0).max()))
    dual = float(np.maximum(-yg, 0).max(initial=0.0)) / sc
    comp = 0.0
    if G is not None and len(yg):
        comp = max(comp, float(np.abs(yg * (np.atleast_2d(G) @ x - h)).max()) / sc)
    if lb is not None and ub is not None:
        lo_gap = x - lb
        up_gap = ub - x
        comp = max(comp, float(np.abs(np.minimum(zb, 0) * lo_gap).max()) / sc,
                   float(np.abs(np.maximum(zb, 0) * up_gap).max()) / sc)
    return {"stat": stat, "prim": prim, "dual": dual, "comp": comp}
