# Host-side API restatement of PorQua (part of the GeomScale project; reference tree
# amolrpatil21/PorQua): src/qp_problems.py.  PorQua is Copyright (c) 2024 Cyril Bachelard and
# Minh Ha Ho and licensed under the GNU LGPL v3; this module keeps that API and its
# behaviour (quirks included) so that the MI355X engine is a drop-in, and is distributed
# under the same licence terms.
"""QuadraticProgram -- drop-in for src/qp_problems.py with the MI355X engine behind a new
``solver_name``.

The reference dispatches every QP to the third-party ``qpsolvers.solve_problem``
(src/qp_problems.py:184-216).  Here ``solver_name='mi355x'`` routes it to the batched HIP
engine (``porqua_amd.engine``); the problem data, the ``solution`` record and
``objective_value`` keep the reference's meaning.  Any other solver name is handed to
``qpsolvers`` exactly as the reference does (ImportError when it is not installed) -- the
engine itself never falls back to a CPU solver.
"""
from __future__ import annotations

import pickle

import numpy as np

from .solution import Solution

ENGINE_SOLVER = "mi355x"
ENGINE_SOLVERS = {ENGINE_SOLVER}

# reference solver sets (src/qp_problems.py:19-30), extended by the dense device engine
IGNORED_SOLVERS = {"gurobi", "mosek", "ecos", "scs", "piqp", "proxqp", "clarabel"}
SPARSE_SOLVERS = {"clarabel", "ecos", "gurobi", "mosek", "highs", "qpalm", "osqp", "qpswift", "scs"}
ALL_SOLVERS = {"clarabel", "cvxopt", "daqp", "ecos", "gurobi", "highs", "mosek", "osqp", "piqp",
               "proxqp", "qpalm", "quadprog", "scs"} | ENGINE_SOLVERS
USABLE_SOLVERS = ALL_SOLVERS - IGNORED_SOLVERS


def _arr(v):
    return None if v is None else np.asarray(v, dtype=np.float64)


class QuadraticProgram(dict):
    """min 0.5 x'Px + q'x (+ constant)  s.t.  Gx <= h, Ax = b, lb <= x <= ub."""

    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self.solver = self["params"]["solver_name"]
        self._l1 = None         # recorded l1 term (l1split.L1Split) + the problem before it

    def _record_l1(self, kind, x0, value, layout="d"):
        """Keep the problem as it was before the (first) l1 linearisation: the engine solves
        the signed split of it (porqua_amd/l1split.py) instead of the 2n linearised rows."""
        from .l1split import L1Split
        if self._l1 is None:
            base = {k: self.get(k) for k in ("P", "q", "G", "h", "A", "b", "lb", "ub")}
            self._l1 = (L1Split(kind, x0, value, layout), base)
        else:
            self._l1 = "unsupported"   # several l1 terms: solved in the linearised form

    # -- l1 linearisations (src/qp_problems.py:40-157): auxiliary variables d >= |x - x0| ----
    def linearize_turnover_constraint(self, x_init, to_budget=float("inf")) -> None:
        """Turnover budget sum|x - x0| <= to_budget via d: [x; d], x - d <= x0, -x - d <= -x0."""
        x0 = np.asarray(x_init, dtype=np.float64).reshape(-1)
        self._record_l1("budget", x0, to_budget)
        n = len(self["q"])
        eye = np.eye(n)
        rows = [np.hstack([eye, -eye]), np.hstack([-eye, -eye]),
                np.concatenate([np.zeros(n), np.ones(n)])[None, :]]
        rhs = [x0, -x0, np.array([to_budget], dtype=np.float64)]
        self._extend_aux(n, rows, rhs, q_aux=np.zeros(n))

    def linearize_turnover_objective(self, x_init, transaction_cost=0.002) -> None:
        """Proportional cost transaction_cost * sum|x - x0| in the objective via d."""
        x0 = np.asarray(x_init, dtype=np.float64).reshape(-1)
        self._record_l1("cost", x0, transaction_cost)
        n = len(self["q"])
        eye = np.eye(n)
        rows = [np.hstack([eye, -eye]), np.hstack([-eye, -eye])]
        self._extend_aux(n, rows, [x0, -x0], q_aux=np.full(n, float(transaction_cost)))

    def linearize_leverage_constraint(self, N=None, leverage_budget=2) -> None:
        """sum|x| <= leverage_budget via x = x+ - x-, x+, x- >= 0 (src/qp_problems.py:79-118)."""
        n = len(self["q"])
        N = n if N is None else int(N)
        if N == n:
            self._record_l1("budget", np.zeros(n), leverage_budget, layout="pm")
        else:
            self._l1 = "unsupported"
        P = self.get("P")
        if P is not None:
            P = np.pad(P, (0, 2 * N))
        q = np.pad(self["q"], (0, 2 * N))
        G_old = self.get("G")
        mG = 0 if G_old is None else G_old.shape[0]
        G = np.zeros((mG + 1, n + 2 * N))
        if G_old is not None:
            G[:mG, :n] = G_old
        G[mG, n:] = 1.0
        h_old = self.get("h")
        h = np.append(np.empty(0) if h_old is None else h_old, leverage_budget)
        A_old = self.get("A")
        A_old = A_old.reshape(-1, n) if A_old is not None else np.zeros((0, n))
        mA = A_old.shape[0]
        A = np.zeros((mA + N, n + 2 * N))
        A[:mA, :n] = A_old
        A[mA:, :N] = np.eye(N)
        A[mA:, n:n + N] = np.eye(N)
        A[mA:, n + N:] = -np.eye(N)
        b_old = self.get("b")
        b = np.concatenate([np.asarray(b_old, dtype=np.float64).reshape(-1) if b_old is not None else np.empty(0),
                            np.zeros(N)])
        lb = np.pad(self["lb"], (0, 2 * N)) if self.get("lb") is not None else None
        ub = np.pad(self["ub"], (0, 2 * N), constant_values=np.inf) if self.get("ub") is not None else None
        self.update({"P": P, "q": q, "G": G, "h": h, "A": A, "b": b, "lb": lb, "ub": ub})

    def _extend_aux(self, n, g_rows, h_parts, q_aux):
        P = self.get("P")
        if P is not None:
            P = np.pad(P, (0, n))
        q = np.concatenate([self["q"], q_aux])
        G_old = self.get("G")
        blocks = []
        if G_old is not None:
            blocks.append(np.hstack([G_old, np.zeros((G_old.shape[0], n))]))
        G = np.vstack(blocks + g_rows)
        h_old = self.get("h")
        h = np.concatenate(([] if h_old is None else [np.asarray(h_old, dtype=np.float64).reshape(-1)]) + h_parts)
        A = self.get("A")
        if A is not None:
            A = np.pad(A.reshape(-1, A.shape[-1]), [(0, 0), (0, n)])
        lb = np.pad(self["lb"], (0, n)) if self.get("lb") is not None else None
        ub = np.pad(self["ub"], (0, n), constant_values=np.inf) if self.get("ub") is not None else None
        self.update({"P": P, "q": q, "G": G, "h": h, "A": A, "lb": lb, "ub": ub})

    # -- solving ------------------------------------------------------------------------
    def is_feasible(self) -> bool:
        """Feasibility of the constraint set (a zero objective, src/qp_problems.py:159-182)."""
        P = self.get("P")
        n = len(self["q"])
        probe = QuadraticProgram(P=np.zeros((n, n)) if P is None else np.zeros_like(P), q=np.zeros(n),
                                 G=self.get("G"), h=self.get("h"), A=self.get("A"), b=self.get("b"),
                                 lb=self.get("lb"), ub=self.get("ub"), params=self["params"])
        probe.solve()
        return bool(probe["solution"].found)

    def solve(self) -> None:
        if self.solver in ENGINE_SOLVERS:
            if isinstance(self._l1, tuple):
                self["solution"] = self._solve_l1_split()
            else:
                self["solution"] = solve_batch([self])[0]
            return None
        return self._solve_qpsolvers()

    def _solve_l1_split(self):
        """The engine solve of a problem with one turnover term: the signed split
        (l1split.split_problem), mapped back to the reference's [x; d] variables and
        objective (0.5 x'Px + q'x + c 1'd, src/qp_problems.py:219-221)."""
        from .l1split import merge_solution, split_problem
        term, base = self._l1
        sp = split_problem(base, term)
        sub = {k: sp[k] for k in ("P", "q", "G", "h", "A", "b", "lb", "ub")}
        sub["params"] = self["params"]
        from . import engine
        from .l1split import split_settings
        sol = solve_batch([sub], settings=split_settings(engine.Settings.from_params(self["params"]),
                                                         self["params"], term.kind))[0]
        if sol.x is not None:
            x, aux = merge_solution(sol.x, term)
            sol.x = np.concatenate([x, aux])
            if sol.found:
                sol.obj = self.objective_value(sol.x, with_const=False)
        sol.z = None      # multipliers of the split rows, not of the 2n linearised rows
        sol.z_box = None
        sol.extras = dict(sol.extras or {}, l1_split=term.kind)
        return sol

    def _solve_qpsolvers(self) -> None:
        """Non-engine solver names keep the reference behaviour (third-party qpsolvers)."""
        import qpsolvers  # noqa: F401  (ImportError when absent, as in the reference)
        import scipy.sparse as sp
        from .helper_functions import isPD, nearestPD
        if self.solver in ("ecos", "scs", "clarabel") and self.get("b") is not None and np.size(self["b"]) == 1:
            self["b"] = np.asarray(self["b"]).reshape(-1)
        P = self.get("P")
        if P is not None and not isPD(P):
            self["P"] = nearestPD(P)
        problem = qpsolvers.Problem(P=self.get("P"), q=self.get("q"), G=self.get("G"), h=self.get("h"),
                                    A=self.get("A"), b=self.get("b"), lb=self.get("lb"), ub=self.get("ub"))
        if self.solver in SPARSE_SOLVERS and self["params"].get("sparse"):
            for f in ("P", "A", "G"):
                if getattr(problem, f) is not None:
                    setattr(problem, f, sp.csc_matrix(getattr(problem, f)))
        self["solution"] = qpsolvers.solve_problem(problem=problem, solver=self.solver,
                                                   initvals=self.get("x0"), verbose=False)
        return None

    def objective_value(self, x: np.ndarray, with_const: bool = True) -> float:
        """0.5 x'Px + q'x (+ constant), src/qp_problems.py:219-221."""
        const = self.get("constant")
        c = 0 if const is None or not with_const else const
        return float(0.5 * (x @ self.get("P") @ x) + self.get("q") @ x) + c

    def serialize(self, path, **kwargs):
        with open(path, "wb") as f:
            pickle.dump(self, f, **kwargs)

    @staticmethod
    def load(path, **kwargs):
        # NB: the reference passes the *path* to pickle.load (src/qp_problems.py:228-230); fixed.
        with open(path, "rb") as f:
            return pickle.load(f, **kwargs)


def solve_batch(qps, settings=None, device=None):
    """Solve a list of QuadraticPrograms of equal dimension on the device in one batch.

    Problems whose constraint matrices are identical share them on the device; the
    solutions are ``Solution`` objects with the qpsolvers fields the reference reads."""
    from . import engine
    if not qps:
        return []
    params = qps[0]["params"]
    settings = settings or engine.Settings.from_params(params)
    P = np.stack([_arr(qp["P"]) for qp in qps])
    n = P.shape[-1]
    q = np.stack([_arr(qp["q"]).reshape(-1) for qp in qps])

    def stack_opt(key, reshape=None):
        vals = [qp.get(key) for qp in qps]
        if all(v is None for v in vals):
            return None
        if any(v is None for v in vals):
            raise ValueError(f"solve_batch: '{key}' present in some problems only")
        arrs = [_arr(v) if reshape is None else _arr(v).reshape(reshape) for v in vals]
        if all(np.array_equal(arrs[0], a) for a in arrs[1:]):
            return arrs[0]
        return np.stack(arrs)

    A = stack_opt("A", (-1, n))
    b = stack_opt("b", (-1,))
    G = stack_opt("G", (-1, n))
    h = stack_opt("h", (-1,))
    lb = stack_opt("lb", (n,))
    ub = stack_opt("ub", (n,))
    if A is not None and A.ndim == 3 and b is not None and b.ndim == 1:
        b = np.broadcast_to(b, (len(qps), b.size)).copy()
    if G is not None and G.ndim == 3 and h is not None and h.ndim == 1:
        h = np.broadcast_to(h, (len(qps), h.size)).copy()
    me = 0 if A is None else A.shape[-2]
    mi = 0 if G is None else G.shape[-2]
    if me + mi > IPM_ROWS or n > DENSE_ADMM_MAX_N:
        return _solve_batch_ipm(P, q, A, b, G, h, lb, ub, device)
    qb = engine.QPBatch.from_dense(P, q, A=A, b=b, G=G, h=h, lb=lb, ub=ub, device=device)
    res = engine.solve(qb, settings)
    return batch_result_to_solutions(res, qb)


IPM_ROWS = 64    # general rows the ADMM engine keeps in LDS; beyond: the device IPM
# the dense ADMM (K3) keeps its n-vectors in LDS up to 1024 assets; larger dense QPs (the
# per-QP drop-in at configs 4/5 sizes: QuadraticProgram.solve with a 3000 x 3000 or 5000 x
# 5000 P, src/qp_problems.py:184-216) go to the device IPM on K2L (pq_factor_large)
DENSE_ADMM_MAX_N = 1024


def _solve_batch_ipm(P, q, A, b, G, h, lb, ub, device=None):
    """More than IPM_ROWS general rows (e.g. the reference's linearised turnover + leverage
    rows together, src/qp_problems.py:40-118) or more than DENSE_ADMM_MAX_N assets:
    porqua_amd.ipm.qp_ipm_batched (Mehrotra predictor-corrector, the algorithm family of the
    reference's default cvxopt backend; normal matrices factored and inverted on K2, or on the
    multi-workgroup K2L beyond 1024 assets).  Problems with their own constraint matrices are
    solved one at a time."""
    import torch
    from . import _lib, engine
    from .ipm import qp_ipm_batched
    if ((A is not None and A.ndim == 3) or (G is not None and G.ndim == 3)
            or (lb is not None and np.ndim(lb) == 2) or (ub is not None and np.ndim(ub) == 2)):
        B = P.shape[0]
        out = []
        for i in range(B):
            pick = lambda v, nd: None if v is None else (v[i] if np.asarray(v).ndim == nd else v)
            out += _solve_batch_ipm(P[i:i + 1], q[i:i + 1], pick(A, 3), pick(b, 2), pick(G, 3), pick(h, 2),
                                    pick(lb, 2), pick(ub, 2), device)
        return out
    dev = device or engine.default_device()
    B, n = q.shape
    T = lambda v: None if v is None else torch.from_numpy(np.array(v, dtype=np.float64)).to(dev)
    def rows(v, m):
        v = np.asarray(v, dtype=np.float64)
        return np.broadcast_to(v.reshape(1, -1) if v.ndim < 2 else v, (B, m))

    bb = None if A is None else rows(b, A.shape[0])
    hh = None if G is None else rows(h, G.shape[0])
    Pd, qd, Ad, bd, Gd, hd, lbd, ubd = T(P), T(q), T(A), T(bb), T(G), T(hh), T(lb), T(ub)
    res = qp_ipm_batched(Pd, qd, Ad, bd, Gd, hd, lbd, ubd)
    # active-set polish of every answer (exact on the detected face when P_FF is PD)
    from .ipm import active_set_polish
    polished = np.zeros(B, dtype=bool)
    if res.z is None:
        res.z = torch.zeros((B, 0), dtype=torch.float64, device=dev)
    for i in range(B):
        if int(res.status[i]) not in (_lib.PQ_SOLVED, _lib.PQ_SOLVED_INACCURATE):
            continue
        xi, yi, zi, zbi, ok = active_set_polish(Pd[i], qd[i], Ad, None if bd is None else bd[i], Gd,
                                                None if hd is None else hd[i], lbd, ubd, res.x[i], -res.lam[i],
                                                res.z[i], res.z_box[i])
        if ok:
            polished[i] = True
            res.x[i], res.lam[i], res.z_box[i] = xi, -yi, zbi
            if Gd is not None:
                res.z[i] = zi
            res.status[i] = _lib.PQ_SOLVED
            Pxi = Pd[i] @ xi
            res.Px[i] = Pxi
            res.obj[i] = 0.5 * (xi @ Pxi) + qd[i] @ xi
    if Gd is None:
        res.z = None
    x = res.x.cpu().numpy()
    st = res.status.cpu().numpy()
    it = res.iters.cpu().numpy()
    obj = res.obj.cpu().numpy()
    merit = res.merit.cpu().numpy()
    ya = res.lam.cpu().numpy()
    zs = res.z.cpu().numpy() if res.z is not None else None
    zb = res.z_box.cpu().numpy()
    # qpsolvers' residuals of the returned point (src/helper_functions.py:69-80;
    # example/compare_solver.ipynb:212-216), from the device P x
    Px = res.Px.cpu().numpy()
    prim, dual, gap = _residuals(x, Px, q, A, bb, G, hh, lb, ub, -ya if A is not None else None, zs, zb)
    sols = []
    for i in range(B):
        s = Solution(x=x[i].copy(), status=int(st[i]), iterations=int(it[i]))
        s.found = int(st[i]) in (_lib.PQ_SOLVED, _lib.PQ_SOLVED_INACCURATE)
        s.y = -ya[i].copy() if A is not None else None      # qpsolvers sign: Px + q + A'y + ... = 0
        s.z = zs[i].copy() if zs is not None else None
        s.z_box = zb[i].copy() if (lb is not None or ub is not None) else None
        s.obj = float(obj[i]) if s.found else None
        s._prim, s._dual, s._gap = float(prim[i]), float(dual[i]), float(gap[i])
        s.extras = {"solver": "device IPM" + (" (K2L, n > 1024)" if n > DENSE_ADMM_MAX_N else
                                             " (more than 64 general rows)"), "merit": float(merit[i]),
                    "active_set_polish": bool(polished[i])}
        if not s.found:
            s.x = None
        sols.append(s)
    return sols


def _residuals(x, Px, q, A, b, G, h, lb, ub, y, z, zb):
    """Per problem: primal residual max(|Ax - b|, [Gx - h]+, [lb - x]+, [x - ub]+), dual
    residual |Px + q + A'y + G'z + z_box|inf and duality gap |x'Px + q'x + b'y + h'z +
    lb'min(z_box, 0) + ub'max(z_box, 0)| (qpsolvers Solution semantics)."""
    B = x.shape[0]
    prim = np.zeros(B)
    g = Px + q
    gap = (x * Px).sum(1) + (q * x).sum(1)
    if A is not None:
        prim = np.maximum(prim, np.abs(x @ A.T - b).max(1))
        g = g + y @ A
        gap = gap + (b * y).sum(1)
    if G is not None:
        prim = np.maximum(prim, np.maximum(x @ G.T - h, 0.0).max(1))
        g = g + z @ G
        gap = gap + (h * z).sum(1)
    if lb is not None:
        lo = np.broadcast_to(lb, x.shape)
        prim = np.maximum(prim, np.maximum(lo - x, 0.0).max(1))
        gap = gap + (np.where(np.isfinite(lo), lo, 0.0) * np.minimum(zb, 0.0)).sum(1)
    if ub is not None:
        up = np.broadcast_to(ub, x.shape)
        prim = np.maximum(prim, np.maximum(x - up, 0.0).max(1))
        gap = gap + (np.where(np.isfinite(up), up, 0.0) * np.maximum(zb, 0.0)).sum(1)
    if lb is not None or ub is not None:
        g = g + zb
    return prim, np.abs(g).max(1), np.abs(gap)


def batch_result_to_solutions(res, qb):
    """Device BatchResult -> list of Solution (one host copy of each array)."""
    from . import _lib
    x = res.x.cpu().numpy()
    y = res.y.cpu().numpy()
    zb = res.z_box.cpu().numpy() if qb.has_box else None
    st = res.status.cpu().numpy()
    it = res.iters.cpu().numpy()
    out = res.out.cpu().numpy()
    me = getattr(qb, "me", qb.mg)
    sols = []
    for i in range(x.shape[0]):
        s = Solution(x=x[i].copy(), status=int(st[i]), iterations=int(it[i]))
        s.found = int(st[i]) in (_lib.PQ_SOLVED, _lib.PQ_SOLVED_INACCURATE)
        s.y = y[i, :me].copy() if me else None
        s.z = y[i, me:qb.mg].copy() if qb.mg > me else None
        s.z_box = zb[i].copy() if zb is not None else None
        s.obj = float(out[i, _lib.PQ_OUT_OBJ]) if s.found else None
        s._prim = float(out[i, _lib.PQ_OUT_PRIM])
        s._dual = float(out[i, _lib.PQ_OUT_DUAL])
        s._gap = float(out[i, _lib.PQ_OUT_GAP])
        s.extras = {"rho": float(out[i, _lib.PQ_OUT_RHO]), "n_free": int(out[i, _lib.PQ_OUT_NFREE]),
                    "polish_rounds": int(out[i, _lib.PQ_OUT_ROUNDS])}
        if not s.found:
            s.x = None if int(st[i]) == _lib.PQ_NON_CONVEX else s.x
        sols.append(s)
    return sols
