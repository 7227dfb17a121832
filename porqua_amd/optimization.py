# Host-side API restatement of PorQua (part of the GeomScale project; reference tree
# amolrpatil21/PorQua): src/optimization.py.  PorQua is Copyright (c) 2024 Cyril Bachelard and
# Minh Ha Ho and licensed under the GNU LGPL v3; this module keeps that API and its
# behaviour (quirks included) so that the MI355X engine is a drop-in, and is distributed
# under the same licence terms.
"""Optimization classes (mirror of the hot-path part of src/optimization.py:40-259).

Each class keeps the reference API (``set_objective(optimization_data)``, ``solve()``,
``model_qpsolvers()``, ``results``) and adds a batched objective builder used by the
batched backtest: ``objective_batch(stage)`` returns the device-resident P (as the K1
output plus a per-date scale / diagonal term), q and the constant for every date at once.

Deliberate differences from the reference ("Reference defects"):
* ``OptimizationParameter`` defaults ``solver_name`` to 'mi355x' (the engine of this
  package) and lets ``verbose=False`` stick (src/optimization.py:45-46).
* ``MeanVariance`` uses the mean estimator that is passed in; the reference stores the
  class instead of the instance (src/optimization.py:165).
LAD runs on the batched device IPM of porqua_amd/lad.py; PercentilePortfolios (ranking,
not the QP path) is not built.
"""
from __future__ import annotations

from abc import ABC, abstractmethod
from typing import Optional

import numpy as np
import pandas as pd

from . import qp_problems
from .constraints import Constraints
from .covariance import Covariance
from .helper_functions import to_numpy
from .mean_estimation import MeanEstimator
from .optimization_data import OptimizationData


class OptimizationParameter(dict):

    def __init__(self, **kwargs):
        super().__init__(**kwargs)
        self.__dict__ = self
        if not self.get("solver_name"):
            self["solver_name"] = qp_problems.ENGINE_SOLVER
        self.setdefault("verbose", True)
        self.setdefault("allow_suboptimal", False)


class Objective(dict):
    pass


def _device_gram(X, y=None):
    """(X'X, X'y, y'y) of one window on the device (K1 Gram mode + pq_gram_xy)."""
    from . import engine
    Xv = np.ascontiguousarray(to_numpy(X), dtype=np.float64)
    T, n = Xv.shape
    yv = None if y is None else np.ascontiguousarray(to_numpy(y), dtype=np.float64).reshape(-1)
    pan = engine.Panel(Xv, yv)
    rows, tlen = pan.rows_to_device(np.arange(T, dtype=np.int32)[None], np.array([T], dtype=np.int32))
    G = pan.cov(rows, tlen, mode=1)[0, :n, :n].cpu().numpy()
    if yv is None:
        return G, None, None
    xty, yty = pan.gram_xy(rows, tlen)
    return G, xty[0, :n].cpu().numpy(), float(yty[0].item())


class Optimization(ABC):

    def __init__(self, params: OptimizationParameter = None, constraints: Constraints = None, **kwargs):
        self.params = OptimizationParameter(**kwargs) if params is None else params
        self.objective = Objective()
        self.constraints = Constraints() if constraints is None else constraints
        self.model = None
        self.results = None

    @abstractmethod
    def set_objective(self, optimization_data: OptimizationData) -> None:
        raise NotImplementedError("Method 'set_objective' must be implemented in derived class.")

    def objective_batch(self, stage):
        """Batched objective for the device backtest; ``None`` = not batchable."""
        return None

    def solve(self) -> bool:
        """src/optimization.py:72-75 (subclasses in the reference only forward here)."""
        self.solve_qpsolvers()
        return self.results["status"]

    def solve_qpsolvers(self) -> None:
        self.model_qpsolvers()
        self.model.solve()
        universe = self.constraints.selection
        sol = self.model["solution"]
        w = sol.x[:len(universe)] if sol.found else [None] * len(universe)
        self.results = {"weights": pd.Series(w, index=universe).to_dict(), "status": sol.found}

    def model_qpsolvers(self) -> None:
        """Assemble the QuadraticProgram exactly as src/optimization.py:91-143."""
        if "P" not in self.objective:
            raise ValueError("Missing matrix 'P' in objective.")
        P = to_numpy(self.objective["P"])
        q = to_numpy(self.objective["q"]) if "q" in self.objective else np.zeros(len(self.constraints.selection))
        self.objective["P"], self.objective["q"] = P, q
        universe = self.constraints.selection
        GhAb = self.constraints.to_GhAb()
        boxed = self.constraints.box["box_type"] != "NA"
        lb = self.constraints.box["lower"].to_numpy() if boxed else None
        ub = self.constraints.box["upper"].to_numpy() if boxed else None
        self.model = qp_problems.QuadraticProgram(P=P, q=q, constant=self.objective.get("constant"),
                                                  G=GhAb["G"], h=GhAb["h"], A=GhAb["A"], b=GhAb["b"],
                                                  lb=lb, ub=ub, params=self.params)
        tocon = self.constraints.l1.get("turnover")
        x0 = tocon["x0"] if tocon is not None and tocon.get("x0") is not None else self.params.get("x0")
        x_init = {a: x0.get(a, 0) for a in universe} if x0 is not None else None
        tc = self.params.get("transaction_cost")
        if tc is not None and x_init is not None:
            self.model.linearize_turnover_objective(pd.Series(x_init), tc)
        if tocon and not tc and x_init is not None:
            self.model.linearize_turnover_constraint(pd.Series(x_init), tocon["rhs"])
        levcon = self.constraints.l1.get("leverage")
        if levcon is not None:
            self.model.linearize_leverage_constraint(N=len(universe), leverage_budget=levcon["rhs"])


class EmptyOptimization(Optimization):

    def set_objective(self, optimization_data=None) -> None:
        pass

    def solve(self) -> bool:
        return super().solve()


class MeanVariance(Optimization):
    """P = 2 * risk_aversion * Sigma, q = -mu_geometric (src/optimization.py:157-177)."""

    batch_handles_nan = True   # windows with gaps: pairwise covariance + skipna means, batched

    def __init__(self, covariance: Optional[Covariance] = None,
                 mean_estimator: Optional[MeanEstimator] = None, **kwargs):
        super().__init__(**kwargs)
        self.covariance = Covariance() if covariance is None else covariance
        self.mean_estimator = MeanEstimator() if mean_estimator is None else mean_estimator
        self.params.setdefault("risk_aversion", 1)

    def set_objective(self, optimization_data: OptimizationData) -> None:
        X = optimization_data["return_series"]
        covmat = self.covariance.estimate(X=X) * self.params["risk_aversion"] * 2
        mu = self.mean_estimator.estimate(X=X) * (-1)
        self.objective = Objective(q=mu, P=covmat)

    def objective_batch(self, stage):
        import torch
        from . import engine
        nan = stage.panel.has_nan   # missing values: pairwise covariance, dense P (no window form)
        lowrank = stage.prefer_lowrank and self.covariance.spec["method"] != "duv" and not nan
        S, pdiag, mu_c, dg = self.covariance.estimate_batch_lr(
            stage.panel, stage.rows, stage.tlen, out=None if lowrank else stage.P_buffer(),
            plan=None if (nan or lowrank) else stage.slide_plan(), materialise=not lowrank,
            groups=stage.group_plan() if lowrank else None)
        ra = float(self.params["risk_aversion"])
        B = stage.batch
        dev = stage.device
        if nan and S is None:
            return None
        if mu_c is None and not nan:  # duv: identity covariance
            S = stage.identity_P()
            pdiag = torch.zeros(B, dtype=torch.float64, device=dev)
        elif lowrank:   # factored form S = Xc'Xc / (T - 1) for the Woodbury solver (no n x n S)
            stage.lowrank = engine.LowRank(stage.panel, stage.rows, stage.tlen, mu=mu_c,
                                           w_scale=1.0 / (stage.tlen.to(torch.float64) - 1.0), dg=dg)
        me = self.mean_estimator
        if me.spec.get("method") != "geometric":
            return None
        a, b = me.window(int(stage.tlen_host.max()))
        if not np.all(stage.tlen_host == stage.tlen_host[0]) and (a, b) != (0, int(stage.tlen_host[0])):
            return None
        mrows, mtlen = stage.sub_windows(a, b)
        if nan:
            mu = stage.panel.window_nanmeans(mrows, mtlen, geometric=True)
            if bool(torch.isnan(mu[:, :stage.n]).any().item()):
                return None
        elif lowrank and mrows is stage.rows and stage.group_plan().ok:
            # the full windows of slide groups: one sliding log-sum pass per group
            mu = stage.panel.window_geomeans_grouped(stage.group_plan(), stage.tlen)
        else:
            mu = stage.panel.window_means(mrows, mtlen, geometric=True)
        sf = me.spec.get("scalefactor")
        if sf not in (None, 1):
            mu = torch.expm1(torch.log1p(mu) * sf)
        scale = torch.full((B,), 2.0 * ra, dtype=torch.float64, device=dev)
        return S, scale, scale * pdiag, -mu, None


class QEQW(Optimization):
    """P = 2 I, q = 0 (src/optimization.py:180-194)."""

    def __init__(self, **kwargs):
        super().__init__(**kwargs)
        self.covariance = Covariance(method="duv")

    def set_objective(self, optimization_data: OptimizationData) -> None:
        X = optimization_data["return_series"]
        self.objective = Objective(P=self.covariance.estimate(X=X) * 2, q=np.zeros(X.shape[1]))

    def objective_batch(self, stage):
        import torch
        B, dev = stage.batch, stage.device
        return (stage.identity_P(), torch.full((B,), 2.0, dtype=torch.float64, device=dev),
                None, torch.zeros((B, stage.ld), dtype=torch.float64, device=dev), None)


def _tracking_rho_defaults(params) -> None:
    """ADMM start for tracking objectives (uncentred Gram P = 2 X'X, q = -2 X'y): rho =
    0.2 mean(diag P) and no |q| floor.  The floor (Settings.rho0_qrel) is for nearly linear
    mean-variance objectives; here |q| ~ diag P and it would start rho ~10x too high.
    Measured on the usa-shaped SPTR replication (494 assets, 4544 daily dates): 22 ADMM
    iterations and no refactorisation, against 168 iterations and 3744 refactorisations with
    the mean-variance defaults (7.6k -> 67.6k QPs/s, tools/diag_ls.py)."""
    params.setdefault("rho0_rel", 0.2)
    params.setdefault("rho0_qrel", 0.0)


class LeastSquares(Optimization):
    """P = 2 X'X (+ 2 l2 I), q = -2 X'y, constant y'y (src/optimization.py:198-229)."""

    def __init__(self, covariance: Optional[Covariance] = None, **kwargs):
        super().__init__(**kwargs)
        self.covariance = covariance
        _tracking_rho_defaults(self.params)

    def set_objective(self, optimization_data: OptimizationData) -> None:
        X = optimization_data["return_series"]
        y = optimization_data["bm_series"]
        if self.params.get("log_transform"):
            X = np.log(1 + X)
            y = np.log(1 + y)
        if isinstance(X, pd.DataFrame) and isinstance(y, (pd.DataFrame, pd.Series)):
            if not X.index.equals(y.index):
                # the reference's X.T @ y raises on misaligned dates (src/optimization.py:215-217)
                raise ValueError("matrices are not aligned")
        G, xty, yty = _device_gram(X, y)
        P = 2 * G
        l2 = self.params.get("l2_penalty")
        if l2 is not None and l2 != 0:
            P = P + 2 * l2 * np.eye(P.shape[0])
        if isinstance(X, pd.DataFrame):
            P = pd.DataFrame(P, index=X.columns, columns=X.columns)
        self.objective = Objective(P=P, q=-2 * xty, constant=yty)

    def objective_batch(self, stage):
        import torch
        if stage.panel.bm is None:
            return None
        from . import engine
        if self.params.get("log_transform"):
            pan = stage.log1p_panel()
        else:
            pan = stage.panel
        gp = stage.group_plan() if stage.prefer_lowrank else None
        if gp is not None and gp.ok:   # the window form with slide groups: X'y, y'y, diag(X'X) in one sliding pass
            dg = torch.zeros((stage.batch, stage.ld), dtype=torch.float64, device=stage.device)
            xty, yty = pan.gram_xy_grouped(gp, stage.tlen, dg=dg)
            G = None
            stage.lowrank = engine.LowRank(pan, stage.rows, stage.tlen, mu=None, dg=dg)
        else:
            if stage.prefer_lowrank:   # factored form X'X (uncentred) for the Woodbury solver (no n x n G)
                G = None
                stage.lowrank = engine.LowRank(pan, stage.rows, stage.tlen, mu=None)
            else:
                G = pan.cov(stage.rows, stage.tlen, mode=1, out=stage.P_buffer(), plan=stage.slide_plan())
            xty, yty = pan.gram_xy(stage.rows, stage.tlen)
        B, dev = stage.batch, stage.device
        l2 = self.params.get("l2_penalty")
        scale = torch.full((B,), 2.0, dtype=torch.float64, device=dev)
        pdiag = torch.full((B,), 2.0 * float(l2), dtype=torch.float64, device=dev) if l2 else None
        return G, scale, pdiag, -2.0 * xty, yty


class WeightedLeastSquares(Optimization):
    """P = 2 X'WX, q = -2 X'Wy with half-life tau weights (src/optimization.py:232-259)."""

    def __init__(self, **kwargs):
        super().__init__(**kwargs)
        _tracking_rho_defaults(self.params)

    def _weights(self, T):
        lam = np.exp(-np.log(2) / self.params["tau"])
        w = lam ** np.arange(T)
        return np.flip(w / np.sum(w) * len(w))

    def set_objective(self, optimization_data: OptimizationData) -> None:
        X = optimization_data["return_series"]
        y = optimization_data["bm_series"]
        if self.params.get("log_transform"):
            X = np.log(1 + X)
            y = np.log(1 + y)
        Xv = np.asarray(to_numpy(X), dtype=np.float64)
        yv = np.asarray(to_numpy(y), dtype=np.float64).reshape(-1)
        sw = np.sqrt(self._weights(Xv.shape[0]))
        G, xty, yty = _device_gram(Xv * sw[:, None], yv * sw)
        self.objective = Objective(P=2 * G, q=-2 * xty, constant=yty)

    def objective_batch(self, stage):
        """Every date's WLS objective from one row-scaled panel.

        The reference's weights (src/optimization.py:242-246) are exponential in the row's
        age: the row r of the window ending at panel row e gets lam^(e - r) T / S_T, with
        S_T = sum_{i<T} lam^i.  Writing lam^(e - r) = lam^(a - r) lam^(e - a) for one anchor
        row a >= e of the whole chunk, the panel is scaled ONCE by sqrt(lam^(a - r)) and
        each date keeps a scalar c_e = lam^(e - a) T / S_T: X'WX = c_e Xs'Xs, X'Wy = c_e Xs'ys.
        K1 (Gram mode, sliding) or the window form then runs on the scaled panel unchanged,
        with c_e folded into p_scale (dense) or w_scale (window path)."""
        import torch
        from . import engine
        if stage.panel.bm is None:
            return None
        pan = stage.log1p_panel() if self.params.get("log_transform") else stage.panel
        lam = float(np.exp(-np.log(2) / self.params["tau"]))
        B, dev = stage.batch, stage.device
        t = stage.tlen_host.astype(np.int64)
        if np.any(t <= 0):
            return None
        # age counts window positions, not panel rows: rank every row the windows use
        # (weekend rows the builders drop are skipped) and require each window to be a run
        used = np.unique(np.concatenate([stage.rows_host[b, :t[b]] for b in range(B)]))
        pos = np.full(pan.D, -1, dtype=np.int64)
        pos[used] = np.arange(used.size)
        first = pos[stage.rows_host[:, 0]]
        last = pos[stage.rows_host[np.arange(B), t - 1]]
        if np.any(last - first != t - 1):
            return None
        a = int(last.max())
        if (a - int(first.min())) * -np.log2(lam) > 600:     # keep lam^(a - r) far from underflow
            return None
        age = np.where(pos >= 0, a - pos, 0)
        sw = torch.from_numpy(np.sqrt(lam ** age.astype(np.float64))).to(dev)
        span = engine.Panel(pan.R * sw[:, None], pan.bm * sw, device=dev)
        s_T = (1.0 - lam ** t) / (1.0 - lam) if lam < 1.0 else t.astype(np.float64)
        c = torch.from_numpy(lam ** (last - a).astype(np.float64) * t / s_T).to(dev)
        if stage.prefer_lowrank:
            G = None
            stage.lowrank = engine.LowRank(span, stage.rows, stage.tlen, mu=None, w_scale=c)
            scale = torch.full((B,), 2.0, dtype=torch.float64, device=dev)
        else:
            G = span.cov(stage.rows, stage.tlen, mode=1, out=stage.P_buffer(), plan=stage.slide_plan())
            scale = 2.0 * c
        xty, yty = span.gram_xy(stage.rows, stage.tlen)
        return G, scale, None, -2.0 * c[:, None] * xty, c * yty


class LAD(Optimization):
    """Least absolute deviation tracking (src/optimization.py:263-345): min sum |y - X w| as
    the reference's LP over [w; u; v].  solver_name 'mi355x' solves it with the batched
    device IPM of porqua_amd/lad.py; other names build the reference's dense LP for
    qpsolvers exactly as src/optimization.py:296-345 does."""

    def __init__(self, **kwargs):
        super().__init__(**kwargs)
        self.params["use_level"] = self.params.get("use_level", True)
        self.params["use_log"] = self.params.get("use_log", True)

    def set_objective(self, optimization_data: OptimizationData) -> None:
        X = optimization_data["return_series"]
        y = optimization_data["bm_series"]
        if self.params.get("use_level"):
            X = (1 + X).cumprod()
            y = (1 + y).cumprod()
            if self.params.get("use_log"):
                X = np.log(X)
                y = np.log(y)
        self.objective = Objective(X=X, y=y)

    def _bounds(self):
        boxed = self.constraints.box["box_type"] != "NA"
        lb = self.constraints.box["lower"].to_numpy(dtype=np.float64) if boxed else None
        ub = self.constraints.box["upper"].to_numpy(dtype=np.float64) if boxed else None
        return lb, ub

    def solve(self) -> bool:
        """src/optimization.py:286-294 (results hold the weights only, as there)."""
        universe = self.constraints.selection
        if self.params.get("solver_name") not in qp_problems.ENGINE_SOLVERS:
            self.model_qpsolvers()
            self.model.solve()
            x = self.model["solution"].x
        else:
            import torch
            from . import engine
            from . import lad as _lad
            if "leverage" in self.constraints.l1:
                raise TypeError("LAD with a leverage constraint: the reference's np.zeros() call "
                                "raises here (src/optimization.py:333)")
            X = np.ascontiguousarray(to_numpy(self.objective["X"]), dtype=np.float64)
            y = np.ascontiguousarray(to_numpy(self.objective["y"]), dtype=np.float64).reshape(-1)
            dev = engine.default_device()
            GhAb = self.constraints.to_GhAb()
            lb, ub = self._bounds()
            pr = _lad.LADProblem(torch.from_numpy(X)[None].to(dev), torch.from_numpy(y)[None].to(dev),
                                 A=GhAb["A"], b=GhAb["b"], G=GhAb["G"], h=GhAb["h"], lb=lb, ub=ub)
            res = _lad.lad_ipm_batched(pr)
            x = res.x[0].cpu().numpy() if bool(res.found[0]) else None
        w = x[:len(universe)] if x is not None else [None] * len(universe)
        self.results = {"weights": pd.Series(w, index=universe).to_dict()}
        return True

    def lad_batch(self, panel, rows, tlen, GhAb, lb, ub):
        """Every window of a backtest chunk in one device IPM: (W, status, obj) or None."""
        import torch
        from . import lad as _lad
        if panel.bm is None or len(tlen) == 0 or np.any(tlen != tlen[0]) or tlen[0] < 1:
            return None
        if "leverage" in self.constraints.l1:
            return None
        # the row table is padded to the longest window of the whole backtest: slice it to
        # this chunk's (uniform) window length, or the padding rows would join the LP
        rows = np.asarray(rows)[:, :int(tlen[0])]
        idx = torch.from_numpy(np.ascontiguousarray(rows, dtype=np.int64)).to(panel.device)
        X, y = panel.R[idx], panel.bm[idx]
        if self.params.get("use_level"):
            X, y = torch.cumprod(1 + X, 1), torch.cumprod(1 + y, 1)
            if self.params.get("use_log"):
                X, y = torch.log(X), torch.log(y)
        pr = _lad.LADProblem(X.contiguous(), y.contiguous(), A=GhAb["A"], b=GhAb["b"], G=GhAb["G"],
                             h=GhAb["h"], lb=lb, ub=ub)
        res = _lad.lad_ipm_batched(pr)
        n = panel.n
        return res.x[:, :n].cpu().numpy(), res.status.cpu().numpy(), res.obj.cpu().numpy()

    def model_qpsolvers(self) -> None:
        """The reference's dense LP for a non-engine solver (src/optimization.py:296-345)."""
        X = to_numpy(self.objective["X"])
        y = to_numpy(self.objective["y"]).reshape(-1)
        GhAb = self.constraints.to_GhAb()
        N, T = X.shape[1], X.shape[0]
        G_t = np.pad(GhAb["G"], [(0, 0), (0, 2 * T)]) if GhAb["G"] is not None else None
        A = GhAb["A"]
        meq = 0 if A is None else 1 if A.ndim == 1 else A.shape[0]
        A_t = np.zeros((T, N + 2 * T)) if A is None else np.pad(np.atleast_2d(A), [(0, T), (0, 2 * T)])
        A_t[meq:T + meq, :N] = X
        A_t[meq:T + meq, N:N + T] = np.eye(T)
        A_t[meq:T + meq, N + T:] = -np.eye(T)
        b_t = y if GhAb["b"] is None else np.append(GhAb["b"], y)
        lb, ub = self._bounds()
        lb = np.pad(np.full(N, -np.inf) if lb is None else lb, (0, 2 * T))
        ub = np.pad(np.full(N, np.inf) if ub is None else ub, (0, 2 * T), constant_values=np.inf)
        if "leverage" in self.constraints.l1:
            raise TypeError("LAD with a leverage constraint: the reference's np.zeros() call raises "
                            "(src/optimization.py:333)")
        self.model = qp_problems.QuadraticProgram(P=np.zeros((N + 2 * T, N + 2 * T)),
                                                  q=np.append(np.zeros(N), np.ones(2 * T)),
                                                  G=G_t, h=GhAb["h"], A=A_t, b=b_t, lb=lb, ub=ub,
                                                  params=self.params)
