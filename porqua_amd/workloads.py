"""The benchmark workloads of BASELINE.json as reusable device problems.

``MinVarianceBacktest`` is configs[2] exactly as ``bench.py`` times it: a synthetic
factor panel (``synthetic.factor_panel``, seed 20240314), n = 1000 assets, 252-day
windows, daily rebalancing (4749 dates per rank), long-only min-variance
(P = 2 * Pearson covariance, q = 0, budget 1'x = 1, box 0 <= x <= 1; the reference's
``MeanVariance`` without a return term and the default ``bibfn_box_constraints``,
src/optimization.py:168-174, src/builders.py:272-287).  The headline parity test
(tests/test_headline_parity_gpu.py) builds the same object, so the problem it checks is
the problem the bench measures.

``window_certificate`` is an independent KKT check of window-path solutions: P x is
recomputed from the panel rows with torch (not by the engine's kernels), so a wrong
kernel cannot certify itself.
"""
from __future__ import annotations

import os

import numpy as np
import torch

from . import engine
from .synthetic import factor_panel

F64 = torch.float64


class MinVarianceBacktest:
    """Config 3 on one device: dates ``[rank * D, (rank + 1) * D)`` of a panel of
    ``T - 1 + D * world`` rows (weak scaling) or, with ``strong=True``, the rank's share of
    ``D`` dates in total (strong scaling, contiguous blocks)."""

    def __init__(self, n: int = 1000, T: int = 252, D: int = 4749, rank: int = 0, world: int = 1,
                 device=None, settings: engine.Settings | None = None, path: str = "auto",
                 group: bool = True, slide: bool = True, with_cov: bool = False, strong: bool = False,
                 seed: int | None = None):
        self.n, self.T = n, T
        self.device = dev = device or engine.default_device()
        if strong:   # D dates in total, contiguous blocks (the last rank takes the remainder)
            per = -(-D // world)
            lo = rank * per
            self.D = max(0, min(D, lo + per) - lo)
            d_total = T - 1 + D
        else:
            lo = rank * D
            self.D = D
            d_total = T - 1 + D * world
        self.global_dates = D if strong else D * world
        D = self.D
        dates, R, y, _ = factor_panel(d_total, n, **({} if seed is None else {"seed": seed}))
        self.R_rank = R[lo:lo + T - 1 + D]                       # rows [lo, lo + T - 1 + D)
        self.y_rank = y[lo:lo + T - 1 + D]
        self.ends_local = np.arange(T - 1, T - 1 + D)            # rebalance row within the slice
        self.row_offset = lo
        sl_dates = dates[lo:lo + T - 1 + D]
        self.dates_rank = sl_dates
        self.rebdates = sl_dates[self.ends_local]
        self.rows, self.tlen = engine.window_rows(sl_dates, self.rebdates, T)
        self.pan = engine.Panel(self.R_rank, device=dev)
        self.rows_d, self.tlen_d = self.pan.rows_to_device(self.rows, self.tlen)
        self.plan = engine.SlidePlan(self.rows, self.tlen, dev) if slide else None
        gmin = int(os.environ.get("PQ_GROUP_MIN", "4"))     # experiments: smallest slide group size
        self.gplan = engine.GroupPlan(self.rows, self.tlen, dev, gmin=gmin) if group else None
        qb = engine.QPBatch.from_dense(np.zeros((1, n, n)), np.zeros((1, n)), A=np.ones((1, n)),
                                       b=np.ones(1), lb=np.zeros(n), ub=np.ones(n), device=dev)
        qb.batch = D                                             # D problems sharing constraints
        qb.P = None
        qb.q = torch.zeros((D, qb.ld), dtype=F64, device=dev)
        qb.p_scale = torch.full((D,), 2.0, dtype=F64, device=dev)   # P = 2 * Sigma
        self.qb = qb
        self.settings = settings or engine.Settings()
        self.mu = self.pan.window_means(self.rows_d, self.tlen_d)
        self.w_scale = 1.0 / (self.tlen_d.to(F64) - 1.0)
        self.lr = engine.LowRank(self.pan, self.rows_d, self.tlen_d, mu=self.mu, w_scale=self.w_scale)
        self.use_lr = path == "lowrank" or (path == "auto" and engine.lowrank_applicable(qb, self.lr))
        self.with_cov = (not self.use_lr) or with_cov
        if self.with_cov:   # K1 writes Sigma every step (dense path: P = 2 Sigma is what K2 factors)
            qb.P = torch.empty((D, qb.ld, qb.ld), dtype=F64, device=dev)
        self.ws = engine.Workspace(qb, dense=not self.use_lr)

    @property
    def grouped(self) -> bool:
        return self.use_lr and engine.grouped_applicable(self.qb, self.lr, self.gplan, self.ws)

    def step(self, events: list | None = None) -> engine.BatchResult:
        """One pass of the hot path over every date of this rank (inputs resident in HBM):
        window moments [-> K1 covariance] -> K2 -> K3 -> K4.  Weights stay on the device."""
        if events is not None:
            e0 = torch.cuda.Event(enable_timing=True)
            e0.record()
        if self.use_lr and self.gplan is not None and self.gplan.ok:
            # mu and diag(Xc'Xc) (the only O(n) per-date moments) in one sliding pass per group
            mu, _ = self.pan.window_moments_grouped(self.gplan, self.tlen_d, self.mu, self.lr.dg)
        else:
            mu = self.pan.window_means(self.rows_d, self.tlen_d, out=self.mu)
            if self.use_lr:
                self.lr.refresh()
        if self.with_cov:
            self.pan.cov(self.rows_d, self.tlen_d, mode=0, out=self.qb.P, mu=mu, plan=self.plan,
                         lower_only=self.use_lr)
        if events is not None:
            e1 = torch.cuda.Event(enable_timing=True)
            e1.record()
            events.append(("moments+cov" if self.with_cov else "moments", e0, e1))
        if self.use_lr:
            return engine.solve_lowrank(self.qb, self.lr, self.settings, self.ws, events=events,
                                        groups=self.gplan)
        return engine.solve(self.qb, self.settings, self.ws, events=events)

    def certificate(self, res: engine.BatchResult, chunk: int = 256) -> dict:
        lb = torch.zeros(self.n, dtype=F64, device=self.device)
        ub = torch.ones(self.n, dtype=F64, device=self.device)
        return window_certificate(self.pan.R, self.rows_d, self.tlen_d, self.mu, self.qb.p_scale * self.w_scale,
                                  self.qb.q[:, :self.n], res, A_row=torch.ones(self.n, dtype=F64, device=self.device),
                                  b=1.0, lb=lb, ub=ub, chunk=chunk)


def window_certificate(R, rows, tlen, mu, scale, q, res: engine.BatchResult, A_row, b, lb, ub,
                       chunk: int = 256) -> dict:
    """KKT residuals of every solution of a window-path batch with one equality row
    ``A_row' x = b`` and a box, P_d = scale_d * Xc_d' Xc_d (Xc = window rows minus ``mu``;
    ``mu`` None = uncentred).  P x is recomputed here with torch from the panel rows.

    Returns the maxima over the batch of
      * ``max_violation``: max(|A x - b|, [lb - x]+, [x - ub]+) (absolute, the BASELINE bar);
      * ``max_rel_stationarity``: ||P x + q + A'y + z_box||inf /
        max(||P x||inf, ||q||inf, ||A'y||inf, ||z_box||inf)  (OSQP-style relative);
      * ``max_rel_complementarity``: max |z_box^- (x - lb)|, |z_box^+ (ub - x)| over the
        same scale;
    and the status histogram."""
    B, n = res.x.shape
    tmax = rows.shape[1]
    viol = torch.zeros((), dtype=F64, device=R.device)
    stat = torch.zeros((), dtype=F64, device=R.device)
    comp = torch.zeros((), dtype=F64, device=R.device)
    ar = torch.arange(tmax, device=R.device)
    for s in range(0, B, chunk):
        e = min(B, s + chunk)
        x = res.x[s:e]
        X = R[rows[s:e].long()]                                         # (b, tmax, n)
        valid = (ar[None, :] < tlen[s:e, None]).to(F64)
        if mu is not None:
            X = X - mu[s:e, None, :n]
        X = X * valid[:, :, None]
        v = torch.bmm(X, x[:, :, None])                                 # (b, tmax, 1)
        Px = scale[s:e, None] * torch.bmm(X.transpose(1, 2), v)[:, :, 0]
        y = res.y[s:e, :1]
        zb = res.z_box[s:e]
        Aty = y * A_row[None, :]
        r = Px + q[s:e] + Aty + zb
        sc = torch.stack([Px.abs().amax(1), q[s:e].abs().amax(1), Aty.abs().amax(1), zb.abs().amax(1)]).amax(0)
        sc = torch.clamp(sc, min=torch.finfo(F64).tiny)
        stat = torch.maximum(stat, (r.abs().amax(1) / sc).max())
        pv = torch.stack([(x @ A_row - b).abs(), (lb - x).clamp(min=0).amax(1), (x - ub).clamp(min=0).amax(1)])
        viol = torch.maximum(viol, pv.max())
        cp = torch.maximum((zb.clamp(max=0) * (x - lb)).abs().amax(1), (zb.clamp(min=0) * (ub - x)).abs().amax(1))
        comp = torch.maximum(comp, (cp / sc).max())
    st = res.status.cpu().numpy()
    return {"max_violation": float(viol.item()), "max_rel_stationarity": float(stat.item()),
            "max_rel_complementarity": float(comp.item()),
            "status_counts": {str(k): int(v) for k, v in zip(*np.unique(st, return_counts=True))}}
