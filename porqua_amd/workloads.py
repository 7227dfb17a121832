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
                 seed: int | None = None, graph: bool = False):
        self.n, self.T = n, T
        # graph mode: the step's stages are sync-free and captured as HIP graphs after a first
        # eager step (engine.StageGraphs), on a stream of its own
        self.graph = graph
        self.graphs = None
        self.sf_rounds = None
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
        self.gplan = engine.GroupPlan(self.rows, self.tlen, dev, gmin=gmin, polish_full=True) if group else None
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
        window moments [-> K1 covariance] -> K2 -> K3 -> K4.  Weights stay on the device.

        Graph mode (``graph=True``, the group-capacitance path): the solve is sync-free
        (engine.solve_lowrank(sync_free=True): one ADMM launch, a fixed number of polish
        rounds -- the most the previous step needed -- and one flag read that runs the
        host-driven repairs only when something is left), every stage after the first step a
        replayed HIP graph on the workload's own stream (joined to the caller's stream on
        both sides, no host sync)."""
        if not (self.graph and self.use_lr and self.grouped):
            return self._step(events)
        if self.graphs is None:
            self.graphs = engine.StageGraphs()
            self._stream = torch.cuda.Stream(device=self.device)
        cur = torch.cuda.current_stream()
        self._stream.wait_stream(cur)
        with torch.cuda.stream(self._stream):
            self.graphs.begin()
            res = self._step(events)
        cur.wait_stream(self._stream)
        if self.sf_rounds is None:   # rounds the polish needed (one host read, first step only)
            self.sf_rounds = max(2, int(res.out[:, engine._lib.PQ_OUT_ROUNDS].max().item()))
        return res

    @property
    def graph_replays(self) -> int:
        """Stage graphs replayed so far (tests, diagnostics)."""
        return self.graphs.replays if self.graphs is not None else 0

    def prepare(self):
        """Graph mode: the first (eager, cache-filling) step and the capturing step, outside
        any timed region -- afterwards every step replays the captured stages."""
        if self.graph:
            for _ in range(2):
                self.step()
            torch.cuda.synchronize()

    def _step(self, events):
        tl = engine._Timeline(events, self.graphs)

        def moments():
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
        tl("moments+cov" if self.with_cov else "moments", moments)
        if self.use_lr:
            return engine.solve_lowrank(self.qb, self.lr, self.settings, self.ws, events=events,
                                        groups=self.gplan, sync_free=self.graphs is not None,
                                        graphs=self.graphs, sf_rounds=self.sf_rounds)
        return engine.solve(self.qb, self.settings, self.ws, events=events)

    def certificate(self, res: engine.BatchResult, chunk: int = 256) -> dict:
        lb = torch.zeros(self.n, dtype=F64, device=self.device)
        ub = torch.ones(self.n, dtype=F64, device=self.device)
        return window_certificate(self.pan.R, self.rows_d, self.tlen_d, self.mu, self.qb.p_scale * self.w_scale,
                                  self.qb.q[:, :self.n], res, A_row=torch.ones(self.n, dtype=F64, device=self.device),
                                  b=1.0, lb=lb, ub=ub, chunk=chunk)


class _LSTrackingBatch:
    """Least-squares tracking backtest on one device (LeastSquares.set_objective,
    src/optimization.py:206-226): P = 2 X'X (uncentred window Gram), q = -2 X'y, budget
    1'x = 1, long-only box [0, 1] and optional shared general rows G x <= h
    (Constraints.add_linear / to_GhAb, src/constraints.py:66-94, 114-167).  The panel slice
    ``R`` / ``y`` / ``dates`` holds exactly the rows this rank's windows touch; its ``D``
    rebalance dates are the slice's rows T - 1 .. T - 2 + D.  q is formed inside ``step``
    (the X'y window products are part of the per-date objective)."""

    def _setup(self, dates, R, y, T, D, device, settings, G=None, h=None, stride=1):
        self.T = T
        self.device = dev = device or engine.default_device()
        self.D = D
        self.n = n = R.shape[1]
        self.R_rank, self.y_rank, self.dates_rank = R, y, dates
        self.ends_local = T - 1 + stride * np.arange(D)
        self.rows, self.tlen = engine.window_rows(dates, dates[self.ends_local], T)
        self.pan = engine.Panel(R, y, device=dev)
        self.rows_d, self.tlen_d = self.pan.rows_to_device(self.rows, self.tlen)
        self.G = G
        qb = engine.QPBatch.from_dense(None, None, A=np.ones((1, n)), b=np.ones(1), G=G, h=h, lb=np.zeros(n),
                                       ub=np.ones(n), device=dev, n=n)
        qb.batch = D
        qb.q = torch.zeros((D, qb.ld), dtype=F64, device=dev)
        qb.p_scale = torch.full((D,), 2.0, dtype=F64, device=dev)
        self.qb = qb
        self.plan = None
        self.mu = None
        self.gplan = engine.GroupPlan(self.rows, self.tlen, dev, polish_full=True)
        self.lr = engine.LowRank(self.pan, self.rows_d, self.tlen_d, mu=None)
        self.use_lr, self.with_cov = True, False
        self.settings = settings
        self.ws = engine.Workspace(qb, dense=False)

    @property
    def grouped(self) -> bool:
        return engine.grouped_applicable(self.qb, self.lr, self.gplan, self.ws)

    def step(self, events: list | None = None) -> engine.BatchResult:
        if events is not None:
            e0 = torch.cuda.Event(enable_timing=True)
            e0.record()
        if self.gplan.ok:   # X'y and diag(X'X) of every window in one sliding pass per group
            xty, _ = self.pan.gram_xy_grouped(self.gplan, self.tlen_d, dg=self.lr.dg)
        else:
            xty, _ = self.pan.gram_xy(self.rows_d, self.tlen_d)
            self.lr.refresh()
        torch.mul(xty, -2.0, out=self.qb.q)
        if events is not None:
            e1 = torch.cuda.Event(enable_timing=True)
            e1.record()
            events.append(("moments", e0, e1))
        return engine.solve_lowrank(self.qb, self.lr, self.settings, self.ws, events=events, groups=self.gplan)

    def certificate(self, res: engine.BatchResult, chunk: int = 128) -> dict:
        qb, n = self.qb, self.n
        return window_certificate(self.pan.R, self.rows_d, self.tlen_d, None, self.qb.p_scale, qb.q[:, :n], res,
                                  lb=torch.zeros(n, dtype=F64, device=self.device),
                                  ub=torch.ones(n, dtype=F64, device=self.device), chunk=chunk,
                                  C=qb.Cg[0, :qb.mg, :n], lg=qb.lg[0, :qb.mg], ug=qb.ug[0, :qb.mg])


class TrackingBacktest(_LSTrackingBatch):
    """Config 4 on one device (BASELINE.json configs[3]): a synthetic factor panel with 20
    sectors, n = 3000 assets, 252-day windows, daily rebalancing, tracking-error least
    squares with budget, long-only box and 20 sector caps G x <= 0.15: 21 shared general
    rows.  ``strong``: ``D`` dates in total, contiguous block per rank; otherwise ``D`` dates
    per rank of one longer panel."""

    N_SECTORS = 20
    CAP = 0.15

    def __init__(self, n: int = 3000, T: int = 252, D: int = 9749, rank: int = 0, world: int = 1,
                 device=None, settings: engine.Settings | None = None, strong: bool = False):
        if strong:
            per = -(-D // world)
            lo = rank * per
            Dr = max(0, min(D, lo + per) - lo)
            d_total = T - 1 + D
        else:
            lo = rank * D
            Dr = D
            d_total = T - 1 + D * world
        self.global_dates = D if strong else D * world
        dates, R, y, sec = factor_panel(d_total, n, n_sectors=self.N_SECTORS)
        self.row_offset = lo
        G = np.stack([(sec == g).astype(float) for g in range(self.N_SECTORS)])
        # tracking objectives start at a small rho (engine.Settings docs; tools/bench_configs.py)
        self._setup(dates[lo:lo + T - 1 + Dr], R[lo:lo + T - 1 + Dr], y[lo:lo + T - 1 + Dr], T, Dr, device,
                    settings or engine.Settings(rho0_rel=0.1, rho0_qrel=0.0), G=G,
                    h=np.full(self.N_SECTORS, self.CAP))


class ReplicationBacktest(_LSTrackingBatch):
    """Configs 1 / 2 on one device (BASELINE.json configs[0..1]): the reference notebook's SPTR
    index replication (example/backtest.ipynb: LeastSquares, budget + LongOnly box, width 252)
    on the usa-shaped panel (synthetic.usa_panel: 494 assets on the last 4795 real SPTR dates;
    usa_returns itself is absent from the reference tree), rebalanced every ``stride`` rows
    from the first full window on: stride 1 = every date (config 2's 4795 - 251 = 4544 daily
    QPs), stride 21 = the notebook's monthly rebalancing (``dates[::21]``, 217 QPs over the
    panel).  ``sptr_days`` / ``sptr``: the real SPTR series (tests/golden/sptr.npz, captured
    from the reference's data/SPTR.csv).

    Multi-GPU: the fixed set of dates is split into contiguous blocks (strong scaling,
    backtest.shard_range); each rank uploads only the panel rows its windows touch."""

    def __init__(self, sptr_days, sptr, T: int = 252, rank: int = 0, world: int = 1, device=None,
                 settings: engine.Settings | None = None, n: int = 494, n_rows: int = 4795, stride: int = 1):
        from .backtest import shard_range
        from .synthetic import usa_panel
        days, R, y = usa_panel(sptr_days, sptr, n_assets=n, n_rows=n_rows)
        total = (len(days) - (T - 1) + stride - 1) // stride
        self.global_dates = total
        lo, hi = shard_range(total, rank, world)
        self.row_offset = lo * stride
        r0, r1 = lo * stride, (hi - 1) * stride + T if hi > lo else lo * stride
        # LeastSquares' tracking rho (porqua_amd/optimization.py: rho0_rel 0.2, no |q| floor)
        self._setup(days[r0:r1], R[r0:r1], y[r0:r1], T, hi - lo, device,
                    settings or engine.Settings(rho0_rel=0.2, rho0_qrel=0.0), stride=stride)
        if self.D and int(self.tlen.min()) != T:
            raise ValueError("ReplicationBacktest: the SPTR calendar slice has a short window")


class SweepBacktest:
    """Config 5 (BASELINE.json configs[4]): synthetic 5000-asset factor panel, ``dates``
    monthly rebalance dates (every 21st row, 252-day windows) x ``n_lambdas`` risk aversions
    log-spaced in [0.1, 100]: 64 x 64 = 4096 mean-variance QPs P = 2 lam Sigma_d, q = -mu_d
    (geometric), budget + long-only box (porqua_amd.sweep; src/optimization.py:157-174).

    Multi-GPU: the fixed grid is sharded by DATE (strong scaling), every
    risk aversion of a date on the rank that owns it, so the date's window Gram and
    eigendecomposition are shared by its lambda row."""

    def __init__(self, n: int = 5000, T: int = 252, dates: int = 64, n_lambdas: int = 64, stride: int = 21,
                 rank: int = 0, world: int = 1, device=None, settings: engine.Settings | None = None,
                 factor: str = "auto"):
        from .sweep import MeanVarianceSweep
        self.n, self.T = n, T
        self.device = dev = device or engine.default_device()
        d_all, R, y, _ = factor_panel(T - 1 + stride * dates, n)
        ends = np.arange(T - 1, T - 1 + stride * dates, stride)
        rows, tlen = engine.window_rows(d_all, d_all[ends], T)
        self.R_rank, self.y_rank, self.dates_rank = R, y, d_all
        self.pan = engine.Panel(R, device=dev)
        self.lambdas = np.logspace(-1, 2, n_lambdas)
        self.sweep = MeanVarianceSweep(self.pan, rows, tlen, self.lambdas, settings=settings, factor=factor,
                                       rank=rank, world=world)
        sw = self.sweep
        self.D = sw.B                                   # problems of this rank
        self.global_dates = dates * n_lambdas           # problems of the whole job
        self.ends_local = ends[sw.lo:sw.hi]
        self.qb, self.lr, self.gplan, self.ws = sw.qb, sw.lr, sw.gp, sw.ws
        self.plan, self.mu = None, sw.mu_c
        self.use_lr, self.with_cov = True, False
        self.settings = sw.settings
        self._meta = None

    @property
    def grouped(self) -> bool:
        return self.gplan is not None and engine.grouped_applicable(self.qb, self.lr, self.gplan, self.ws)

    def step(self, events: list | None = None) -> engine.BatchResult:
        res, self._meta = self.sweep.solve(events)
        return res

    def certificate(self, res: engine.BatchResult, chunk: int = 128) -> dict:
        return sweep_certificate(self.pan, res, self._meta, chunk=chunk)


def window_certificate(R, rows, tlen, mu, scale, q, res: engine.BatchResult, A_row=None, b=None, lb=None, ub=None,
                       chunk: int = 256, C=None, lg=None, ug=None, rows_of=None, p_diag=None) -> dict:
    """KKT residuals of every solution of a window-path batch, P_p = scale_p * Xc_p' Xc_p
    (Xc = window rows minus ``mu``; ``mu`` None = uncentred).  P x is recomputed here with
    torch from the panel rows, not by the engine's kernels.

    General rows: ``C`` (mg, n) with bounds ``lg <= C x <= ug`` (equalities lg == ug, as the
    engine stores them: equality rows first) and multipliers ``res.y`` (mg); the legacy form
    ``A_row' x = b`` is one equality row.  Box ``lb <= x <= ub`` with multipliers
    ``res.z_box``.  ``rows_of`` (optional int64 device tensor, one entry per problem) maps
    problem p to its window / moments row in ``rows``, ``tlen``, ``mu`` (e.g. the date of a
    risk-aversion sweep problem).  ``p_diag`` (optional, one value per problem): a ridge,
    P_p = scale_p Xc_p'Xc_p + p_diag_p I.

    Returns the maxima over the batch of
      * ``max_violation``: max(|C x - b| on equality rows, [C x - ug]+, [lg - C x]+,
        [lb - x]+, [x - ub]+) (absolute, the BASELINE bar);
      * ``max_rel_stationarity``: ||P x + q + C'y + z_box||inf /
        max(||P x||inf, ||q||inf, ||C'y||inf, ||z_box||inf)  (OSQP-style relative);
      * ``max_rel_complementarity``: the multipliers' complementarity products (box and
        inequality rows) over the same scale; plus ``max_dual_sign``: the largest wrong-sign
        multiplier of an inequality row over the scale;
    and the status histogram."""
    B, n = res.x.shape
    dev = R.device
    tmax = rows.shape[1]
    if C is None:
        C = A_row.reshape(1, n)
        lg = ug = torch.full((1,), float(b), dtype=F64, device=dev)
    C = C.to(dev, F64)
    lg = lg.to(dev, F64)
    ug = ug.to(dev, F64)
    mg = C.shape[0]
    eq = lg == ug
    viol = torch.zeros((), dtype=F64, device=dev)
    stat = torch.zeros((), dtype=F64, device=dev)
    comp = torch.zeros((), dtype=F64, device=dev)
    dsign = torch.zeros((), dtype=F64, device=dev)
    ar = torch.arange(tmax, device=dev)
    for s in range(0, B, chunk):
        e = min(B, s + chunk)
        x = res.x[s:e]
        ri = torch.arange(s, e, device=dev) if rows_of is None else rows_of[s:e]
        X = R[rows[ri].long()]                                          # (b, tmax, n)
        valid = (ar[None, :] < tlen[ri, None]).to(F64)
        if mu is not None:
            X = X - mu[ri, None, :n]
        X = X * valid[:, :, None]
        v = torch.bmm(X, x[:, :, None])                                 # (b, tmax, 1)
        Px = scale[s:e, None] * torch.bmm(X.transpose(1, 2), v)[:, :, 0]
        if p_diag is not None:
            Px = Px + p_diag[s:e, None] * x
        y = res.y[s:e, :mg]
        zb = res.z_box[s:e]
        Cty = y @ C
        r = Px + q[s:e] + Cty + zb
        sc = torch.stack([Px.abs().amax(1), q[s:e].abs().amax(1), Cty.abs().amax(1), zb.abs().amax(1)]).amax(0)
        sc = torch.clamp(sc, min=torch.finfo(F64).tiny)
        stat = torch.maximum(stat, (r.abs().amax(1) / sc).max())
        cx = x @ C.T                                                    # (b, mg)
        gv = torch.maximum((cx - ug).clamp(min=0), (lg - cx).clamp(min=0))
        pv = torch.stack([gv.amax(1), (lb - x).clamp(min=0).amax(1), (x - ub).clamp(min=0).amax(1)])
        viol = torch.maximum(viol, pv.max())
        cp = torch.maximum((zb.clamp(max=0) * (x - lb)).abs().amax(1), (zb.clamp(min=0) * (ub - x)).abs().amax(1))
        if bool((~eq).any()):
            ye = y[:, ~eq]
            ugf = torch.where(torch.isfinite(ug[~eq]), ug[~eq], torch.zeros_like(ug[~eq]))
            lgf = torch.where(torch.isfinite(lg[~eq]), lg[~eq], torch.zeros_like(lg[~eq]))
            # a multiplier of the right sign at an infinite bound is caught by max_dual_sign
            cg = torch.maximum((ye.clamp(min=0) * (ugf - cx[:, ~eq]) * torch.isfinite(ug[~eq])).abs(),
                               (ye.clamp(max=0) * (cx[:, ~eq] - lgf) * torch.isfinite(lg[~eq])).abs()).amax(1)
            cp = torch.maximum(cp, cg)
            # a one-sided row (lg = -inf) must carry y >= 0, (ug = +inf) y <= 0
            ws = torch.maximum((-ye).clamp(min=0) * torch.isinf(lg[~eq]), ye.clamp(min=0) * torch.isinf(ug[~eq]))
            dsign = torch.maximum(dsign, (ws.amax(1) / sc).max())
        comp = torch.maximum(comp, (cp / sc).max())
    st = res.status.cpu().numpy()
    return {"max_violation": float(viol.item()), "max_rel_stationarity": float(stat.item()),
            "max_rel_complementarity": float(comp.item()), "max_dual_sign": float(dsign.item()),
            "problems": int(B),
            "status_counts": {str(k): int(v) for k, v in zip(*np.unique(st, return_counts=True))}}


def sweep_certificate(panel, res: engine.BatchResult, meta: dict, chunk: int = 128) -> dict:
    """window_certificate of a porqua_amd.sweep.mean_variance_sweep batch (P = 2 lam Sigma_d,
    q = -mu_d, budget + box), from the batch as it was solved (``meta['qb']``, ``meta['lr']``)."""
    qb, lr = meta["qb"], meta["lr"]
    n, mg = qb.n, qb.mg
    scale = qb.p_scale * lr.w_scale
    return window_certificate(panel.R, lr.rows, lr.tlen, lr.mu, scale, qb.q[:, :n], res,
                              lb=qb.lb[0, :n], ub=qb.ub[0, :n], chunk=chunk, C=qb.Cg[0, :mg, :n],
                              lg=qb.lg[0, :mg], ug=qb.ug[0, :mg])
