"""Risk-aversion x date grid of mean-variance QPs on the window path (BASELINE.json configs[4]).

For rebalance date d and risk aversion lam the reference's MeanVariance objective is
P = 2 lam Sigma_d, q = -mu_d (src/optimization.py:168-174; mu from
MeanEstimator.estimate_geometric, src/mean_estimation.py:39-48), solved per date by
QuadraticProgram.solve (src/qp_problems.py:184-216).  Here every (date, lam) pair is one
problem of a single batch, date-major: all problems of a date share its window rows, so
the grouped low-rank ADMM (engine.GroupPlan with identical windows) streams those rows
once per iteration for up to 16 risk aversions.  Nothing n x n is formed.

Multi-GPU (config 5 "across 8xMI355X"; SURVEY.md §8(e) "shard by date, keep all lambda of a
date on one rank so the factorisation is shared"): ``rank`` / ``world`` give each rank a
contiguous block of dates with every risk aversion of those dates, and ``gather`` all-gathers
the weight panels afterwards (MeanVarianceSweep).

Factor once per date (``factor='eig'``): the capacitance of problem (d, lam) is
M = I + (2 lam w / c) Xc_d Xc_d' + border rows, so one symmetric eigendecomposition of the
date's T x T window Gram diagonalises M for EVERY lam and every rho
(engine.EigCap / pq_eigcap_form): each problem keeps its own |q|-aware rho and its adaptive
rho updates, and its M^-1 is formed from the shared eigenvectors by one MFMA tile product
instead of a Cholesky factorisation per problem.  ``factor='chol'`` keeps the per-problem
factorisation (rounds 1-2).  Measured at the config-5 shape (profiles/r02g_*, tools/exp_eigh.py):
the 64 eigendecompositions cost 10.4 ms (rocSOLVER syevd, strided-batched; its Jacobi variant
71 ms) + 3.7 ms of forming, the 4096 batched Choleskys 8.2 ms -- 2.0 us per problem against
190 us per date + 0.9 us per problem, so ``factor='auto'`` (the default) takes the eigen form
from EIG_MIN_PER_DATE risk aversions per date (and whenever the windows are not all full, the
Cholesky form).  A round-2 attempt that instead rescaled every problem of a date
to P = 2 Sigma_d, q = -mu_d / lam (one capacitance per slide group) had to share one rho
per group and left the nearly linear problems (lam <= 0.13) on 4000-iteration ADMM tails:
102 QPs/s against 12.7k -- the eigen form needs no shared rho.
"""
from __future__ import annotations

import numpy as np
import torch

from . import engine

EIG_MIN_PER_DATE = 192   # factor='auto': eigen form from this many problems per date
# |q| floor of the initial rho for the sweep (engine.Settings.rho0_qrel, default 10): its
# small risk aversions are nearly linear.  Measured at the config-5 shape
# (tools/bench_configs.py --only 5 --set rho0_qrel=...): 3 -> 1826 max ADMM iterations, 10 -> 55, 30 -> 34 (27.8k -> 32.8k
# QPs/s), 60 -> 26, 100 -> problems fall to the eps_retry ADMM; 30 keeps a factor 3 from both
# cliffs.  (A single mean-variance backtest at risk aversion 1 is faster at 10.)
SWEEP_RHO0_QREL = 30.0
# The sweep's settings: the rho floor above, and the loose ADMM stop before the grouped polish
# on its per-problem capacitance (Settings.eps_grouped_percap; the problems of a date differ in
# P's scale, so they cannot share the group capacitance the loose stop was tuned on).
# Measured at the config-5 shape (profiles/r05c_*, r05d_*): eps 2e-3 (no loose stop) / 0.3 /
# 0.5 / 1.0 -> 58.6k / 94.2k / 100.1k / 67.4k QPs/s (24.6 / 13.2 / 11.6 / 8.0 ADMM iterations,
# 2.06 / 2.63 / 2.83 / 3.48 polish rounds; at 1.0 the free sets outgrow the LDS solve and dates
# fall back to the per-date polish after resuming ADMM); min_iter_grouped 6 / 8 / 10 changes
# nothing at 0.3
SWEEP_SETTINGS = {"rho0_qrel": SWEEP_RHO0_QREL, "eps_grouped": 0.5, "eps_grouped_percap": True}


class MeanVarianceSweep:
    """A risk-aversion x date grid staged once on the device; ``solve()`` is one pass of the
    hot path over it (window moments -> geometric means -> [eigen capacitance] -> K2-K4).

    Multi-GPU: ``rank`` / ``world`` shard the DATES into
    contiguous blocks (backtest.shard_range) and keep every risk aversion of a date on the
    rank that owns the date, so the date's window Gram / eigendecomposition is formed once
    and shared by its whole lambda row; this rank's problems are dates [lo, hi) x all
    lambdas, date-major (local problem p = (d - lo) * L + j).  No data-path collective: the
    weight panels are all-gathered afterwards (``gather``)."""

    def __init__(self, panel: engine.Panel, rows, tlen, lambdas, lb=0.0, ub=1.0, budget=1.0,
                 geometric=True, settings: engine.Settings | None = None, group=True,
                 factor: str = "auto", gmax: int = engine.GROUP_MAX_DATES,
                 ws: "engine.Workspace | None" = None, eig_backend: str = "rocsolver",
                 rank: int = 0, world: int = 1):
        from .backtest import shard_range
        if factor not in ("auto", "eig", "chol"):
            raise ValueError("mean_variance_sweep: factor must be 'auto', 'eig' or 'chol'")
        if not (0 <= rank < world):
            raise ValueError("mean_variance_sweep: 0 <= rank < world required")
        rows = np.asarray(rows, dtype=np.int32)
        tlen = np.asarray(tlen, dtype=np.int32)
        self.lam = lam = np.asarray(lambdas, dtype=np.float64).reshape(-1)
        self.nd_total = len(tlen)
        self.lo, self.hi = shard_range(self.nd_total, rank, world)
        self.rank, self.world = rank, world
        rows, tlen = rows[self.lo:self.hi], tlen[self.lo:self.hi]
        nd, L, n = len(tlen), len(lam), panel.n
        self.nd, self.L, self.n = nd, L, n
        self.panel, self.geometric, self.eig_backend = panel, geometric, eig_backend
        dev = self.device = panel.device
        self.r_d, self.t_d = panel.rows_to_device(rows, tlen)
        k_ld = engine.round_up(rows.shape[1] + 1, 64)
        ld = engine.round_up(n, 64)
        self.mu_c = torch.zeros((nd, ld), dtype=torch.float64, device=dev)      # centring of Sigma
        self.mu_q = torch.zeros((nd, ld), dtype=torch.float64, device=dev) if geometric else self.mu_c
        rows_p = np.repeat(rows, L, axis=0)
        tlen_p = np.repeat(tlen, L)
        self.rp_d, self.tp_d = panel.rows_to_device(rows_p, tlen_p)
        B = self.B = nd * L
        qb = engine.QPBatch(n, B, 1, device=dev, P=torch.empty(0, dtype=torch.float64, device=dev))
        qb.P = None
        qb.Cg[0, 0, :n] = 1.0
        qb.lg[0, 0] = qb.ug[0, 0] = float(budget)
        qb.lb[0, :n] = lb
        qb.ub[0, :n] = ub
        qb.lb[0, n:] = qb.ub[0, n:] = 0.0
        lam_p = torch.from_numpy(np.tile(lam, nd)).to(dev)
        qb.p_scale = 2.0 * lam_p
        self.qb = qb
        self.mu_p = torch.zeros((B, ld), dtype=torch.float64, device=dev)
        self.dg_c = torch.zeros((nd, ld), dtype=torch.float64, device=dev)   # diag(Xc'Xc) per date
        self.lr = engine.LowRank(panel, self.rp_d, self.tp_d, mu=self.mu_p,
                                 w_scale=1.0 / (self.tp_d.to(torch.float64) - 1.0),
                                 dg=torch.zeros((B, ld), dtype=torch.float64, device=dev))
        full = bool(nd) and bool((tlen == rows.shape[1]).all())
        if factor == "auto":
            factor = "eig" if L >= EIG_MIN_PER_DATE else "chol"
        self.use_eig = factor == "eig" and full and engine.lowrank_shape_ok(n, rows.shape[1], qb.mg)
        self.k_ld = k_ld
        self.pdate = torch.arange(nd, dtype=torch.int32, device=dev).repeat_interleave(L)
        self.gp = engine.GroupPlan(rows_p, tlen_p, dev, gmax=gmax) if (group and B) else None
        # the ADMM's own groups: the risk aversions of a date (up to 64 per group) on one window
        # and one q = -mu_d, two chip-wide launches per iteration (engine.SweepPlan, admm_sweep.hip)
        self.sp = engine.SweepPlan([L] * nd, dev, q_shared=True) if (group and B) else None
        self.settings = settings if settings is not None else engine.Settings.from_params(SWEEP_SETTINGS)
        self.ws = ws if ws is not None else engine.Workspace(qb, dense=False)

    def solve(self, events: list | None = None):
        """One pass over this rank's grid; returns (BatchResult, meta)."""
        tl = engine._Timeline(events)
        pan, L = self.panel, self.L
        if self.B == 0:   # more ranks than dates: an empty block (the rank still joins gather())
            ws = self.ws
            res = engine.BatchResult(x=ws.x[:, :self.n], y=ws.y[:, :1], z_box=ws.y[:, :self.n], status=ws.status,
                                     iters=ws.iters, out=ws.out)
            return res, {"dates": 0, "lambdas": self.lam, "date_range": (self.lo, self.hi), "rank": self.rank,
                         "world": self.world, "qb": self.qb, "lr": self.lr, "capacitance": "", "factor": "",
                         "grouped": False, "ngroups": 0, "factorizations": 0}

        def moments():
            pan.window_means(self.r_d, self.t_d, out=self.mu_c)
            if self.geometric:
                pan.window_means(self.r_d, self.t_d, geometric=True, out=self.mu_q)
            torch.neg(self.mu_q.repeat_interleave(L, dim=0), out=self.qb.q)
            self.mu_p.copy_(self.mu_c.repeat_interleave(L, dim=0))
            # diag(Xc'Xc) once per DATE (its window is every lambda's), then repeated to the
            # problems: one window pass per date instead of one per (date, lambda)
            pan.window_sumsq(self.r_d, self.t_d, self.mu_c, out=self.dg_c)
            self.lr.dg.copy_(self.dg_c.repeat_interleave(L, dim=0))
        tl("moments", moments)
        eig = None
        if self.use_eig:
            eig = tl("eig", lambda: engine.EigCap(pan, self.r_d, self.t_d, self.mu_c, self.qb, self.pdate, self.k_ld,
                                                  backend=self.eig_backend))
        res = engine.solve_lowrank(self.qb, self.lr, self.settings, ws=self.ws, groups=self.gp, events=events,
                                   eig=eig, sweep=self.sp)
        gp = self.gp
        meta = {"dates": self.nd, "lambdas": self.lam, "grouped": gp is not None and gp.ok,
                "ngroups": None if gp is None else gp.ngroups, "capacitance": res.capacitance,
                "factor": "eig" if eig is not None else "chol",
                # factorisations: one eigendecomposition per date (eig) or one Cholesky per
                # problem and per adaptive-rho change (chol; the eig form re-forms instead)
                "factorizations": self.nd if eig is not None else
                ((gp.ngroups if res.capacitance == "group" else self.B) + res.refactors),
                "date_range": (self.lo, self.hi), "rank": self.rank, "world": self.world,
                # the batch as solved (certificates: workloads.window_certificate)
                "qb": self.qb, "lr": self.lr}
        return res, meta

    def gather(self, res: engine.BatchResult, dist) -> tuple:
        """All-gather every rank's (dates x lambdas) block of weights, status and objective
        (one collective over the date-sharded panels; RCCL on GPUs, gloo on CPU).  Returns
        numpy (X [nd_total * L, n], status [nd_total * L], obj [nd_total * L]), date-major."""
        from .backtest import gather_blocks
        L, n = self.L, self.n
        blk = torch.cat([res.x[:, :n].reshape(self.nd, L * n), res.status.to(torch.float64).reshape(self.nd, L),
                         res.obj.reshape(self.nd, L)], 1)
        full = gather_blocks(blk, self.nd_total, self.world, dist)
        X = full[:, :L * n].reshape(-1, n)
        st = full[:, L * n:L * n + L].reshape(-1).astype(np.int32)
        obj = full[:, L * n + L:].reshape(-1)
        return X, st, obj


def mean_variance_sweep(panel: engine.Panel, rows, tlen, lambdas, lb=0.0, ub=1.0, budget=1.0,
                        geometric=True, settings: engine.Settings | None = None, group=True,
                        factor: str = "auto", gmax: int = engine.GROUP_MAX_DATES,
                        events: list | None = None, ws: "engine.Workspace | None" = None,
                        eig_backend: str = "rocsolver", rank: int = 0, world: int = 1):
    """Solve min lam x'Sigma_d x - mu_d'x  s.t. 1'x = budget, lb <= x <= ub for every
    rebalance window (rows, tlen: host arrays of engine.window_rows) and every lam
    (``rank`` / ``world``: this rank's contiguous block of dates, all lambdas; see
    MeanVarianceSweep).

    Returns (BatchResult, meta): local problem p = (d - lo) * len(lambdas) + j is (date d,
    lambdas[j]), (lo, hi) = meta['date_range']."""
    sw = MeanVarianceSweep(panel, rows, tlen, lambdas, lb=lb, ub=ub, budget=budget, geometric=geometric,
                           settings=settings, group=group, factor=factor, gmax=gmax, ws=ws,
                           eig_backend=eig_backend, rank=rank, world=world)
    return sw.solve(events)
