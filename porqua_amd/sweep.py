"""Risk-aversion x date grid of mean-variance QPs on the window path (BASELINE.json configs[4]).

For rebalance date d and risk aversion lam the reference's MeanVariance objective is
P = 2 lam Sigma_d, q = -mu_d (src/optimization.py:168-174; mu from
MeanEstimator.estimate_geometric, src/mean_estimation.py:39-48), solved per date by
QuadraticProgram.solve (src/qp_problems.py:184-216).  Here every (date, lam) pair is one
problem of a single batch, date-major: all problems of a date share its window rows, so
the grouped low-rank ADMM (engine.GroupPlan with identical windows) streams those rows
once per iteration for up to 16 risk aversions.  Nothing n x n is formed.

Factor once per date (``factor='eig'``; SURVEY.md §8(e) "keep all lambda of a date on one
rank so the factorisation is shared"): the capacitance of problem (d, lam) is
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


def mean_variance_sweep(panel: engine.Panel, rows, tlen, lambdas, lb=0.0, ub=1.0, budget=1.0,
                        geometric=True, settings: engine.Settings | None = None, group=True,
                        factor: str = "auto", gmax: int = engine.GROUP_MAX_DATES,
                        events: list | None = None, ws: "engine.Workspace | None" = None,
                        eig_backend: str = "rocsolver"):
    """Solve min lam x'Sigma_d x - mu_d'x  s.t. 1'x = budget, lb <= x <= ub for every
    rebalance window (rows, tlen: host arrays of engine.window_rows) and every lam.

    Returns (BatchResult, meta): problem p = d * len(lambdas) + j is (date d, lambdas[j])."""
    if factor not in ("auto", "eig", "chol"):
        raise ValueError("mean_variance_sweep: factor must be 'auto', 'eig' or 'chol'")
    rows = np.asarray(rows, dtype=np.int32)
    tlen = np.asarray(tlen, dtype=np.int32)
    lam = np.asarray(lambdas, dtype=np.float64).reshape(-1)
    nd, L, n = len(tlen), len(lam), panel.n
    dev = panel.device
    tl = engine._Timeline(events)
    r_d, t_d = panel.rows_to_device(rows, tlen)
    mu_c = panel.window_means(r_d, t_d)                               # centring of Sigma
    mu_q = panel.window_means(r_d, t_d, geometric=geometric) if geometric else mu_c
    rows_p = np.repeat(rows, L, axis=0)
    tlen_p = np.repeat(tlen, L)
    rp_d, tp_d = panel.rows_to_device(rows_p, tlen_p)
    B = nd * L
    qb = engine.QPBatch(n, B, 1, device=dev, P=torch.empty(0, dtype=torch.float64, device=dev))
    qb.P = None
    qb.Cg[0, 0, :n] = 1.0
    qb.lg[0, 0] = qb.ug[0, 0] = float(budget)
    qb.lb[0, :n] = lb
    qb.ub[0, :n] = ub
    qb.lb[0, n:] = qb.ub[0, n:] = 0.0
    lam_p = torch.from_numpy(np.tile(lam, nd)).to(dev)
    qb.q = -mu_q.repeat_interleave(L, dim=0).contiguous()
    qb.p_scale = 2.0 * lam_p
    mu_p = mu_c.repeat_interleave(L, dim=0).contiguous()
    lr = engine.LowRank(panel, rp_d, tp_d, mu=mu_p, w_scale=1.0 / (tp_d.to(torch.float64) - 1.0))
    eig = None
    full = bool((tlen == rows.shape[1]).all())
    if factor == "auto":
        factor = "eig" if L >= EIG_MIN_PER_DATE else "chol"
    if factor == "eig" and full and engine.lowrank_shape_ok(n, rows.shape[1], qb.mg):
        k_ld = engine.round_up(rows.shape[1] + qb.mg, 64)
        pdate = torch.arange(nd, dtype=torch.int32, device=dev).repeat_interleave(L)
        eig = tl("eig", lambda: engine.EigCap(panel, r_d, t_d, mu_c, qb, pdate, k_ld, backend=eig_backend))
    gp = engine.GroupPlan(rows_p, tlen_p, dev, gmax=gmax) if group else None
    if settings is None:
        settings = engine.Settings(rho0_qrel=SWEEP_RHO0_QREL)
    res = engine.solve_lowrank(qb, lr, settings, ws=ws, groups=gp, events=events, eig=eig)
    meta = {"dates": nd, "lambdas": lam, "grouped": gp is not None and gp.ok,
            "ngroups": None if gp is None else gp.ngroups, "capacitance": res.capacitance,
            "factor": "eig" if eig is not None else "chol",
            # factorisations: one eigendecomposition per date (eig) or one Cholesky per
            # problem and per adaptive-rho change (chol; the eig form re-forms instead)
            "factorizations": nd if eig is not None else
            ((gp.ngroups if res.capacitance == "group" else B) + res.refactors),
            # the batch as solved (certificates: workloads.window_certificate)
            "qb": qb, "lr": lr}
    return res, meta
