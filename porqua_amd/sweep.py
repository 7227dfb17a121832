"""Risk-aversion x date grid of mean-variance QPs on the window path (BASELINE.json configs[4]).

For rebalance date d and risk aversion lam the reference's MeanVariance objective is
P = 2 lam Sigma_d, q = -mu_d (src/optimization.py:168-174; mu from
MeanEstimator.estimate_geometric, src/mean_estimation.py:39-48), solved per date by
QuadraticProgram.solve (src/qp_problems.py:184-216).  Here every (date, lam) pair is one
problem of a single batch, date-major: all problems of a date share its window rows, so
the grouped low-rank ADMM (engine.GroupPlan with identical windows) streams those rows
once per iteration for up to 16 risk aversions.  Nothing n x n is formed.

Factor once per date (``shared_factor=True``, off by default): lam x'Sigma x - mu'x and x'Sigma x -
(mu / lam)'x have the same minimiser, so every problem of a date is given P = 2 Sigma_d and
q = -mu_d / lam: the KKT operator no longer depends on lam, a slide group of one date's risk
aversions shares one capacitance matrix (engine group capacitance: one factorisation per 16
problems instead of one per problem), and the ADMM runs them as a multi-right-hand-side
block.  Objectives and multipliers are scaled back by lam afterwards, so the results are
those of the reference's objective.  Measured (tools/exp_sweep.py, n = 5000, 16 dates x 64
lam): 256 factorisations instead of 1024, but the nearly linear problems (lam <= 0.13, q
dominating) then share one rho with their group and fall through to the eps_retry ADMM
(up to 4000 iterations): 102 QPs/s against 12.7k QPs/s with one capacitance per problem and
a per-problem, |q|-aware rho -- so the per-problem form stays the default.
"""
from __future__ import annotations

import numpy as np
import torch

from . import engine


RHO_BUCKET = 2.0       # shared factorisation: largest rho0 ratio inside one group


def mean_variance_sweep(panel: engine.Panel, rows, tlen, lambdas, lb=0.0, ub=1.0, budget=1.0,
                        geometric=True, settings: engine.Settings | None = None, group=True,
                        shared_factor=False, gmax: int = engine.GROUP_MAX_DATES):
    """Solve min lam x'Sigma_d x - mu_d'x  s.t. 1'x = budget, lb <= x <= ub for every
    rebalance window (rows, tlen: host arrays of engine.window_rows) and every lam.

    Returns (BatchResult, meta): problem p = d * len(lambdas) + j is (date d, lambdas[j])."""
    rows = np.asarray(rows, dtype=np.int32)
    tlen = np.asarray(tlen, dtype=np.int32)
    lam = np.asarray(lambdas, dtype=np.float64).reshape(-1)
    nd, L, n = len(tlen), len(lam), panel.n
    dev = panel.device
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
    if shared_factor:   # P = 2 Sigma_d for every lam, q = -mu_d / lam
        qb.q = (-mu_q.repeat_interleave(L, dim=0) / lam_p[:, None]).contiguous()
        qb.p_scale = torch.full((B,), 2.0, dtype=torch.float64, device=dev)
    else:
        qb.q = -mu_q.repeat_interleave(L, dim=0).contiguous()
        qb.p_scale = 2.0 * lam_p
    mu_p = mu_c.repeat_interleave(L, dim=0).contiguous()
    lr = engine.LowRank(panel, rp_d, tp_d, mu=mu_p, w_scale=1.0 / (tp_d.to(torch.float64) - 1.0))
    breaks = None
    if shared_factor and group:
        # one capacitance per group needs one rho per group: the problems of a date share
        # P = 2 Sigma_d, and rho0 = max(4 mean diag P, 10 |q|_max) (engine.Settings) varies
        # with lam only through q = -mu_d / lam -- so a group holds the risk aversions of one
        # date whose rho0 lie within a factor RHO_BUCKET of each other (bucket breaks here)
        Tw = torch.as_tensor(tlen, dtype=torch.float64, device=dev)
        dg = panel.window_sumsq(r_d, t_d, mu_c)[:, :n]
        pdiag = (2.0 * dg.mean(1) / (Tw - 1.0)).cpu().numpy()
        qmax = mu_q[:, :n].abs().amax(1).cpu().numpy()
        r0 = np.maximum(4.0 * pdiag[:, None], 10.0 * qmax[:, None] / lam[None, :])     # (nd, L)
        bucket = np.floor(np.log(r0 / r0.min(1, keepdims=True)) / np.log(RHO_BUCKET)).astype(np.int64)
        brk = np.ones((nd, L), dtype=bool)
        brk[:, 1:] = bucket[:, 1:] != bucket[:, :-1]
        breaks = brk.reshape(-1)
    gp = engine.GroupPlan(rows_p, tlen_p, dev, gmax=gmax, breaks=breaks) if group else None
    res = engine.solve_lowrank(qb, lr, settings, groups=gp)
    if shared_factor:   # back to lam x'Sigma x - mu'x: objective and multipliers times lam
        res.obj.mul_(lam_p)
        res.y.mul_(lam_p[:, None])
        res.z_box.mul_(lam_p[:, None])
    meta = {"dates": nd, "lambdas": lam, "grouped": gp is not None and gp.ok,
            "ngroups": None if gp is None else gp.ngroups, "capacitance": res.capacitance,
            "shared_factor": shared_factor,
            # capacitance factorisations: one per slide group (group form) or per problem
            "factorizations": (gp.ngroups if res.capacitance == "group" else B) + res.refactors}
    return res, meta
