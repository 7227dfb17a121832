"""Risk-aversion x date grid of mean-variance QPs on the window path (BASELINE.json configs[4]).

For rebalance date d and risk aversion lam the reference's MeanVariance objective is
P = 2 lam Sigma_d, q = -mu_d (src/optimization.py:168-174; mu from
MeanEstimator.estimate_geometric, src/mean_estimation.py:39-48), solved per date by
QuadraticProgram.solve (src/qp_problems.py:184-216).  Here every (date, lam) pair is one
problem of a single batch, date-major: all problems of a date share its window rows, so
the grouped low-rank ADMM (engine.GroupPlan with identical windows) streams those rows
once per iteration for up to 16 risk aversions.  Nothing n x n is formed.
"""
from __future__ import annotations

import numpy as np
import torch

from . import engine


def mean_variance_sweep(panel: engine.Panel, rows, tlen, lambdas, lb=0.0, ub=1.0, budget=1.0,
                        geometric=True, settings: engine.Settings | None = None, group=True):
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
    qb.q = -mu_q.repeat_interleave(L, dim=0).contiguous()
    qb.p_scale = torch.from_numpy(np.tile(2.0 * lam, nd)).to(dev)
    mu_p = mu_c.repeat_interleave(L, dim=0).contiguous()
    lr = engine.LowRank(panel, rp_d, tp_d, mu=mu_p, w_scale=1.0 / (tp_d.to(torch.float64) - 1.0))
    gp = engine.GroupPlan(rows_p, tlen_p, dev) if group else None
    res = engine.solve_lowrank(qb, lr, settings, groups=gp)
    meta = {"dates": nd, "lambdas": lam, "grouped": gp is not None and gp.ok,
            "ngroups": None if gp is None else gp.ngroups}
    return res, meta
