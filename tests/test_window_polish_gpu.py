"""Window-form polish (pq_polish_w_batched): the low-rank path never reads an n x n P --
P_FF is formed from the free columns of the window, every P x from two window passes.
Checked against the oracle IPM (oracle/qp_ipm.py) beyond the n <= 1024 LDS limit of the
dense kernels, and on free sets larger than the first compact scratch (relaunch path)."""
import numpy as np
import pytest
import torch

from oracle.qp_ipm import solve_qp
from oracle.ref_pipeline import cov_pearson
from porqua_amd import _lib, engine
from porqua_amd.synthetic import factor_panel

pytestmark = pytest.mark.gpu


def _mv_batch(device, n, T, ends, ub, shrink, D=None):
    D = D or (max(ends) + 1)
    dates, R, y, sec = factor_panel(D, n)
    rows, tlen = engine.window_rows(dates, dates[ends], T)
    pan = engine.Panel(R, y, device=device)
    r_d, t_d = pan.rows_to_device(rows, tlen)
    B = len(ends)
    qb = engine.QPBatch.from_dense(np.zeros((1, n, n)), np.zeros((1, n)), A=np.ones((1, n)), b=np.ones(1),
                                   lb=np.zeros(n), ub=np.full(n, ub), device=device)
    qb.batch = B
    qb.P = None          # the window path never reads P
    qb.q = torch.zeros((B, qb.ld), dtype=torch.float64, device=device)
    qb.p_scale = torch.full((B,), 2.0, dtype=torch.float64, device=device)
    mu = pan.window_means(r_d, t_d)
    lr = engine.LowRank(pan, r_d, t_d, mu=mu, w_scale=1.0 / (t_d.to(torch.float64) - 1.0))
    if shrink:
        qb.p_diag = 2.0 * shrink * lr.dg[:, :n].mean(dim=1) / (t_d.to(torch.float64) - 1.0)
    return R, rows, tlen, qb, lr


def _oracle(R, e, T, n, ub, shrink):
    S = cov_pearson(R[e - T + 1:e + 1])
    P = 2 * S + (2 * shrink * np.mean(np.diag(S)) * np.eye(n) if shrink else 0)
    o = solve_qp(P, np.zeros(n), A=np.ones((1, n)), b=np.ones(1), lb=np.zeros(n), ub=np.full(n, ub))
    return P, o


def test_window_polish_n2000_grouped_vs_oracle(device):
    """n = 2000 > 1024 (dense kernels' LDS limit): grouped low-rank ADMM + window polish."""
    n, T, ub, shrink = 2000, 252, 0.05, 0.05
    ends = list(range(300, 308))
    R, rows, tlen, qb, lr = _mv_batch(device, n, T, ends, ub, shrink)
    gp = engine.GroupPlan(rows, tlen, device)
    ws = engine.Workspace(qb, dense=False)
    assert engine.grouped_applicable(qb, lr, gp, ws)
    res = engine.solve_lowrank(qb, lr, ws=ws, groups=gp)
    x = res.x.cpu().numpy()
    assert np.all(res.status.cpu().numpy() == _lib.PQ_SOLVED)
    assert np.abs(x.sum(1) - 1).max() < 1e-9 and x.min() > -1e-9 and x.max() < ub + 1e-9
    for i in (0, len(ends) - 1):
        P, o = _oracle(R, ends[i], T, n, ub, shrink)
        assert np.abs(x[i] - o.x).max() < 1e-5
        obj = 0.5 * x[i] @ P @ x[i]
        assert abs(obj - o.obj) <= 1e-6 * abs(o.obj)
        assert abs(res.obj[i].item() - obj) <= 1e-9 * abs(obj)


def test_window_polish_relaunch_large_free_set(device):
    """A free set larger than the first compact scratch (ldk = 64 here) goes through the
    relaunch with ldk = min(ld, 1024) and still reaches the oracle optimum."""
    n, T, ub, shrink = 400, 120, 1.0, 2.0
    ends = [200, 260, 333]
    R, rows, tlen, qb, lr = _mv_batch(device, n, T, ends, ub, shrink)
    ws = engine.Workspace(qb, dense=False, kcap=64)
    assert ws.ldk == 64
    res = engine.solve_lowrank(qb, lr, ws=ws)
    x = res.x.cpu().numpy()
    out = res.out.cpu().numpy()
    assert np.all(res.status.cpu().numpy() == _lib.PQ_SOLVED)
    assert out[:, _lib.PQ_OUT_NFREE].min() > 64          # every problem needed the relaunch
    for i, e in enumerate(ends):
        P, o = _oracle(R, e, T, n, ub, shrink)
        assert np.abs(x[i] - o.x).max() < 1e-5
        assert abs(0.5 * x[i] @ P @ x[i] - o.obj) <= 1e-6 * abs(o.obj)
