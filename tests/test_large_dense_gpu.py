"""The per-QP drop-in beyond 1024 assets: QuadraticProgram.solve is the
reference's only solver dispatch (src/qp_problems.py:184-216) and the serial Backtest.run calls
it once per date (src/backtest.py:185-199).  Dense QPs with n > 1024 go to the device IPM on
K2L (pq_factor_large: multi-workgroup blocked Cholesky + inverse on FP64 MFMA).

* K2L against numpy: the factor L L' = K and the inverse K^-1 K = I, padding (n not a multiple
  of 64), a subset launch (idx) and the non-PD flag (info / PQ_NON_CONVEX).
* A dense n = 2000 QP (porqua_amd.synthetic.dense_qp: shrunk covariance, budget, box, group
  caps) through QuadraticProgram.solve(solver_name='mi355x') against the committed oracle
  optimum (tools/capture_dense_large.py -> tests/golden/dense_n2000_oracle.npz).
* The serial Backtest.run (settings batched=False) of config 4's problem -- n = 3000 LS
  tracking with budget, long-only box and 20 sector caps -- on 3 dates, against the oracle
  objectives of tests/golden/config4f_oracle.npz (the optimum keeps all 3000 weights free on a
  rank-252 P, so only the objective is defined)."""
import ctypes

import numpy as np
import pandas as pd
import pytest
import torch

from porqua_amd import _lib, engine
from porqua_amd.synthetic import dense_qp, factor_panel
from tests.conftest import load_golden

pytestmark = pytest.mark.gpu


def _factor_large(mats, invert, idx=None):
    B, n, _ = mats.shape
    qb = engine.QPBatch(n, B, 0, device=torch.device("cuda", 0), has_box=False)
    qb.P[:, :n, :n] = torch.from_numpy(mats).to(qb.device)
    ws = engine.Workspace(qb)
    s = engine.Settings(sigma=0.0).to_c()
    pb, st = qb.c_struct(), ws.c_struct()
    scratch = torch.empty((B, qb.ld, qb.ld), dtype=torch.float64, device=qb.device)
    it = None if idx is None else torch.tensor(idx, dtype=torch.int32, device=qb.device)
    _lib.check(_lib.load().pq_factor_large(ctypes.byref(pb), ctypes.byref(st), None if it is None else it.data_ptr(),
                                           0 if it is None else len(idx), ctypes.byref(s), invert,
                                           scratch.data_ptr(), scratch.stride(0), engine._stream()), "pq_factor_large")
    torch.cuda.synchronize()
    return ws.K[:, :n, :n].cpu().numpy(), ws.info.cpu().numpy(), ws.status.cpu().numpy()


@pytest.mark.parametrize("n", [1100, 2048])
def test_factor_large_cholesky_and_inverse(device, n):
    rng = np.random.default_rng(n)
    M = rng.normal(size=(2, n, n))
    A = M @ M.transpose(0, 2, 1) / n + np.eye(n)
    L, info, _ = _factor_large(A, 0)
    assert np.all(info == 0)
    for b in range(2):
        Lb = np.tril(L[b])
        assert np.abs(Lb @ Lb.T - A[b]).max() <= 1e-12 * np.abs(A[b]).max()
    Ki, info, _ = _factor_large(A, 2)
    assert np.all(info == 0)
    for b in range(2):
        assert np.abs(Ki[b] @ A[b] - np.eye(n)).max() <= 1e-10
        assert np.abs(Ki[b] - Ki[b].T).max() <= 1e-13 * np.abs(Ki[b]).max()
    # subset launch: only problem 1 is factored
    Ki1, info1, _ = _factor_large(A, 2, idx=[1])
    assert np.abs(Ki1[1] @ A[1] - np.eye(n)).max() <= 1e-10


def test_factor_large_flags_non_pd(device):
    n = 1500
    rng = np.random.default_rng(5)
    Q, _ = np.linalg.qr(rng.normal(size=(n, n)))
    ev = np.linspace(1.0, 2.0, n)
    ev[700] = -0.5
    A = (Q * ev) @ Q.T
    _, info, status = _factor_large(A[None], 2)
    assert info[0] > 0 and status[0] == _lib.PQ_NON_CONVEX


def test_dense_quadratic_program_n2000_matches_oracle(device):
    from porqua_amd.qp_problems import QuadraticProgram
    pr = dense_qp(2000)
    gold = load_golden("dense_n2000_oracle")
    qp = QuadraticProgram(**pr, params={"solver_name": "mi355x"})
    qp.solve()
    sol = qp["solution"]
    assert sol.found
    x = sol.x
    assert np.abs(x - gold["x"]).max() <= 1e-5, np.abs(x - gold["x"]).max()
    obj = qp.objective_value(x, with_const=False)
    assert abs(obj - float(gold["obj"])) <= 1e-6 * abs(float(gold["obj"]))
    assert abs(sol.obj - obj) <= 1e-9 * abs(obj)
    assert abs(x.sum() - 1) <= 1e-7 and x.min() >= -1e-7 and x.max() <= 0.05 + 1e-7
    assert (pr["G"] @ x - pr["h"]).max() <= 1e-7
    # qpsolvers' residuals of the returned point (src/helper_functions.py:69-80)
    assert sol.primal_residual() <= 1e-7
    assert sol.dual_residual() <= 1e-7 * max(1.0, np.abs(pr["q"]).max())


def bibfn_sector_caps(bs, rebdate, **kw):
    """20 sector caps G x <= cap as linear '<=' rows (Constraints.add_linear, src/constraints.py:66-94)."""
    G = kw["G"]
    bs.optimization.constraints.add_linear(Amat=G, sense=pd.Series(["<="] * len(G), index=G.index),
                                           rhs=pd.Series(kw["cap"], index=G.index))


def test_serial_backtest_n3000_ls_tracking_matches_oracle(device):
    from porqua_amd.backtest import Backtest, BacktestService
    from porqua_amd.builders import (OptimizationItemBuilder, SelectionItemBuilder, bibfn_box_constraints,
                                     bibfn_bm_series, bibfn_budget_constraint, bibfn_return_series,
                                     bibfn_selection_data)
    from porqua_amd.optimization import LeastSquares
    gold = load_golden("config4f_oracle")
    n, T, ns, cap = 3000, 252, 20, float(gold["cap"])
    ends = [int(e) for e in gold["ends"][:3]]
    dates, R, y, sec = factor_panel(10000, n, n_sectors=ns)
    rows = slice(0, max(ends) + 1)
    idx = pd.DatetimeIndex(dates[rows])
    cols = [f"a{i:04d}" for i in range(n)]
    X = pd.DataFrame(R[rows], index=idx, columns=cols)
    Y = pd.DataFrame({"bm": y[rows]}, index=idx)
    G = pd.DataFrame(np.stack([(sec == g).astype(float) for g in range(ns)]), columns=cols,
                     index=[f"sector{g}" for g in range(ns)])
    svc = BacktestService(
        data={"return_series": X, "bm_series": Y},
        selection_item_builders={"data": SelectionItemBuilder(bibfn=bibfn_selection_data)},
        optimization_item_builders={
            "return_series": OptimizationItemBuilder(bibfn=bibfn_return_series, width=T),
            "bm_series": OptimizationItemBuilder(bibfn=bibfn_bm_series, width=T),
            "budget_constraint": OptimizationItemBuilder(bibfn=bibfn_budget_constraint, budget=1),
            "box_constraints": OptimizationItemBuilder(bibfn=bibfn_box_constraints, box_type="LongOnly"),
            "sector_caps": OptimizationItemBuilder(bibfn=bibfn_sector_caps, G=G, cap=cap)},
        optimization=LeastSquares(solver_name="mi355x"), rebdates=[str(d.date()) for d in idx[ends]],
        quiet=True, batched=False)
    bt = Backtest()
    bt.run(svc)
    W = bt.strategy.get_weights_df().to_numpy(dtype=float)
    assert W.shape == (3, n)
    for i, e in enumerate(ends):
        w = W[i]
        assert abs(w.sum() - 1) <= 1e-7 and w.min() >= -1e-7 and w.max() <= 1 + 1e-7
        assert (G.to_numpy() @ w).max() <= cap + 1e-7
        v = R[e - T + 1:e + 1] @ w
        obj = v @ v - 2 * (y[e - T + 1:e + 1] @ v)
        assert abs(obj - gold["obj"][i]) <= 1e-6 * abs(gold["obj"][i]), (e, obj, gold["obj"][i])
