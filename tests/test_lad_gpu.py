"""LAD (src/optimization.py:263-345) on the device: the reference's LP solved by the batched
IPM of porqua_amd/lad.py (w-space normal equations factored on K2), checked against the
golden LPs captured from the reference's own backtest (tools/capture_lad.py) and HiGHS
(oracle/lad.py).  An LP's optimal value is unique; weights are compared only through it."""
import numpy as np
import pandas as pd
import pytest

from oracle import lad as olad
from porqua_amd.backtest import Backtest
from porqua_amd.constraints import Constraints
from porqua_amd.optimization import LAD
from porqua_amd.optimization_data import OptimizationData
from tests.conftest import load_golden
from tests.test_api_gpu import _service, msci

pytestmark = pytest.mark.gpu


def _check_weights(W, g, X, y, box_ub, use_level, use_log, tol=1e-7):
    dates = X.index.values.astype("datetime64[D]")
    R, yv = X.to_numpy(), y.to_numpy()[:, 0]
    for i, rb in enumerate(g["rebdates"]):
        e = np.searchsorted(dates, np.datetime64(str(rb)), side="right")
        rows = np.arange(e - int(g["width"]), e)
        Xl = olad.levels(R[rows], use_level, use_log)
        yl = olad.levels(yv[rows], use_level, use_log)
        w = W[i]
        f = np.abs(yl - Xl @ w).sum()
        assert abs(f - g["obj"][i]) <= tol * g["obj"][i], (i, f, g["obj"][i])
        assert abs(w.sum() - 1) < 1e-9 and w.min() > -1e-9 and w.max() < box_ub + 1e-9


@pytest.mark.parametrize("tag,kw,box", [("msci_lad", {}, {}),
                                        ("msci_lad_ret", {"use_level": False}, {"upper": 0.3})])
def test_lad_backtest_batched_matches_golden(device, tag, kw, box):
    X, y = msci()
    g = load_golden(tag)
    rebdates = [str(d) for d in g["rebdates"]]
    bt = Backtest()
    bt.run(_service(LAD(solver_name="mi355x", **kw), X, y, rebdates, box))
    assert bt.stats["path"] == "lp-ipm" and bt.stats["solved"] == len(rebdates)
    W = bt.strategy.get_weights_df().to_numpy(dtype=float)
    _check_weights(W, g, X, y, box.get("upper", 1.0), kw.get("use_level", True), True)


def test_lad_serial_equals_batched_value(device):
    X, y = msci()
    g = load_golden("msci_lad_ret")
    rebdates = [str(d) for d in g["rebdates"][:6]]
    bs = _service(LAD(solver_name="mi355x", use_level=False), X, y, rebdates, {"upper": 0.3})
    bs.settings["batched"] = False
    bt = Backtest()
    bt.run(bs)
    W = bt.strategy.get_weights_df().to_numpy(dtype=float)
    sub = {k: g[k][:6] if k in ("rebdates", "obj") else g[k] for k in ("rebdates", "obj", "width")}
    _check_weights(W, sub, X, y, 0.3, False, True)


def test_lad_solve_with_group_caps_matches_highs(device):
    """LAD.solve (the reference API) with budget, box and two '<=' group rows, on windows
    with and without a box; value vs HiGHS on the reference's LP."""
    X, y = msci()
    n = X.shape[1]
    rng = np.random.default_rng(3)
    groups = [(rng.random(n) < 0.4).astype(float) for _ in range(2)]
    for end, boxed in [(900, True), (1700, True), (2500, False)]:
        Xw, yw = X.iloc[end - 252:end], y.iloc[end - 252:end]
        cons = Constraints(selection=X.columns)
        cons.add_budget()
        if boxed:
            cons.add_box("LongOnly", upper=0.25)
        for gv in groups:
            cons.add_linear(None, pd.Series(gv, index=X.columns), "<=", 0.3)
        opt = LAD(solver_name="mi355x", constraints=cons)
        opt.set_objective(OptimizationData(return_series=Xw, bm_series=yw))
        assert opt.solve() is True
        w = pd.Series(opt.results["weights"]).to_numpy(dtype=float)
        Xl = olad.levels(Xw.to_numpy())
        yl = olad.levels(yw.to_numpy()[:, 0])
        GhAb = cons.to_GhAb()
        lb = cons.box["lower"].to_numpy(dtype=float) if boxed else None
        ub = cons.box["upper"].to_numpy(dtype=float) if boxed else None
        q, A, b, G, h, lbt, ubt = olad.lad_lp(Xl, yl, A=GhAb["A"], b=GhAb["b"], G=GhAb["G"], h=GhAb["h"],
                                              lb=lb, ub=ub)
        ref = olad.solve_lp(q, A, b, lbt, ubt, G, h)
        f = np.abs(yl - Xl @ w).sum()
        assert abs(f - ref.fun) <= 1e-7 * ref.fun, (end, f, ref.fun)
        assert abs(w.sum() - 1) < 1e-9 and (GhAb["G"] @ w <= GhAb["h"] + 1e-9).all()


def test_lad_backtest_n300_matches_highs(device):
    """n = 300 > window: 24 daily windows of the synthetic factor panel in one batch."""
    from porqua_amd.synthetic import factor_panel
    n, D, width = 300, 320, 252
    dates, R, yv, _ = factor_panel(D, n, seed=5)
    idx = pd.DatetimeIndex(dates)
    X = pd.DataFrame(R, index=idx, columns=[f"a{i}" for i in range(n)])
    y = pd.DataFrame({"bm": yv}, index=idx)
    rebdates = [str(d.date()) for d in idx[width + 10:width + 34]]
    bt = Backtest()
    bt.run(_service(LAD(solver_name="mi355x"), X, y, rebdates, {"upper": 0.05}, width=width))
    assert bt.stats["path"] == "lp-ipm" and bt.stats["solved"] == len(rebdates)
    W = bt.strategy.get_weights_df().to_numpy(dtype=float)
    for i in (0, 13, 23):
        e = idx.get_loc(pd.Timestamp(rebdates[i])) + 1
        Xl, yl = olad.levels(R[e - width:e]), olad.levels(yv[e - width:e])
        q, A, b, G, h, lb, ub = olad.lad_lp(Xl, yl, A=np.ones(n), b=np.array(1.0), lb=np.zeros(n),
                                            ub=np.full(n, 0.05))
        ref = olad.solve_lp(q, A, b, lb, ub)
        f = np.abs(yl - Xl @ W[i]).sum()
        assert abs(f - ref.fun) <= 1e-7 * ref.fun, (i, f, ref.fun)
        assert abs(W[i].sum() - 1) < 1e-9 and W[i].min() > -1e-9 and W[i].max() < 0.05 + 1e-9


@pytest.mark.parametrize("n,k,strided", [(1000, 1, True), (300, 3, False), (7, 4, False), (64, 2, True)])
def test_lad_mv_kernel_matches_torch(device, n, k, strided):
    """pq_lad_mv_batched (M V and S - M V) against a torch FP64 product."""
    import torch
    from porqua_amd.lad import _mv
    g = torch.Generator(device="cpu").manual_seed(n + k)
    B = 5
    ld = ((n + 63) // 64) * 64 if strided else n
    Mfull = torch.randn(B, ld, ld, generator=g, dtype=torch.float64).to("cuda")
    M = Mfull[:, :n, :n]
    V = torch.randn(B, n, k, generator=g, dtype=torch.float64).to("cuda")
    S = torch.randn(B, n, k, generator=g, dtype=torch.float64).to("cuda")
    ref = torch.bmm(M, V)
    out = _mv(M, V)
    assert torch.allclose(out, ref, rtol=1e-12, atol=1e-12)
    out2 = _mv(M, V, S)
    assert torch.allclose(out2, S - ref, rtol=1e-12, atol=1e-12)


@pytest.mark.parametrize("B,k,n,diag", [(3, 252, 1000, False), (2, 70, 131, True), (4, 64, 64, False)])
def test_wgram_kernel_matches_torch(device, B, k, n, diag):
    """pq_wgram_batched: M = diag(d) + diag(r) U diag(w) U' diag(r) (lower tiles, identity
    padding to k_ld) against a torch FP64 product."""
    import torch
    from porqua_amd import _lib, engine
    g = torch.Generator(device="cpu").manual_seed(k + n)
    U = torch.randn(B, k, n + 3, generator=g, dtype=torch.float64)[:, :, :n].to("cuda")   # row stride > n
    w = torch.rand(B, n, generator=g, dtype=torch.float64).to("cuda") + 0.1
    r = torch.rand(B, k, generator=g, dtype=torch.float64).to("cuda") + 0.5
    d = (torch.rand(B, k, generator=g, dtype=torch.float64).to("cuda") + 1.0) if diag else None
    k_ld = (k + 63) // 64 * 64
    M = torch.full((B, k_ld, k_ld), np.nan, dtype=torch.float64, device="cuda")
    lib = _lib.load()
    _lib.check(lib.pq_wgram_batched(U.data_ptr(), U.stride(1), U.stride(0), k, n, B, w.data_ptr(), w.stride(0),
                                    r.data_ptr(), r.stride(0), None if d is None else d.data_ptr(),
                                    0 if d is None else d.stride(0), M.data_ptr(), k_ld, M.stride(0),
                                    engine._stream()), "pq_wgram_batched")
    S = r.unsqueeze(2) * U
    ref = torch.bmm(S * w.unsqueeze(1), S.transpose(1, 2))
    ref.diagonal(dim1=1, dim2=2).add_(1.0 if d is None else d)
    low = torch.tril(torch.ones(k, k, dtype=torch.bool, device="cuda"))
    got = M[:, :k, :k]
    assert torch.allclose(got[:, low], ref[:, low], rtol=1e-12, atol=1e-12 * float(ref.abs().max()))
    pad = M[:, k:, k:]
    if k < k_ld:
        eye = torch.eye(k_ld - k, dtype=torch.float64, device="cuda")
        assert torch.equal(torch.tril(pad), eye.expand_as(pad))


def test_normal_m_solve_matches_dense(device):
    """woodbury.NormalM: M^-1 g and M y against the dense M = U diag(w) U' + diag(d), with
    IPM-like scaling spreads (w over 1e-6 .. 1e6, d over 1e-4 .. 1e4, one row d = 0): the
    refined solve's backward error is at the rounding level."""
    import torch
    from porqua_amd.woodbury import NormalM
    g = torch.Generator(device="cpu").manual_seed(7)
    B, k, n = 3, 121, 400
    U = (0.01 * torch.randn(B, k, n, generator=g, dtype=torch.float64)).to("cuda")
    w = torch.exp(torch.empty(B, n, dtype=torch.float64).uniform_(-14, 14, generator=g)).to("cuda")
    d = torch.exp(torch.empty(B, k, dtype=torch.float64).uniform_(-9, 9, generator=g)).to("cuda")
    d[:, 0] = 0.0                                         # an equality row
    R = torch.randn(B, k, 2, generator=g, dtype=torch.float64).to("cuda")
    nm = NormalM(U.contiguous())
    assert not bool(nm.factor(w, d).any())
    M = torch.bmm(U * w.unsqueeze(1), U.transpose(1, 2))
    M.diagonal(dim1=1, dim2=2).add_(d)
    Y = nm.solve(R)
    res = (R - torch.bmm(M, Y)).abs().amax() / (torch.bmm(M.abs(), Y.abs()).amax() + R.abs().amax())
    assert float(res) < 1e-12
    MY = torch.bmm(M, Y)
    assert float((nm.apply(Y) - MY).abs().amax() / torch.bmm(M.abs(), Y.abs()).amax()) < 1e-13
