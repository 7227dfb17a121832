"""Host-side logic of the product package (no GPU needed)."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pandas as pd
import pytest
import torch

from oracle import ref_pipeline as rp
from porqua_amd import _lib, engine
from porqua_amd.backtest import shard_range
from porqua_amd.constraints import Constraints
from porqua_amd.synthetic import business_days, factor_panel
from tests.conftest import ROOT, load_golden


def test_window_rows_match_reference_semantics():
    g = load_golden("msci_panel")
    dates = g["dates"].astype("datetime64[D]")
    reb = dates[300::97]
    rows, tlen = engine.window_rows(dates, reb, 252)
    for b, d in enumerate(reb):
        assert np.array_equal(rows[b, :tlen[b]], rp.window_rows(dates, d, 252))
    # calendars with weekend rows: they are dropped, as src/builders.py:211 does
    cal = np.datetime64("2020-01-01") + np.arange(60)
    rows, tlen = engine.window_rows(cal, cal[[20, 59]], 10)
    for b, d in enumerate(cal[[20, 59]]):
        r = rp.window_rows(cal, d, 10)
        assert np.array_equal(rows[b, :tlen[b]], r) and len(r) < 10
    # a rebalance date before the data starts -> empty window
    rows, tlen = engine.window_rows(cal, [np.datetime64("2019-01-01")], 10)
    assert tlen[0] == 0


def test_slide_plan_groups_overlapping_windows():
    dates, _, _, _ = factor_panel(600, 3)
    # daily: every window is the previous one shifted by one row -> groups of 32
    rows, tlen = engine.window_rows(dates, dates[251:600], 252)
    gs, sh = engine.slide_plan(rows, tlen, group=32)
    assert list(gs[:3]) == [0, 32, 64] and gs[-1] == len(tlen)
    assert np.all(sh[gs[:-1]] <= 1) and np.all(np.delete(sh, gs[:-1]) == 1)
    # monthly stride 21 -> shift 21; beyond smax -> anchors only
    rows, tlen = engine.window_rows(dates, dates[251:600:21], 252)
    gs, sh = engine.slide_plan(rows, tlen)
    assert len(gs) == 2 and np.all(sh[1:] == 21)
    gs, sh = engine.slide_plan(rows, tlen, smax=20)
    assert len(gs) == len(tlen) + 1 and np.all(sh == 0)
    # every slid window really is its predecessor shifted by s rows
    cal = np.datetime64("2020-01-01") + np.arange(400)
    rows, tlen = engine.window_rows(cal, cal[100:160], 30)
    gs, sh = engine.slide_plan(rows, tlen)
    for d in np.flatnonzero(sh):
        T, s = tlen[d], sh[d]
        assert tlen[d - 1] == T and np.array_equal(rows[d, :T - s], rows[d - 1, s:T])
    # ragged (weekend-filtered) windows break groups
    assert len(gs) - 1 > 1 and sh[0] == 0


def test_business_days_and_panel_are_deterministic():
    d = business_days("2005-01-03", 10)
    assert ((d.astype(np.int64) + 3) % 7 < 5).all() and len(d) == 10
    a = factor_panel(50, 7)[1]
    b = factor_panel(50, 7)[1]
    assert np.array_equal(a, b)


def test_shard_range_covers_dates():
    for total in [1, 7, 4749, 10000]:
        for world in [1, 2, 3, 8]:
            parts = [shard_range(total, r, world) for r in range(world)]
            assert parts[0][0] == 0 and parts[-1][1] == total
            assert all(parts[i][1] == parts[i + 1][0] for i in range(world - 1))
            sizes = [e - s for s, e in parts]
            assert max(sizes) - min(sizes) <= 1


def test_qpbatch_layout_cpu():
    rng = np.random.default_rng(0)
    B, n = 3, 70
    P = rng.standard_normal((B, n, n))
    qb = engine.QPBatch.from_dense(P, rng.standard_normal((B, n)), A=np.ones((1, n)), b=np.ones(1),
                                   G=rng.random((2, n)), h=np.ones(2), lb=np.zeros(n), ub=np.ones(n),
                                   device=torch.device("cpu"))
    assert qb.ld == 128 and qb.mg == 3 and qb.shared
    assert np.array_equal(qb.P[:, :n, :n].numpy(), P) and float(qb.P[:, n:, :].abs().sum()) == 0
    assert qb.lg[0, 0] == qb.ug[0, 0] == 1.0 and np.isinf(qb.lg[0, 1].item()) and qb.ug[0, 2] == 1.0
    assert float(qb.lb[0, n:].abs().sum()) == 0 and float(qb.ub[0, n:].abs().sum()) == 0
    cs = qb.c_struct()
    assert cs.n == n and cs.ld == 128 and cs.Cg_stride == 0 and cs.P_stride == 128 * 128
    # per-problem constraints switch to strided storage
    qb2 = engine.QPBatch.from_dense(P, np.zeros((B, n)), A=np.ones((B, 1, n)), b=np.ones((B, 1)),
                                    device=torch.device("cpu"))
    assert not qb2.shared and qb2.c_struct().Cg_stride == qb2.Cg.stride(0)


def test_settings_from_params():
    s = engine.Settings.from_params({"eps_abs": 1e-7, "admm_max_iter": 50, "solver_name": "mi355x"})
    assert s.eps_abs == 1e-7 and s.max_iter == 50 and isinstance(s.max_iter, int)
    c = s.to_c()
    assert abs(c.eps_abs - 1e-7) < 1e-20 and c.max_iter == 50


def test_constraints_mirror_reference_shapes():
    """The reference's own known-answer test (test/tests_quadratic_program.py:28-58)."""
    g = load_golden("msci_panel")
    universe = pd.Index([str(c) for c in g["columns"]])
    c = Constraints(selection=universe)
    c.add_budget()
    c.add_box("LongOnly")
    rng = np.random.default_rng(1)
    c.add_linear(None, pd.Series(rng.random(universe.size), index=universe), "<=", 1)
    c.add_linear(None, pd.Series(rng.random(universe.size), index=universe), ">=", -1)
    c.add_linear(None, pd.Series(rng.random(universe.size), index=universe), "=", 0.5)
    sub = universe[: universe.size // 2]
    c.add_linear(pd.DataFrame(rng.random((3, sub.size)), columns=sub), None, pd.Series(np.repeat("=", 3)),
                 pd.Series(np.ones(3)), None)
    o = c.to_GhAb()
    assert o["G"].shape == (2, universe.size) and o["h"].shape == (2,)
    assert o["A"].shape == (5, universe.size) and o["b"].shape == (5,)
    o = c.to_GhAb(True)
    assert o["G"].shape == (2 + 2 * universe.size, universe.size) and o["h"].shape == (2 + 2 * universe.size,)


def test_constraints_values_match_reference_golden():
    g = load_golden("ghab")
    cols = [f"c{i}" for i in range(24)]
    u = pd.Index(cols)
    c = Constraints(selection=u)
    c.add_budget()
    c.add_box("LongOnly")
    c.add_linear(None, pd.Series(g["a1"], index=u), "<=", 1)
    c.add_linear(None, pd.Series(g["a2"], index=u), ">=", -1)
    c.add_linear(None, pd.Series(g["a3"], index=u), "=", 0.5)
    c.add_linear(pd.DataFrame(g["blk"], columns=u[:12]), None, pd.Series(np.repeat("=", 3)), pd.Series(np.ones(3)), None)
    for lbub, s in [(False, "0"), (True, "1")]:
        o = c.to_GhAb(lbub)
        for k in "GhAb":
            assert np.allclose(o[k], g[k + s])
    c2 = Constraints(selection=u)
    c2.add_budget()
    c2.add_box("LongShort")
    c2.add_linear(None, pd.Series(g["a3"], index=u), "=", 0.5)
    c2.add_linear(pd.DataFrame(g["blk"], columns=u[:12]), None, pd.Series(np.repeat("=", 3)), pd.Series(np.ones(3)), None)
    o = c2.to_GhAb(True)
    assert np.allclose(o["G"], g["G2"]) and np.allclose(o["h"], g["h2"])


def test_library_loads_and_exports_every_header_symbol():
    lib = _lib.load()
    header = open(os.path.join(ROOT, "include", "porqua_hip.h")).read()
    declared = set(re.findall(r"^(?:int|int64_t|const char\*)\s+(pq_\w+)\(", header, flags=re.M))
    assert declared and declared == set(_lib.exported_symbols())
    for name in declared:
        assert hasattr(lib, name)
    assert lib.pq_version() == 100
    # size query (host-only arithmetic, no GPU): dense and window layouts, bad arguments
    n, B, mg = 1000, 7, 1
    ld, mgp = 1024, 8
    dense = B * (8 * (ld * ld + (ld // 64) * 4096) + 16 * ld + 16 * (mgp + ld) + 8 + 12 + 64
                 + 8 * ((9 + mgp) * ld + 512))
    assert lib.pq_workspace_bytes(n, B, mg, 0, 0, 0) == dense
    win = lib.pq_workspace_bytes(n, B, mg, 1, 252, 256)
    assert win == dense - B * 8 * (ld * ld - 256 * 256 + (ld // 64 - 4) * 4096) + \
        B * (8 * (2 * 256 * 256 + 4 * 4096) + 12)
    assert lib.pq_workspace_bytes(0, B, mg, 0, 0, 0) == -1
    nm = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    for name in declared:
        assert re.search(rf"\bT {name}\b", nm), name


def test_ctypes_structs_match_c_layout(tmp_path):
    src = tmp_path / "sz.c"
    src.write_text('#include "porqua_hip.h"\n#include <stdio.h>\n#include <stddef.h>\n'
                   'int main(void){printf("%zu %zu %zu %zu %zu %zu\\n", sizeof(pq_problem), sizeof(pq_state),'
                   ' sizeof(pq_settings), offsetof(pq_problem, lb), offsetof(pq_state, work),'
                   ' offsetof(pq_settings, refine_iters)); return 0;}\n')
    exe = tmp_path / "sz"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    got = list(map(int, subprocess.run([str(exe)], capture_output=True, text=True).stdout.split()))
    exp = [ctypes.sizeof(_lib.PQProblem), ctypes.sizeof(_lib.PQState), ctypes.sizeof(_lib.PQSettings),
           _lib.PQProblem.lb.offset, _lib.PQState.work.offset, _lib.PQSettings.refine_iters.offset]
    assert got == exp


def test_product_path_fails_loudly_without_gpu():
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(_lib.PorquaHipError):
        engine.default_device()
    from porqua_amd.qp_problems import QuadraticProgram
    n = 4
    qp = QuadraticProgram(P=np.eye(n), q=np.zeros(n), A=np.ones((1, n)), b=np.ones(1), lb=np.zeros(n),
                          ub=np.ones(n), params={"solver_name": "mi355x"})
    with pytest.raises(_lib.PorquaHipError):
        qp.solve()
    # more than 64 general rows (device IPM) and LAD (device LP IPM): no CPU fallback either
    big = QuadraticProgram(P=np.eye(n), q=np.zeros(n), G=np.ones((70, n)), h=np.ones(70),
                           params={"solver_name": "mi355x"})
    with pytest.raises(_lib.PorquaHipError):
        big.solve()
    import pandas as pd
    from porqua_amd.constraints import Constraints
    from porqua_amd.optimization import LAD
    from porqua_amd.optimization_data import OptimizationData
    idx = pd.bdate_range("2020-01-01", periods=30)
    X = pd.DataFrame(np.random.default_rng(0).normal(0, 0.01, (30, n)), index=idx, columns=list("abcd"))
    y = pd.DataFrame({"bm": X.mean(1)}, index=idx)
    cons = Constraints(selection=X.columns)
    cons.add_budget()
    lad = LAD(solver_name="mi355x", constraints=cons)
    lad.set_objective(OptimizationData(return_series=X, bm_series=y))
    with pytest.raises(_lib.PorquaHipError):
        lad.solve()


def test_lad_model_qpsolvers_matches_reference_lp():
    """LAD.model_qpsolvers (the non-engine route) builds the reference's LP
    (src/optimization.py:296-336) entry for entry: golden problems from tools/capture_lad.py."""
    import pandas as pd
    from porqua_amd.constraints import Constraints
    from porqua_amd.optimization import LAD
    from porqua_amd.optimization_data import OptimizationData
    from tests.conftest import load_golden
    p = load_golden("msci_panel")
    g = load_golden("msci_lad_ret")
    idx = pd.DatetimeIndex(p["dates"].astype("datetime64[D]"))
    cols = [str(c) for c in p["columns"]]
    X = pd.DataFrame(p["returns"], index=idx, columns=cols)
    y = pd.DataFrame({"bm": p["bm"]}, index=idx)
    for i in (0, 11):
        e = idx.searchsorted(pd.Timestamp(str(g["rebdates"][i])), side="right")
        cons = Constraints(selection=cols)
        cons.add_budget()
        cons.add_box("LongOnly", upper=0.3)
        lad = LAD(solver_name="cvxopt", use_level=False, constraints=cons)
        lad.set_objective(OptimizationData(return_series=X.iloc[e - 252:e], bm_series=y.iloc[e - 252:e]))
        lad.model_qpsolvers()
        m = lad.model
        assert np.array_equal(m["q"], g["q"][i]) and np.allclose(m["A"], g["A"][i], rtol=1e-13, atol=0)
        assert np.allclose(m["b"], g["b"][i], rtol=1e-13, atol=0)
        assert np.array_equal(m["lb"], g["lb"][i]) and np.array_equal(m["ub"], g["ub"][i])
        assert not np.any(m["P"]) and m["G"] is None


def test_api_objects_construct_without_gpu():
    from porqua_amd.backtest import Backtest, BacktestService
    from porqua_amd.builders import OptimizationItemBuilder, SelectionItemBuilder, bibfn_selection_data
    from porqua_amd.covariance import Covariance
    from porqua_amd.optimization import (EmptyOptimization, LeastSquares, MeanVariance, QEQW,
                                         WeightedLeastSquares)
    for cls in (LeastSquares, MeanVariance, QEQW, WeightedLeastSquares, EmptyOptimization):
        o = cls(solver_name="mi355x")
        assert o.params["solver_name"] == "mi355x"
    assert LeastSquares().params["solver_name"] == "mi355x" and LeastSquares(verbose=False).params["verbose"] is False
    mv = MeanVariance(covariance=Covariance(method="linear_shrinkage", lambda_covmat_regularization=0.1))
    assert mv.params["risk_aversion"] == 1 and mv.covariance.spec["method"] == "linear_shrinkage"
    bs = BacktestService(data={}, selection_item_builders={"d": SelectionItemBuilder(bibfn=bibfn_selection_data)},
                         optimization_item_builders={}, optimization=mv, rebdates=[])
    Backtest().run(bs)


def test_group_plan_joins_identical_windows_of_a_sweep():
    """A risk-aversion sweep repeats every date's window; the grouped-ADMM plan joins the
    repeats (shift 0, same union), the sliding-K1 plan does not."""
    dates, _, _, _ = factor_panel(400, 3)
    rows, tlen = engine.window_rows(dates, dates[[300, 390]], 120)   # 90-row gap: no slide
    rep_rows, rep_tlen = np.repeat(rows, 6, axis=0), np.repeat(tlen, 6)
    gs, sh = engine.slide_plan(rep_rows, rep_tlen, group=16, smin=0)
    assert list(gs) == [0, 6, 12] and np.all(sh == 0)
    gs1, _ = engine.slide_plan(rep_rows, rep_tlen, group=16)
    assert len(gs1) - 1 == 12
    gp = engine.GroupPlan(rep_rows, rep_tlen, torch.device("cpu"))   # 12 problems: groups of <= 4
    assert gp.ok and list(gp.gdates.numpy()) == [0, 4, 6, 10, 12]
    assert np.all(gp.ucnt.numpy() == 120) and np.all(gp.uoff.numpy() == 0)


def test_kkt_certificate_accepts_oracle_and_rejects_perturbed():
    from oracle.qp_ipm import solve_qp
    from tests.kkt import kkt_residuals
    rng = np.random.default_rng(3)
    n = 40
    X = rng.normal(0, 0.02, (30, n))
    P = 2 * X.T @ X + 1e-4 * np.eye(n)
    q = -rng.normal(0, 0.01, n)
    G = (rng.random((3, n)) < 0.4).astype(float)
    h = np.full(3, 0.3)
    o = solve_qp(P, q, G=G, h=h, A=np.ones((1, n)), b=np.ones(1), lb=np.zeros(n), ub=np.full(n, 0.2))
    y = np.concatenate([np.atleast_1d(o.y), np.atleast_1d(o.z)])
    k = kkt_residuals(P, q, o.x, A=np.ones((1, n)), b=np.ones(1), G=G, h=h, lb=np.zeros(n),
                      ub=np.full(n, 0.2), y=y, z_box=o.z_box)
    assert max(k.values()) < 1e-9, k
    xp = o.x.copy()
    xp[:2] += np.array([1e-4, -1e-4])
    k2 = kkt_residuals(P, q, xp, A=np.ones((1, n)), b=np.ones(1), G=G, h=h, lb=np.zeros(n),
                       ub=np.full(n, 0.2), y=y, z_box=o.z_box)
    assert max(k2.values()) > 1e-7


def _loop_slide_plan(rows, tlen, group, smax, smin):
    """Direct restatement of engine.slide_plan's contract: d joins d-1 when its window is
    that window shifted by smin <= s <= smax rows (same length), groups of <= ``group``."""
    B = len(tlen)
    shift = np.zeros(B, dtype=np.int32)
    gs = [0] if B else []
    cnt = 1
    for d in range(1, B):
        tp, tc = int(tlen[d - 1]), int(tlen[d])
        prev, cur = rows[d - 1, :tp], rows[d, :tc]
        s = int((prev < cur[0]).sum()) if tc else 0
        ok = tp == tc and tc > 1 and smin <= s <= smax and np.array_equal(prev[s:], cur[:tc - s])
        if ok:
            shift[d] = s
        if not ok or cnt == group:
            gs.append(d)
            cnt = 0
        cnt += 1
    gs.append(B)
    return np.asarray(gs, dtype=np.int32), shift


def test_planners_match_their_contracts_on_random_calendars():
    """window_rows (vs the oracle's per-date restatement of src/builders.py:208-211),
    slide_plan (vs a per-date loop) and GroupPlan (every date's window is its union slice
    [uoff, uoff + T), unions within umax) on calendars with weekends, gaps, repeated
    rebalance dates, descending or shuffled rebalance dates and short histories."""
    import torch
    rng = np.random.default_rng(11)
    for trial in range(30):
        n = int(rng.integers(30, 1500))
        cal = np.arange(np.datetime64("2003-01-01"), np.datetime64("2003-01-01") + n)
        if trial % 3:
            cal = cal[((cal.astype("int64") + 3) % 7) < 5]
        if trial % 2:
            cal = cal[rng.random(len(cal)) < 0.93]
        if len(cal) < 3:
            continue
        T = int(rng.integers(2, 120))
        reb = cal[int(rng.integers(0, min(len(cal) - 1, T + 3))):][::int(rng.choice([1, 1, 3, 21]))]
        if trial % 4 == 0:
            reb = np.repeat(reb, int(rng.integers(1, 4)))
        if trial % 5 == 1:     # descending rebalance dates: a later window starts earlier
            reb = reb[::-1].copy()
        elif trial % 5 == 3:   # shuffled (the slide plan must not take them as identical)
            reb = reb[rng.permutation(len(reb))]
        rows, tlen = engine.window_rows(cal, reb, T)
        for b in range(0, len(reb), max(1, len(reb) // 17)):
            assert np.array_equal(rows[b, :tlen[b]], rp.window_rows(cal, reb[b], T))
        for group, smax, smin in ((32, 64, 1), (16, 64, 0), (3, 5, 0)):
            gs, sh = engine.slide_plan(rows, tlen, group, smax, smin)
            gs2, sh2 = _loop_slide_plan(rows, tlen, group, smax, smin)
            assert np.array_equal(gs, gs2) and np.array_equal(sh, sh2)
        gp = engine.GroupPlan(rows, tlen, torch.device("cpu"), gmax=16, gmin=16)
        if not gp.ok:
            continue
        gd, ur, uc, uo = (gp.gdates.numpy(), gp.urows.numpy(), gp.ucnt.numpy(), gp.uoff.numpy())
        assert gd[0] == 0 and gd[-1] == len(tlen) and (np.diff(gd) >= 1).all() and (uc <= gp.umax).all()
        for g in range(gp.ngroups):
            for d in range(gd[g], gd[g + 1]):
                t = int(tlen[d])
                assert np.array_equal(ur[g, uo[d]:uo[d] + t], rows[d, :t])


def test_sparse_columns_of_group_rows():
    """engine._sparse_columns: budget + 0/1 sector rows -> per-column (row, value) lists with
    -1 padding; dense or few rows -> none (the grouped ADMM then reads Cg densely)."""
    import torch
    n = 10
    sec = np.array([0, 1, 2, 0, 1, 2, 3, 3, 0, 1])
    G = np.stack([(sec == g).astype(float) for g in range(4)])
    qb = engine.QPBatch.from_dense(None, None, n=n, A=np.ones((1, n)), b=np.ones(1), G=G, h=np.full(4, 0.5),
                                   lb=np.zeros(n), ub=np.ones(n), device=torch.device("cpu"))
    rows, vals, nzmax = engine._sparse_columns(qb)
    assert nzmax == 2 and rows.shape == (qb.ld, 2)
    C = qb.Cg[0, :qb.mg, :n].numpy()
    for i in range(n):
        dense = np.zeros(qb.mg)
        for r, v in zip(rows[i].tolist(), vals[i].tolist()):
            if r >= 0:
                dense[r] = v
        assert np.array_equal(dense, C[:, i])
    assert (rows[n:] == -1).all()
    qb2 = engine.QPBatch.from_dense(None, None, n=n, A=np.ones((1, n)), b=np.ones(1), G=np.ones((4, n)),
                                    h=np.full(4, 0.5), lb=np.zeros(n), ub=np.ones(n), device=torch.device("cpu"))
    assert engine._sparse_columns(qb2)[2] == 0     # 5 nonzeros per column: dense reads


def test_trailing_window_slice_matches_the_boolean_mask():
    """builders._upto (one positional slice on a sorted DatetimeIndex) returns exactly
    data[data.index <= rebdate].tail(width) (src/builders.py:188-251), for dates inside,
    before and after the panel, dates between rows, any width, and an unsorted index."""
    import pandas as pd
    from porqua_amd import builders
    idx = pd.bdate_range("2020-01-01", periods=300)
    df = pd.DataFrame(np.arange(600.0).reshape(300, 2), index=idx, columns=["a", "b"])
    for data in (df, df.iloc[::-1], df["a"]):
        for date in ("2019-06-01", "2020-01-01", "2020-03-07", str(idx[150].date()), str(idx[-1].date()),
                     "2030-01-01"):
            for width in (1, 21, 252, 1000, None):
                ref = data[data.index <= date]
                ref = ref.tail(width) if width is not None else ref
                assert builders._upto(data, date, width).equals(ref), (date, width)


def test_single_binary_filter_selection():
    import pandas as pd
    from porqua_amd.selection import Selection
    s = Selection()
    s.add_filtered("data", pd.Series([1, 0, 1, 1], index=list("abcd"), name="binary"))
    assert list(s.selected) == ["a", "c", "d"] and isinstance(s.selected, pd.Index)
    s.add_filtered("more", pd.Series([1, 1, 0, 1], index=list("abcd"), name="binary"))
    assert list(s.selected) == ["a", "d"]


def test_panel_upload_resolves_the_device_on_the_calling_thread(monkeypatch):
    """_PanelUpload asks for the device on the caller's thread (torch's current device is
    per host thread: a worker would see device 0, not the rank's set_device choice) and copies
    to that device on the worker."""
    import threading
    from porqua_amd import backtest as bt
    seen = []

    def fake_device():
        seen.append(threading.current_thread())
        return torch.device("cpu")

    monkeypatch.setattr(engine, "default_device", fake_device)
    frame = pd.DataFrame(np.arange(12.0).reshape(4, 3))
    up = bt._PanelUpload(frame)
    out = up.result()
    assert seen == [threading.current_thread()]
    assert out.device.type == "cpu" and np.array_equal(out.numpy(), frame.to_numpy())


def test_loose_stop_eps_rule():
    """engine.loose_stop_eps: centred windows take eps_grouped; tracking windows take
    eps_grouped_tracking, or eps_grouped_tracking_small (off by default) for batches of at
    most small_batch dates (the notebook's monthly run), or eps_grouped_tracking_wide with more
    than 4 general rows (config 4's sector caps); eps_grouped = 0 turns every loose stop off."""
    from porqua_amd import engine
    s = engine.Settings()
    assert engine.loose_stop_eps(s, True, 4749) == s.eps_grouped
    assert engine.loose_stop_eps(s, False, 4544) == 0.0
    assert s.eps_grouped_tracking_small == 0.0 and engine.loose_stop_eps(s, False, 13) == 0.0
    assert engine.loose_stop_eps(s, False, 13, mg=21) == s.eps_grouped_tracking_wide   # small wide batch
    sm = engine.Settings(eps_grouped_tracking_small=1e-2)
    assert engine.loose_stop_eps(sm, False, 13) == 1e-2
    assert engine.loose_stop_eps(sm, False, sm.small_batch) == 1e-2
    assert engine.loose_stop_eps(sm, False, sm.small_batch + 1) == 0.0
    off = engine.Settings(eps_grouped=0.0)
    assert engine.loose_stop_eps(off, False, 13) == 0.0 and engine.loose_stop_eps(off, True, 13) == 0.0
    assert engine.loose_stop_eps(s, False, 9749, mg=21) == s.eps_grouped_tracking_wide > 0.0
    assert engine.loose_stop_eps(s, False, 9749, mg=4) == 0.0
    assert engine.loose_stop_eps(off, False, 9749, mg=21) == 0.0
    own = engine.Settings(eps_grouped_tracking=3e-2)
    assert engine.loose_stop_eps(own, False, 13) == 3e-2 and engine.loose_stop_eps(own, False, 4544) == 3e-2


def test_sweep_plan_groups_and_applicability():
    """engine.SweepPlan (the risk-aversion groups of pq_admm_lr_sweep): rows of up to 64
    problems, a longer row split, and the kernel's shape conditions."""
    sp = engine.SweepPlan([40, 70, 64], "cpu")
    assert sp.gdates.tolist() == [0, 40, 104, 110, 174] and sp.ngroups == 4
    assert engine.SweepPlan([], "cpu").ngroups == 0
    n = 300
    qb = engine.QPBatch(n, 174, 1, device="cpu", P=torch.empty(0, dtype=torch.float64))

    class LR:
        tmax = 252
    assert sp.applicable(qb, LR(), 256)
    LR.tmax = 300                       # window beyond the kernel's 256 rows
    assert not sp.applicable(qb, LR(), 256)
    LR.tmax = 252
    assert not sp.applicable(qb, LR(), 320)   # capacitance beyond k_ld 256
    q5 = engine.QPBatch(n, 174, 5, device="cpu", P=torch.empty(0, dtype=torch.float64))
    assert not sp.applicable(q5, LR(), 256)   # more than 4 general rows
    qs = engine.QPBatch(n, 174, 1, device="cpu", shared_constraints=False, P=torch.empty(0, dtype=torch.float64))
    assert not sp.applicable(qs, LR(), 256)   # per-problem rows / boxes
    need = _lib.load().pq_sweep_scratch_doubles(5000, 4096, 64)
    assert need == 4096 * 80 + 64 * 20 * 64 * (256 + 16) + 64 * 256 * 64 + 64
