"""World-size-2 gloo tests of the date-sharded multi-GPU paths, on CPU.

* The config-5 partition (porqua_amd.sweep.MeanVarianceSweep): each rank owns a contiguous
  block of dates with EVERY risk aversion of those dates (so a date's window Gram /
  eigendecomposition is shared by its lambda row), and ``gather`` reassembles the date-major
  (date, lambda) grid of weights, status and objective with one collective.
* The sharded drop-in (Backtest.run, src/backtest.py:201-224): two ranks each run the batched
  Backtest.run over their block of rebalance dates with a host stub in place of the device
  solve (Backtest._solve_shard); the gathered Strategy equals the single-rank one.
"""
import os

import numpy as np
import pandas as pd
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from porqua_amd.backtest import Backtest, BacktestService, shard_range
from porqua_amd.builders import (OptimizationItemBuilder, SelectionItemBuilder, bibfn_box_constraints,
                                 bibfn_budget_constraint, bibfn_return_series, bibfn_selection_data)
from porqua_amd.optimization import MeanVariance

ND, L, N, T = 7, 5, 24, 40


def _panel():
    rng = np.random.default_rng(7)
    dates = pd.bdate_range("2020-01-01", periods=T - 1 + 21 * ND)
    R = rng.normal(3e-4, 0.02, size=(len(dates), N))
    return dates, R


def _sweep_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from porqua_amd import engine
    from porqua_amd.sweep import MeanVarianceSweep
    dates, R = _panel()
    d = dates.values.astype("datetime64[D]")
    ends = np.arange(T - 1, T - 1 + 21 * ND, 21)
    rows, tlen = engine.window_rows(d, d[ends], T)
    cpu = torch.device("cpu")
    pan = engine.Panel(R, device=cpu)
    lam = np.logspace(-1, 2, L)
    sw = MeanVarianceSweep(pan, rows, tlen, lam, rank=rank, world=world, group=False)
    lo, hi = shard_range(ND, rank, world)
    ok = (sw.lo, sw.hi) == (lo, hi) and sw.B == (hi - lo) * L
    # every local problem (d - lo) * L + j is date d with lambdas[j], on date d's window rows
    rp = sw.rp_d.numpy()
    ps = sw.qb.p_scale.numpy()
    for p in range(sw.B):
        dd, j = lo + p // L, p % L
        ok &= bool(np.array_equal(rp[p], rows[dd])) and abs(ps[p] - 2.0 * lam[j]) < 1e-15
    # a stand-in result whose entries encode (date, lambda): the gather must put each block
    # back in date-major order
    B = sw.B
    x = torch.zeros((B, N), dtype=torch.float64)
    st = torch.zeros(B, dtype=torch.int32)
    out = torch.zeros((B, 8), dtype=torch.float64)
    for p in range(B):
        dd, j = lo + p // L, p % L
        x[p] = dd * 100.0 + j + torch.arange(N, dtype=torch.float64) * 1e-3
        st[p] = 1 + (dd + j) % 3
    from porqua_amd import _lib
    out[:, _lib.PQ_OUT_OBJ] = x[:, 0] * 2.0
    res = engine.BatchResult(x=x, y=x[:, :1], z_box=x, status=st, iters=st, out=out)
    X, S, O = sw.gather(res, dist)
    want = np.array([[dd * 100.0 + j + k * 1e-3 for k in range(N)] for dd in range(ND) for j in range(L)])
    ok &= X.shape == (ND * L, N) and np.array_equal(X, want)
    ok &= np.array_equal(S, np.array([1 + (dd + j) % 3 for dd in range(ND) for j in range(L)]))
    ok &= np.array_equal(O, want[:, 0] * 2.0)
    q.put((rank, bool(ok)))
    dist.barrier()
    dist.destroy_process_group()


def _spawn(target, world, port, extra=()):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=target, args=(r, world, port) + tuple(extra) + (q,)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=180) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    return res


def test_sweep_partition_keeps_lambda_rows_and_gathers_world2():
    assert _spawn(_sweep_worker, 2, 32500 + os.getpid() % 2000) == [(0, True), (1, True)]


def test_sweep_partition_more_ranks_than_dates():
    # 7 dates over 3 ranks: blocks 3 / 2 / 2 -- still every lambda of a date on one rank
    assert _spawn(_sweep_worker, 3, 33500 + os.getpid() % 2000) == [(0, True), (1, True), (2, True)]


class StubBacktest(Backtest):
    """Backtest.run with the device solve replaced by a host stub: the inverse-variance
    portfolio of each date's window (deterministic, depends on the date's rows only)."""

    def _solve_shard(self, bs, st, lo, hi):
        X = st["Xs"].to_numpy(dtype=np.float64)
        rows, tlen = st["rows"], st["tlen"]
        W = np.zeros((hi - lo, X.shape[1]))
        for i in range(lo, hi):
            win = X[rows[i, :tlen[i]]]
            iv = 1.0 / win.var(0, ddof=1)
            W[i - lo] = iv / iv.sum()
        ST = np.ones(hi - lo, dtype=np.int32)
        OBJ = W.sum(1) + np.arange(lo, hi)
        self.shard = (lo, hi)
        return True, W, ST, OBJ, "stub"


def _service():
    dates, R = _panel()
    Xdf = pd.DataFrame(R, index=dates, columns=[f"a{i}" for i in range(N)])
    reb = [str(x.date()) for x in dates[T - 1::3]]
    return BacktestService(
        data={"return_series": Xdf},
        selection_item_builders={"data": SelectionItemBuilder(bibfn=bibfn_selection_data)},
        optimization_item_builders={
            "return_series": OptimizationItemBuilder(bibfn=bibfn_return_series, width=T),
            "budget_constraint": OptimizationItemBuilder(bibfn=bibfn_budget_constraint, budget=1),
            "box_constraints": OptimizationItemBuilder(bibfn=bibfn_box_constraints)},
        optimization=MeanVariance(solver_name="mi355x"), rebdates=reb, quiet=True)


def _backtest_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    bt = StubBacktest()
    bs = _service()
    bt.run(bs)
    W = bt.strategy.get_weights_df().to_numpy(dtype=float)
    q.put((rank, bt.shard, W.tolist(), list(bt.stats["objective"]), bt.stats["solved"]))
    dist.barrier()
    dist.destroy_process_group()


def test_sharded_backtest_run_matches_single_rank_world2():
    single = StubBacktest()
    bs = _service()
    single.run(bs)
    nreb = len(bs.settings["rebdates"])
    W1 = single.strategy.get_weights_df().to_numpy(dtype=float)
    assert single.shard == (0, nreb) and W1.shape == (nreb, N)
    res = _spawn(_backtest_worker, 2, 34500 + os.getpid() % 2000)
    assert [r[0] for r in res] == [0, 1]
    assert [tuple(r[1]) for r in res] == [shard_range(nreb, 0, 2), shard_range(nreb, 1, 2)]
    for _, _, W, obj, solved in res:   # every rank holds the whole gathered strategy
        assert solved == nreb
        assert np.array_equal(np.asarray(W), W1)
        assert np.allclose(obj, single.stats["objective"], rtol=0, atol=0)
