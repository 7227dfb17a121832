#!/usr/bin/env python3
"""Phase split of the drop-in Backtest.run at the config-3 shape (bench.py's end_to_end line:
MeanVariance, 4749 daily dates, n = 1000): each phase bracketed by device synchronisations so
host and device time land on the phase that causes them.  Experiment tooling.

    python tools/dropin_phases.py [runs]"""
import os
import sys
import time
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from porqua_amd import backtest as bt_mod, engine  # noqa: E402
from porqua_amd.backtest import Backtest  # noqa: E402
from tools.prof_dropin import mv3_service  # noqa: E402

ACC = defaultdict(float)
CNT = defaultdict(int)


def timed(owner, name, label):
    fn = getattr(owner, name)

    def wrap(*a, **k):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r = fn(*a, **k)
        torch.cuda.synchronize()
        ACC[label] += time.perf_counter() - t0
        CNT[label] += 1
        return r
    wrap.__wrapped_orig__ = fn
    setattr(owner, name, wrap)


def main():
    runs = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    make = mv3_service()
    Backtest().run(make())          # warm-up (library load, allocator, plans' first use)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(runs):
        Backtest().run(make())
    torch.cuda.synchronize()
    plain = (time.perf_counter() - t0) / runs
    print(f"plain run: {plain * 1e3:.2f} ms  ({4749 / plain:.0f} QPs/s)", flush=True)
    timed(bt_mod.BacktestService, "prepare_rebalancing", "prepare_rebalancing (builders, first date)")
    timed(engine, "window_rows", "window_rows")
    timed(engine.Panel, "__init__", "Panel upload")
    timed(bt_mod.BatchStage, "__init__", "BatchStage (rows upload)")
    timed(engine.QPBatch, "from_dense", "QPBatch.from_dense")
    timed(bt_mod.BatchStage, "group_plan", "GroupPlan")
    timed(engine, "solve_lowrank", "solve_lowrank")
    timed(Backtest, "_finish_batched", "finish (Portfolio objects)")
    opt_cls = type(make().optimization)
    timed(opt_cls, "objective_batch", "objective_batch")
    ACC.clear()
    CNT.clear()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(runs):
        Backtest().run(make())
    torch.cuda.synchronize()
    tot = (time.perf_counter() - t0) / runs
    print(f"bracketed run: {tot * 1e3:.2f} ms", flush=True)
    named = 0.0
    for k, v in sorted(ACC.items(), key=lambda kv: -kv[1]):
        print(f"  {k:48s} {v / runs * 1e3:8.2f} ms  ({CNT[k] // runs} calls)")
        named += v / runs
    print(f"  {'(rest: service build, result copies, glue)':48s} {(tot - named) * 1e3:8.2f} ms")
    # the top-level phases of Backtest.run (no inner brackets: each phase's host work and
    # the device time it waits for), and the service build that the bench line also times
    for owner, name in ((engine.Panel, "__init__"), (bt_mod.BatchStage, "__init__"), (engine.QPBatch, "from_dense"),
                        (bt_mod.BatchStage, "group_plan"), (engine, "solve_lowrank"), (Backtest, "_finish_batched"),
                        (opt_cls, "objective_batch"), (bt_mod.BacktestService, "prepare_rebalancing"),
                        (engine, "window_rows")):
        setattr(owner, name, getattr(owner, name).__wrapped_orig__ if hasattr(getattr(owner, name), "__wrapped_orig__")
                else getattr(owner, name))
    ACC.clear()
    CNT.clear()
    top = [(Backtest, "_stage_batched", "A stage (host: builders, windows, constraints)"),
           (bt_mod._PanelUpload, "result", "B0 wait for the panel upload"),
           (Backtest, "_solve_shard", "B solve shard (incl. the upload wait)"),
           (Backtest, "_finish_batched", "C finish (Portfolio objects)")]
    for owner, name, label in top:
        timed(owner, name, label)
    t_make = 0.0
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(runs):
        tm = time.perf_counter()
        svc = make()
        t_make += time.perf_counter() - tm
        Backtest().run(svc)
    torch.cuda.synchronize()
    tot = (time.perf_counter() - t0) / runs
    print(f"top-level split: {tot * 1e3:.2f} ms per run (service build {t_make / runs * 1e3:.2f} ms)", flush=True)
    for k, v in sorted(ACC.items()):
        print(f"  {k:48s} {v / runs * 1e3:8.2f} ms  ({CNT[k] // runs} calls)")
    # the device solve of one more run, stage by stage (HIP events) with its iteration and
    # round counts: where the drop-in's solve differs from the bench step's
    from porqua_amd import _lib
    inner = engine.solve_lowrank.__wrapped__ if hasattr(engine.solve_lowrank, "__wrapped__") else None
    seen = {}

    def probe(*a, **k):
        ev = []
        k["events"] = ev
        ws = k["ws"] = engine.Workspace(a[0], dense=False)
        r = (inner or orig)(*a, **k)
        torch.cuda.synchronize()
        rall = ws.pg_record().cpu().numpy()
        print("polish rounds per date:", np.unique(rall[:, _lib.PQ_PG_STATE + 1], return_counts=True))
        fb = getattr(ws, "pg_fallback", None)
        if fb is not None:   # the dates the grouped polish handed back, and their records
            R = ws.pg_record()[fb.long()].cpu().numpy()
            o = r.out[fb.long()].cpu().numpy()
            print("handed back:", len(R), "k", np.unique(R[:, 0], return_counts=True),
                  "ma", np.unique(R[:, 1], return_counts=True), "rounds", np.unique(R[:, 4], return_counts=True),
                  "final nfree", np.unique(o[:, _lib.PQ_OUT_NFREE], return_counts=True))
        seen["ev"] = [(nm, x.elapsed_time(y)) for nm, x, y in ev]
        out = r.out.cpu().numpy()
        seen["stats"] = dict(iters=float(r.iters.float().mean()), rounds=float(out[:, _lib.PQ_OUT_ROUNDS].mean()),
                             nfree=float(out[:, _lib.PQ_OUT_NFREE].mean()), kw=sorted(k))
        return r
    orig = engine.solve_lowrank
    engine.solve_lowrank = probe
    Backtest().run(make())
    print("drop-in solve stages:", ", ".join(f"{nm} {t:.2f} ms" for nm, t in seen.get("ev", [])))
    print("drop-in solve stats:", seen.get("stats"))


if __name__ == "__main__":
    main()
