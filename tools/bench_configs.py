#!/usr/bin/env python3
"""Throughput of BASELINE.json configs 1/2, 4 and 5 on one MI355X (the bench line is config 3).

* configs 1/2: SPTR index replication on the usa-shaped panel (494 assets on the last 4795
  real SPTR dates, porqua_amd.synthetic.usa_panel), least-squares tracking, budget + LongOnly
  box, width 252 (example/backtest.ipynb): config 2 = Backtest.run with solver_name='mi355x'
  (drop-in, host staging included) on the 13 monthly dates and on every date of the panel
  (4543 daily QPs); config 1 = the CPU reference path restated by the oracle (window, P = 2X'X,
  q = -2X'y, oracle.qp_ipm) on the monthly dates, serial, timed on this host.

* config 4: synthetic 3000 assets x 10000 dates, 252-day windows, daily rebalance
  (9749 QPs), tracking-error least squares (P = 2 X'X uncentred, q = -2 X'y) with budget,
  long-only box and 20 sector caps <= 0.15 (G 20 x n) -- the window path with 21 general
  rows.  --dates limits the number of rebalance dates (memory / time).
* config 5: synthetic 5000 assets, 64 rebalance dates x 64 risk aversions log-spaced in
  [0.1, 100] = 4096 mean-variance QPs (porqua_amd.sweep).

Prints one JSON line per config: QPs/s over --steps timed solves after one warmup, status
counts and ADMM iterations.  Experiment tooling; numbers are quoted in DESIGN.md §9."""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from porqua_amd import _lib, engine  # noqa: E402
from porqua_amd.sweep import mean_variance_sweep  # noqa: E402
from porqua_amd.synthetic import factor_panel  # noqa: E402
from porqua_amd.workloads import TrackingBacktest, sweep_certificate  # noqa: E402


def timed(fn, steps):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        res = fn()
    torch.cuda.synchronize()
    return res, (time.perf_counter() - t0) / steps


def summary(res):
    st = res.status.cpu().numpy()
    return {"status_counts": {str(k): int(v) for k, v in zip(*np.unique(st, return_counts=True))},
            "mean_iters": float(res.iters.float().mean().item()), "max_iters": int(res.iters.max().item()),
            "polish_rounds_mean": float(res.out[:, _lib.PQ_OUT_ROUNDS].mean().item()),
            "nfree_min": int(res.out[:, _lib.PQ_OUT_NFREE].min().item())}


def config4(dates_limit, steps, dev, overrides=None):
    """The config-4 workload exactly as bench.py --workload config4 and
    tests/test_full_configs_gpu.py build it (workloads.TrackingBacktest)."""
    settings = engine.Settings.from_params(dict({"rho0_rel": 0.1, "rho0_qrel": 0.0}, **(overrides or {})))
    wl = TrackingBacktest(D=dates_limit, device=dev, settings=settings)
    ev = []

    def run():
        ev.clear()
        return wl.step(events=ev)     # q = -2 X'y per date (window products) inside the step

    res, dt = timed(run, steps)
    torch.cuda.synchronize()
    return dict({"config": "config4: n=3000 tracking LS, budget + box + 20 sector caps, daily",
                 "qps": wl.D / dt, "ms_per_step": dt * 1e3, "dates": wl.D, "stage_ms": stage_ms(ev)},
                **summary(res), certificate=wl.certificate(res))


def stage_ms(events):
    """Per-stage milliseconds of the last timed step (engine._Timeline HIP event pairs)."""
    out = {}
    for name, e0, e1 in events:
        out[name] = out.get(name, 0.0) + e0.elapsed_time(e1)
    return {k: round(v, 3) for k, v in out.items()}


def config5(steps, dev, settings=None, factor="auto"):
    n, T, nd, L = 5000, 252, 64, 64
    dates, R, _, _ = factor_panel(T - 1 + 21 * nd, n)
    ends = np.arange(T - 1, T - 1 + 21 * nd, 21)
    rows, tlen = engine.window_rows(dates, dates[ends], T)
    pan = engine.Panel(R, device=dev)
    lambdas = np.logspace(-1, 2, L)
    meta = {}
    ev = []

    def run():
        ev.clear()
        r, m = mean_variance_sweep(pan, rows, tlen, lambdas, settings=settings, events=ev, factor=factor)
        meta.update(m)
        return r
    res, dt = timed(run, steps)
    torch.cuda.synchronize()
    cert = sweep_certificate(pan, res, meta)
    return dict({"config": "config5: n=5000 mean-variance, 64 monthly dates x 64 risk aversions",
                 "certificate": cert,
                 "qps": nd * L / dt, "ms_per_step": dt * 1e3, "qps_per_step": nd * L,
                 "capacitance": meta.get("capacitance"), "factorizations_per_step": meta.get("factorizations"),
                 "factor": meta.get("factor"), "stage_ms": stage_ms(ev)}, **summary(res))


def config12(steps, dev, params=None):
    import pandas as pd
    from oracle.qp_ipm import solve_qp
    from oracle.ref_pipeline import objective_least_squares, window_rows
    from porqua_amd.backtest import Backtest
    from tests.test_configs12_gpu import service, usa_data
    X, y = usa_data()
    d = X.index.values.astype("datetime64[D]")
    monthly = [str(r) for r in d[d > np.datetime64("2022-06-01")][::21]]
    daily = [str(r) for r in d[251:]]
    out = []
    for tag, reb in (("monthly", monthly), ("daily", daily)):
        def run():
            bt = Backtest()
            bt.run(service(X, y, reb, params=params))
            return bt
        bt, dt = timed(run, steps)
        out.append({"config": f"config2: SPTR replication, n=494 LS tracking, {tag} ({len(reb)} dates), "
                              "Backtest.run(solver_name='mi355x')", "qps": len(reb) / dt, "ms_per_run": dt * 1e3,
                    "dates": len(reb), "solved": bt.stats["solved"], "path": bt.stats["path"],
                    "params": params or {}})
    Xv, yv = X.to_numpy(), y.to_numpy()[:, 0]
    n = Xv.shape[1]
    t0 = time.perf_counter()
    for rd in monthly:
        rows = window_rows(d, rd, 252)
        P, q, _ = objective_least_squares(Xv[rows], yv[rows])
        solve_qp(P, q, A=np.ones((1, n)), b=np.ones(1), lb=np.zeros(n), ub=np.ones(n))
    dt = time.perf_counter() - t0
    out.append({"config": "config1: same monthly backtest, CPU reference path (oracle restatement, serial, "
                          "multithreaded BLAS; qpsolvers/cvxopt unavailable)", "qps": len(monthly) / dt,
                "seconds": dt, "dates": len(monthly)})
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--dates", type=int, default=9749, help="config 4 rebalance dates")
    ap.add_argument("--only", choices=["12", "4", "5"], default=None)
    ap.add_argument("--factor", default="auto", help="config 5 capacitance factor(s): auto, eig, chol or eig,chol")
    ap.add_argument("--set", action="append", default=[], metavar="KEY=VALUE",
                    help="engine.Settings override (experiments): configs 1/2 through the optimization's "
                         "params, configs 4/5 directly")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    if args.only in (None, "12"):
        for line in config12(args.steps, dev, dict(kv.split("=", 1) for kv in args.set) or None):
            print(json.dumps(line), flush=True)
    if args.only in (None, "4"):
        ov = dict(kv.split("=", 1) for kv in args.set)
        print(json.dumps(dict(config4(args.dates, args.steps, dev, ov), settings_overrides=args.set)), flush=True)
    if args.only in (None, "5"):
        st = engine.Settings.from_params(dict(kv.split("=", 1) for kv in args.set)) if args.set else None
        for fac in args.factor.split(","):
            print(json.dumps(dict(config5(args.steps, dev, st, factor=fac), settings_overrides=args.set)), flush=True)


if __name__ == "__main__":
    main()
