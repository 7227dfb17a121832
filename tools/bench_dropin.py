#!/usr/bin/env python3
"""Drop-in throughput: Backtest.run(bs) through the reference API (solver_name='mi355x') on
the config-3 shape (synthetic 5000 x 1000 panel, 252-day windows, daily rebalance = 4749
QPs, budget + long-only box), MeanVariance (Pearson covariance, geometric mean) -- timed from
Backtest.run to the weights in strategy.portfolios, after one warm-up run; --profile adds a
cProfile of one run.  Prints one JSON line.  Experiment tooling."""
import argparse
import cProfile
import io
import json
import os
import pstats
import sys
import time

import pandas as pd
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
from bench_wls import service  # noqa: E402
from porqua_amd.backtest import Backtest  # noqa: E402
from porqua_amd.optimization import MeanVariance  # noqa: E402
from porqua_amd.synthetic import factor_panel  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1000)
    ap.add_argument("--days", type=int, default=5000)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--profile", action="store_true")
    a = ap.parse_args()
    width = 252
    dates, R, y, _ = factor_panel(a.days, a.n)
    idx = pd.DatetimeIndex(dates)
    X = pd.DataFrame(R, index=idx, columns=[f"a{i}" for i in range(a.n)])
    Y = pd.DataFrame({"bm": y}, index=idx)
    rebdates = [str(d.date()) for d in idx[width - 1:]]

    def run():
        bt = Backtest()
        bt.run(service(MeanVariance(solver_name="mi355x"), X, Y, rebdates, width))
        torch.cuda.synchronize()
        return bt
    run()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        bt = run()
    dt = (time.perf_counter() - t0) / a.steps
    out = {"workload": "Backtest.run, MeanVariance (pearson, geometric mean), config-3 shape",
           "dates": len(rebdates), "s_per_run": dt, "qps": len(rebdates) / dt, "path": bt.stats["path"],
           "solved": bt.stats["solved"]}
    if a.profile:
        pr = cProfile.Profile()
        pr.enable()
        run()
        pr.disable()
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats("cumulative").print_stats(35)
        print(s.getvalue(), file=sys.stderr)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
