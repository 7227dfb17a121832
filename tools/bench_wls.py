#!/usr/bin/env python3
"""End-to-end Backtest.run throughput of the tracking objectives on the config-3 shape
(synthetic 5000 x 1000 panel, 252-day windows, daily rebalance = 4749 QPs, budget + long-only
box) through the reference API (porqua_amd.backtest, solver_name='mi355x'):

* WeightedLeastSquares, tau = 252 (the reference's own use,
  src/_quick_and_dirty_interactive_testing.py:159-162): one row-scaled panel + per-date scalars;
* LeastSquares on the same data, for comparison.

Timed from Backtest.run(bs) to the weights in strategy.portfolios (host pandas bookkeeping
included) after one warmup run.  Prints one JSON line per objective.  Experiment tooling."""
import argparse
import json
import os
import sys
import time

import numpy as np
import pandas as pd
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from porqua_amd.backtest import Backtest, BacktestService  # noqa: E402
from porqua_amd.builders import (OptimizationItemBuilder, SelectionItemBuilder,  # noqa: E402
                                 bibfn_box_constraints, bibfn_bm_series, bibfn_budget_constraint,
                                 bibfn_return_series, bibfn_selection_data)
from porqua_amd.optimization import LeastSquares, WeightedLeastSquares  # noqa: E402
from porqua_amd.synthetic import factor_panel  # noqa: E402


def service(opt, X, y, rebdates, width):
    return BacktestService(
        data={"return_series": X, "bm_series": y},
        selection_item_builders={"data": SelectionItemBuilder(bibfn=bibfn_selection_data)},
        optimization_item_builders={
            "return_series": OptimizationItemBuilder(bibfn=bibfn_return_series, width=width),
            "bm_series": OptimizationItemBuilder(bibfn=bibfn_bm_series, width=width),
            "budget_constraint": OptimizationItemBuilder(bibfn=bibfn_budget_constraint, budget=1),
            "box_constraints": OptimizationItemBuilder(bibfn=bibfn_box_constraints)},
        optimization=opt, rebdates=rebdates, quiet=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1000)
    ap.add_argument("--days", type=int, default=5000)
    ap.add_argument("--dates", type=int, default=4749)
    ap.add_argument("--steps", type=int, default=2)
    a = ap.parse_args()
    width = 252
    dates, R, y, _ = factor_panel(a.days, a.n)
    idx = pd.DatetimeIndex(dates)
    X = pd.DataFrame(R, index=idx, columns=[f"a{i}" for i in range(a.n)])
    Y = pd.DataFrame({"bm": y}, index=idx)
    rebdates = [str(d.date()) for d in idx[width - 1:][:a.dates]]
    for name, make in [("WeightedLeastSquares(tau=252)", lambda: WeightedLeastSquares(tau=252)),
                       ("LeastSquares", lambda: LeastSquares())]:
        def run():
            bt = Backtest()
            bt.run(service(make(), X, Y, rebdates, width))
            return bt
        run()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            bt = run()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / a.steps
        print(json.dumps({"objective": name, "n": a.n, "dates": len(rebdates), "s_per_run": dt,
                          "qps_per_s": len(rebdates) / dt, "path": bt.stats.get("path"),
                          "solved": bt.stats.get("solved")}), flush=True)


if __name__ == "__main__":
    main()
