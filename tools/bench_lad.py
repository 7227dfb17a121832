#!/usr/bin/env python3
"""LAD (src/optimization.py:263-345) throughput through Backtest.run on the config-3 shape:
synthetic 5000 x 1000 panel, 252-day windows, daily rebalance, budget + long-only box.
--dates limits the number of rebalance dates.  Prints one JSON line (LPs/s, IPM iterations).
Experiment tooling; the number is quoted in DESIGN.md."""
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
sys.path.insert(0, os.path.join(ROOT, "tools"))
from bench_wls import service  # noqa: E402
from porqua_amd.backtest import Backtest  # noqa: E402
from porqua_amd.optimization import LAD  # noqa: E402
from porqua_amd.synthetic import factor_panel  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1000)
    ap.add_argument("--days", type=int, default=5000)
    ap.add_argument("--dates", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=1)
    a = ap.parse_args()
    width = 252
    dates, R, y, _ = factor_panel(a.days, a.n)
    idx = pd.DatetimeIndex(dates)
    X = pd.DataFrame(R, index=idx, columns=[f"a{i}" for i in range(a.n)])
    Y = pd.DataFrame({"bm": y}, index=idx)
    rebdates = [str(d.date()) for d in idx[width - 1:][:a.dates]]

    def run():
        bt = Backtest()
        bt.run(service(LAD(), X, Y, rebdates, width))
        return bt
    run()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        bt = run()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.steps
    st = bt.stats["status"]
    print(json.dumps({"objective": "LAD (use_level, use_log)", "n": a.n, "dates": len(rebdates),
                      "s_per_run": dt, "lps_per_s": len(rebdates) / dt, "path": bt.stats.get("path"),
                      "status_counts": {str(k): int(v) for k, v in zip(*np.unique(st, return_counts=True))}}),
          flush=True)


if __name__ == "__main__":
    main()
