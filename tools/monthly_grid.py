#!/usr/bin/env python3
"""The reference notebook's monthly run (config 2 shape, 13 dates through Backtest.run) under
settings variants: wall time (median of 5 after a warm-up) and the largest weight / objective
difference from the default settings' answers (experiment tooling).
Usage: monthly_grid.py '{"eps_grouped_tracking": 0.01}' ..."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from porqua_amd.backtest import Backtest  # noqa: E402
from tests.test_configs12_gpu import service, usa_data  # noqa: E402


def main():
    X, y = usa_data()
    d = X.index.values.astype("datetime64[D]")
    reb = [str(r) for r in d[d > np.datetime64("2022-06-01")][::21]]
    ref = None
    for spec in ["{}"] + sys.argv[1:]:
        params = json.loads(spec)

        def run():
            bt = Backtest()
            bt.run(service(X, y, reb, params=params))
            torch.cuda.synchronize()
            return bt
        run()
        ts = []
        for _ in range(5):
            t0 = time.perf_counter()
            bt = run()
            ts.append(time.perf_counter() - t0)
        W = bt.strategy.get_weights_df().to_numpy(dtype=float)
        obj = np.asarray(bt.stats["objective"], dtype=float)
        if ref is None:
            ref = (W, obj)
        dw = np.abs(W - ref[0]).max()
        dob = np.abs(obj - ref[1]).max() / max(1e-300, np.abs(ref[1]).max())
        print(f"{spec:45s} run {np.median(ts) * 1e3:7.2f} ms  solved {bt.stats['solved']}/{len(reb)}  "
              f"max|dW| {dw:.1e}  max rel dobj {dob:.1e}", flush=True)


if __name__ == "__main__":
    main()
