#!/usr/bin/env python3
"""Config-5 sweep variants (capacitance factor form x group size): QPs/s, iterations,
factorisations.  Experiment tool:  python tools/exp_sweep.py  (ND dates, default 16)"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from porqua_amd import engine  # noqa: E402
from porqua_amd.sweep import mean_variance_sweep  # noqa: E402
from porqua_amd.synthetic import factor_panel  # noqa: E402


def main():
    n, T, nd, L = 5000, 252, int(os.environ.get("ND", "16")), 64
    dates, R, _, _ = factor_panel(T - 1 + 21 * nd, n)
    ends = np.arange(T - 1, T - 1 + 21 * nd, 21)
    rows, tlen = engine.window_rows(dates, dates[ends], T)
    pan = engine.Panel(R, device=torch.device("cuda", 0))
    lambdas = np.logspace(-1, 2, L)
    for factor, gmax in (("chol", 16), ("eig", 16)):
        st = engine.Settings()
        mean_variance_sweep(pan, rows, tlen, lambdas, factor=factor, gmax=gmax, settings=st)
        torch.cuda.synchronize()
        ev = []
        t0 = time.perf_counter()
        res, meta = mean_variance_sweep(pan, rows, tlen, lambdas, factor=factor, gmax=gmax, settings=st, events=ev)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        stages = {}
        for name, e0, e1 in ev:
            stages[name] = round(stages.get(name, 0.0) + e0.elapsed_time(e1), 3)
        it = res.iters.cpu().numpy()
        print(json.dumps({"factor": factor, "gmax": gmax, "qps": nd * L / dt, "s": dt, "stage_ms": stages,
                          "iters_mean": float(it.mean()), "iters_max": int(it.max()),
                          "factorizations": meta["factorizations"], "capacitance": meta["capacitance"],
                          "status": {str(k): int(v) for k, v in zip(*np.unique(res.status.cpu().numpy(),
                                                                                return_counts=True))}}),
              flush=True)


if __name__ == "__main__":
    main()
