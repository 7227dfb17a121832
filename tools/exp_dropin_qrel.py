#!/usr/bin/env python3
"""Backtest.run MeanVariance at the config-3 shape with rho0_qrel in {10, 30}: s per run.
Experiment tool."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from porqua_amd.backtest import Backtest  # noqa: E402
from tools.prof_dropin import mv3_service  # noqa: E402


def main():
    make = mv3_service()
    for qrel in (10.0, 30.0, 10.0, 30.0):
        svc = make()
        svc.optimization.params["rho0_qrel"] = qrel
        bt = Backtest()
        bt.run(svc)
        torch.cuda.synchronize()
        svc = make()
        svc.optimization.params["rho0_qrel"] = qrel
        t0 = time.perf_counter()
        bt = Backtest()
        bt.run(svc)
        torch.cuda.synchronize()
        print("rho0_qrel", qrel, "s", round(time.perf_counter() - t0, 4), "solved", bt.stats["solved"], flush=True)


if __name__ == "__main__":
    main()
