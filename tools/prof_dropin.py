#!/usr/bin/env python3
"""cProfile of the drop-in path: Backtest.run(solver_name='mi355x') on the usa-shaped panel,
every date (configs 1/2 shape), after one warm-up run.  Experiment tooling."""
import cProfile
import os
import pstats
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
    reb = [str(r) for r in d[251:]]

    def run():
        bt = Backtest()
        bt.run(service(X, y, reb))
        torch.cuda.synchronize()
        return bt
    run()
    t0 = time.perf_counter()
    run()
    print("run s", time.perf_counter() - t0, flush=True)
    pr = cProfile.Profile()
    pr.enable()
    run()
    pr.disable()
    st = pstats.Stats(pr)
    st.sort_stats("cumulative").print_stats(40)
    st.sort_stats("tottime").print_stats(25)


if __name__ == "__main__":
    main()
