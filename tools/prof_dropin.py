#!/usr/bin/env python3
"""cProfile of the drop-in path: Backtest.run(solver_name='mi355x') after one warm-up run --
default: the usa-shaped panel, every date (configs 1/2 shape); ``mv3``: bench.py's end-to-end
line (MeanVariance, config-3 synthetic panel, 4749 daily dates); ``monthly``: config 2 as the
reference notebook runs it (13 monthly dates).  Experiment tooling."""
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


def mv3_service():
    import pandas as pd
    from porqua_amd.backtest import BacktestService
    from porqua_amd.builders import (OptimizationItemBuilder, SelectionItemBuilder, bibfn_box_constraints,
                                     bibfn_budget_constraint, bibfn_return_series, bibfn_selection_data)
    from porqua_amd.optimization import MeanVariance
    from porqua_amd.synthetic import factor_panel
    T, n, D = 252, 1000, 4749
    dates, R, _, _ = factor_panel(T - 1 + D, n)
    idx = pd.DatetimeIndex(dates)
    Xdf = pd.DataFrame(R, index=idx, columns=[f"a{i}" for i in range(n)])
    reb = [str(d.date()) for d in idx[T - 1:]]
    return lambda: BacktestService(
        data={"return_series": Xdf},
        selection_item_builders={"data": SelectionItemBuilder(bibfn=bibfn_selection_data)},
        optimization_item_builders={
            "return_series": OptimizationItemBuilder(bibfn=bibfn_return_series, width=T),
            "budget_constraint": OptimizationItemBuilder(bibfn=bibfn_budget_constraint, budget=1),
            "box_constraints": OptimizationItemBuilder(bibfn=bibfn_box_constraints)},
        optimization=MeanVariance(solver_name="mi355x"), rebdates=reb, quiet=True)


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "mv3":
        make = mv3_service()
    elif len(sys.argv) > 1 and sys.argv[1] == "monthly":   # config 2 as the notebook runs it: 13 dates
        X, y = usa_data()
        d = X.index.values.astype("datetime64[D]")
        reb = [str(r) for r in d[d > np.datetime64("2022-06-01")][::21]]
        make = lambda: service(X, y, reb)  # noqa: E731
    else:
        X, y = usa_data()
        d = X.index.values.astype("datetime64[D]")
        reb = [str(r) for r in d[251:]]
        make = lambda: service(X, y, reb)  # noqa: E731

    def run():
        bt = Backtest()
        bt.run(make())
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
