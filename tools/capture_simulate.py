#!/usr/bin/env python3
"""Capture golden vectors for the strategy-simulation row from the
PorQua reference (run in the build container only).

Imports ``/root/reference/src/portfolio.py`` read-only (``sys.dont_write_bytecode``; that
module needs no solver) and records, on the msci panel (``tests/golden/msci_panel.npz``)
with the golden least-squares weights (``tests/golden/msci_ls.npz``) and a long/short
variant of them:

* ``Strategy.simulate(return_series, fc, vc=0)`` (``src/portfolio.py:209-248``) for
  fc in {0, 0.01};
* ``Portfolio.float_weights(..., rescale)`` end rows (``src/portfolio.py:74-86``,
  ``floating_weights`` ``:259-296``) for every consecutive pair of dates;
* ``Portfolio.turnover(previous, ..., rescale)`` (``src/portfolio.py:111-123``) for every
  date after the first, rescale in {False, True};
* whether ``Strategy.simulate(..., vc != 0)`` / ``Strategy.turnover`` raise (they do: the
  first date's empty previous portfolio reaches ``pd.to_datetime(None) > Timestamp``).

Usage:  python tools/capture_simulate.py
"""
from __future__ import annotations

import os
import sys
import warnings

import numpy as np
import pandas as pd

REF = "/root/reference"
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(REPO, "tests", "golden")

sys.dont_write_bytecode = True
sys.path.insert(0, os.path.join(REF, "src"))
warnings.simplefilter("ignore")

import portfolio as refp  # noqa: E402


def strategy(names, rebdates, W):
    return refp.Strategy([refp.Portfolio(rebalancing_date=d, weights=dict(zip(names, W[i])))
                          for i, d in enumerate(rebdates)])


def main():
    g = np.load(os.path.join(OUT, "msci_ls.npz"))
    p = np.load(os.path.join(OUT, "msci_panel.npz"))
    dates = pd.DatetimeIndex(p["dates"].astype("datetime64[D]"))
    names = [str(c) for c in p["columns"]]
    X = pd.DataFrame(p["returns"], index=dates, columns=names)
    reb = [str(d) for d in g["rebdates"]]
    W_long = np.asarray(g["x"], dtype=np.float64)
    rng = np.random.default_rng(7)
    # long/short variant: exercises margin, cash and loan (sum of longs != 1)
    W_ls = W_long + rng.normal(0.0, 0.05, W_long.shape)
    out = {"rebdates": np.array(reb), "W_long": W_long, "W_ls": W_ls}
    for tag, W in (("long", W_long), ("ls", W_ls)):
        for fc in (0.0, 0.01):
            r = strategy(names, reb, W).simulate(return_series=X, fc=fc, vc=0)
            key = f"sim_{tag}_fc{int(fc * 100)}"
            out[key + "_days"] = r.index.values.astype("datetime64[D]").astype(np.int64)
            out[key + "_ret"] = r.values.astype(np.float64)
        S = strategy(names, reb, W)
        for rescale in (False, True):
            ends, tos = [], []
            for i in range(1, len(reb)):
                prev, cur = S.portfolios[i - 1], S.portfolios[i]
                wf = prev.float_weights(return_series=X, end_date=cur.rebalancing_date, rescale=rescale)
                ends.append(wf.iloc[-1].values.astype(np.float64))
                # fresh objects: Portfolio.initial_weights caches its first answer
                a = refp.Portfolio(rebalancing_date=prev.rebalancing_date, weights=dict(prev.weights))
                b = refp.Portfolio(rebalancing_date=cur.rebalancing_date, weights=dict(cur.weights))
                tos.append(float(b.turnover(portfolio=a, return_series=X, rescale=rescale)))
            out[f"float_end_{tag}_r{int(rescale)}"] = np.array(ends)
            out[f"turnover_{tag}_r{int(rescale)}"] = np.array(tos)
    for what, fn in (("simulate_vc", lambda S: S.simulate(return_series=X, fc=0, vc=0.002)),
                     ("strategy_turnover", lambda S: S.turnover(return_series=X, rescale=False))):
        try:
            fn(strategy(names, reb, W_long))
            out[f"raises_{what}"] = np.array("")
        except Exception as e:  # noqa: BLE001 - the reference's own failure is the fixture
            out[f"raises_{what}"] = np.array(type(e).__name__)
    np.savez_compressed(os.path.join(OUT, "msci_simulate.npz"), **out)
    print({k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
