#!/usr/bin/env python3
"""SPTR benchmark fixture for configs 1/2 (BASELINE.json configs[0..1]): the real S&P 500
total-return daily returns the reference ships as data/SPTR.csv (read as the reference's
example/backtest.ipynb does: index_col=0, dates '%d/%m/%Y') -> tests/golden/sptr.npz
(dates as datetime64[D] day numbers, returns).  The GPU box has no /root/reference, so the
tests read the fixture.  Test infrastructure only:  python tools/capture_sptr.py"""
import os
import sys

import numpy as np
import pandas as pd

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = "/root/reference/data/SPTR.csv"


def main():
    s = pd.read_csv(SRC, index_col=0)
    s.index = pd.to_datetime(s.index, format="%d/%m/%Y")
    v = s.iloc[:, 0].to_numpy(dtype=np.float64)
    days = s.index.values.astype("datetime64[D]").astype(np.int64)
    assert np.all(np.diff(days) > 0) and np.isfinite(v).all()
    np.savez_compressed(os.path.join(ROOT, "tests", "golden", "sptr.npz"), days=days, returns=v,
                        name=np.array(str(s.columns[0])))
    print(len(v), s.index[0].date(), s.index[-1].date(), file=sys.stderr)


if __name__ == "__main__":
    main()
