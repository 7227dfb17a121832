# Host-side API restatement of PorQua (part of the GeomScale project; reference tree
# amolrpatil21/PorQua): src/mean_estimation.py.  PorQua is Copyright (c) 2024 Cyril Bachelard and
# Minh Ha Ho and licensed under the GNU LGPL v3; this module keeps that API and its
# behaviour (quirks included) so that the MI355X engine is a drop-in, and is distributed
# under the same licence terms.
"""Geometric mean estimator (mirror of src/mean_estimation.py:23-48), on the device."""
from __future__ import annotations

import numpy as np
import pandas as pd


class MeanEstimator:

    def __init__(self, **kwargs) -> None:
        self.spec = {"method": "geometric", "scalefactor": 1, "n_mom": None, "n_rev": None}
        self.spec.update(kwargs)

    def estimate(self, X: pd.DataFrame):
        fun = getattr(self, f"estimate_{self.spec['method']}")
        return fun(X=X)

    def window(self, T: int):
        """Row range [start, stop) of the T-row window that enters the estimate:
        X.tail(n_mom).head(n_mom - n_rev) (src/mean_estimation.py:40-45)."""
        n_mom = T if self.spec.get("n_mom") is None else int(self.spec["n_mom"])
        n_rev = 0 if self.spec.get("n_rev") is None else int(self.spec["n_rev"])
        start = max(0, T - n_mom)
        stop = start + max(0, min(n_mom, T) - n_rev) if n_mom > 0 else start
        return start, max(start, stop)

    def estimate_geometric(self, X: pd.DataFrame):
        """exp(mean(log(1 + X)) * scalefactor) - 1 with the K1 window-reduction kernel."""
        from . import engine
        sf = self.spec.get("scalefactor")
        sf = 1 if sf is None else sf
        Xv = np.ascontiguousarray(X.to_numpy() if hasattr(X, "to_numpy") else X, dtype=np.float64)
        T, n = Xv.shape
        a, b = self.window(T)
        pan = engine.Panel(Xv[a:b] if b > a else np.zeros((1, n)))
        L = b - a
        rows, tlen = pan.rows_to_device(np.arange(max(L, 1), dtype=np.int32)[None],
                                        np.array([L], dtype=np.int32))
        if L == 0:
            mu = np.full(n, np.nan)
        else:
            if isinstance(X, pd.DataFrame) and np.isnan(Xv[a:b]).any():   # pandas mean: skipna
                g = pan.window_nanmeans(rows, tlen, geometric=True)[0, :n].cpu().numpy()
            else:
                g = pan.window_means(rows, tlen, geometric=True)[0, :n].cpu().numpy()
            mu = g if sf == 1 else np.exp(np.log1p(g) * sf) - 1
        if isinstance(X, pd.DataFrame):
            return pd.Series(mu, index=X.columns)
        return mu
