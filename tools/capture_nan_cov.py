#!/usr/bin/env python3
"""Golden vectors for windows with missing values: the reference's Covariance.estimate and
raw DataFrame.cov() (pandas' pairwise-complete covariance, src/covariance.py:40-56,65-66)
on NaN-bearing windows -> tests/golden/nan_cov.npz.

Imports /root/reference/src read-only (sys.dont_write_bytecode) in the build container
only; the GPU tests read the fixture.  Cases: assets entering late / leaving early / holes on
the real msci panel (n = 24 < T, PD), the same with linear shrinkage, and a synthetic n = 80 >
T = 60 window (pairwise covariance not PD: Covariance.estimate repairs it with nearestPD), plus
a raw-only case where one pair has fewer than 2 common rows (NaN entries).
Test infrastructure only:  python tools/capture_nan_cov.py"""
import os
import sys
import warnings

import numpy as np
import pandas as pd

REF = "/root/reference"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.dont_write_bytecode = True
sys.path.insert(0, os.path.join(REF, "src"))
sys.path.insert(0, ROOT)
warnings.simplefilter("ignore")

from covariance import Covariance  # noqa: E402  (reference)


def msci_window():
    X = pd.read_csv(os.path.join(REF, "data", "msci_country_indices.csv"), index_col=0)
    X.index = pd.to_datetime(X.index, format="%d-%m-%Y")
    return X.astype(float).sort_index().iloc[1000:1252].copy()   # the file holds returns


def main():
    rng = np.random.default_rng(7)
    out = {}
    W = msci_window()
    W.iloc[:100, 3] = np.nan            # enters late
    W.iloc[-50:, 7] = np.nan            # leaves early
    for c in (10, 11, 12):              # holes
        W.iloc[rng.random(len(W)) < 0.02, c] = np.nan
    out["msci_holes__X"] = W.to_numpy()
    out["msci_holes__raw"] = W.cov().to_numpy()
    out["msci_holes__est"] = Covariance(method="pearson").estimate(W).to_numpy()
    out["msci_holes__shrink"] = Covariance(method="linear_shrinkage",
                                           lambda_covmat_regularization=0.1).estimate(W).to_numpy()
    from porqua_amd.synthetic import factor_panel
    _, R, _, _ = factor_panel(60, 80, seed=5)
    Z = pd.DataFrame(R)
    for j in range(0, 80, 7):
        Z.iloc[:int(rng.integers(5, 30)), j] = np.nan   # staggered entries
    Z.iloc[-10:, 5] = np.nan
    out["wide__X"] = Z.to_numpy()
    out["wide__raw"] = Z.cov().to_numpy()
    out["wide__est"] = Covariance(method="pearson").estimate(Z).to_numpy()
    V = pd.DataFrame(rng.normal(0, 0.01, size=(40, 6)))
    V.iloc[:39, 2] = np.nan                 # one observation: its column / row is NaN
    V.iloc[20:, 4] = np.nan
    V.iloc[:21, 5] = np.nan                 # columns 4 and 5 share no row
    out["sparse__X"] = V.to_numpy()
    out["sparse__raw"] = V.cov().to_numpy()
    np.savez_compressed(os.path.join(ROOT, "tests", "golden", "nan_cov.npz"), **out)
    for k, v in out.items():
        print(k, v.shape, int(np.isnan(v).sum()), file=sys.stderr)


if __name__ == "__main__":
    main()
