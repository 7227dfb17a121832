"""Windows with missing values on the device: Covariance.estimate / DataFrame.cov() semantics
(pandas' pairwise-complete covariance, src/covariance.py:40-56,65-66) from the masked MFMA
Grams of pq_cov_pairwise_batched, against fixtures captured from the reference
(tools/capture_nan_cov.py): raw covariance <= 1e-12 relative with the reference's NaN
pattern, and the estimate after the PD check / nearestPD repair."""
import numpy as np
import pandas as pd
import pytest

from oracle import ref_pipeline as rp
from porqua_amd.covariance import Covariance, cov_pearson
from tests.conftest import load_golden

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return np.abs(a - b).max() / np.abs(b).max()


@pytest.mark.parametrize("case", ["msci_holes", "wide", "sparse"])
def test_pairwise_cov_matches_reference(device, case):
    g = load_golden("nan_cov")
    X = pd.DataFrame(g[f"{case}__X"])
    S = cov_pearson(X).to_numpy()
    ref = g[f"{case}__raw"]
    assert np.array_equal(np.isnan(S), np.isnan(ref))
    ok = ~np.isnan(ref)
    assert np.abs(S[ok] - ref[ok]).max() <= 1e-12 * np.abs(ref[ok]).max()


def test_covariance_estimate_with_nan_matches_reference(device):
    g = load_golden("nan_cov")
    X = pd.DataFrame(g["msci_holes__X"])
    assert _rel(Covariance(method="pearson").estimate(X).to_numpy(), g["msci_holes__est"]) <= 1e-12
    S = Covariance(method="linear_shrinkage", lambda_covmat_regularization=0.1).estimate(X).to_numpy()
    assert _rel(S, g["msci_holes__shrink"]) <= 1e-12
    # n = 80 > T = 60: the pairwise covariance is not PD and Covariance.estimate repairs it
    W = pd.DataFrame(g["wide__X"])
    assert not rp.is_pd(g["wide__raw"])
    est = Covariance(method="pearson").estimate(W).to_numpy()
    assert rp.is_pd(est)
    assert _rel(est, g["wide__est"]) <= 1e-9


def test_pairwise_cov_large_window_matches_oracle(device):
    """n = 300 assets with staggered entries / exits over a 252-row window (several 64-wide
    tiles, odd remainder) against the oracle restatement."""
    from porqua_amd.synthetic import factor_panel
    rng = np.random.default_rng(3)
    _, R, _, _ = factor_panel(252, 300, seed=9)
    R = R.copy()
    for j in range(300):
        r = rng.random()
        if r < 0.2:
            R[:int(rng.integers(1, 200)), j] = np.nan
        elif r < 0.3:
            R[-int(rng.integers(1, 200)):, j] = np.nan
    S = cov_pearson(pd.DataFrame(R)).to_numpy()
    ref = rp.cov_pairwise(R)
    assert np.array_equal(np.isnan(S), np.isnan(ref))
    ok = ~np.isnan(ref)
    assert np.abs(S[ok] - ref[ok]).max() <= 1e-12 * np.abs(ref[ok]).max()
