"""The covariance bar (north_star: within 1e-12 relative in FP64) at the CONFIG sizes:
n = 1000 (config 3) and n = 3000 (config 4) assets on 252-day windows, against the oracle's
np.cov restatement (oracle.ref_pipeline.cov_pearson, src/covariance.py:40-66).

* K1 (pq_cov_batched, full SYRK per date, and pq_cov_slide_batched, anchor SYRK + rank-2
  slides for consecutive daily windows) on every window of a short daily run;
* the API: Covariance.estimate (pearson, no PD repair requested; linear shrinkage, which is
  PD so nothing is repaired; the default spec, which finds the rank-deficient n > T
  covariance non-PD and runs nearestPD on the device, src/helper_functions.py:29-58);
* windows with missing values at n = 1000: pandas' pairwise-complete covariance
  (pq_cov_pairwise_batched) against the vectorised oracle restatement (cov_pairwise_rows,
  pinned to the reference's fixtures by tests/test_oracle_golden.py).

Relative error = Frobenius norm of the difference over that of the oracle."""
import numpy as np
import pandas as pd
import pytest

from oracle import ref_pipeline as rp
from porqua_amd import engine
from porqua_amd.covariance import Covariance
from porqua_amd.synthetic import factor_panel

pytestmark = pytest.mark.gpu

T = 252


def _rel(a, b):
    return np.linalg.norm(a - b) / np.linalg.norm(b)


@pytest.mark.parametrize("n", [1000, 3000])
def test_k1_covariance_at_config_size(device, n):
    nd = 4
    dates, R, _, _ = factor_panel(T - 1 + nd, n)
    rows, tlen = engine.window_rows(dates, dates[T - 1:], T)
    assert (tlen == T).all() and len(tlen) == nd
    pan = engine.Panel(R, device=device)
    r_d, t_d = pan.rows_to_device(rows, tlen)
    full = pan.cov(r_d, t_d, mode=0)
    plan = engine.SlidePlan(rows, tlen, device, group=16)
    assert plan.ngroups == 1                                     # one anchor + 3 slid dates
    slid = pan.cov(r_d, t_d, mode=0, plan=plan)
    for b in range(nd):
        ref = rp.cov_pearson(R[rows[b]])
        f = full[b, :n, :n].cpu().numpy()
        s = slid[b, :n, :n].cpu().numpy()
        assert _rel(f, ref) <= 1e-12, (n, b, _rel(f, ref))
        assert _rel(s, ref) <= 1e-12, (n, b, _rel(s, ref))
        assert np.array_equal(f, f.T)


@pytest.mark.parametrize("n", [1000, 3000])
def test_covariance_estimate_at_config_size(device, n):
    dates, R, _, _ = factor_panel(T, n, seed=n)
    X = pd.DataFrame(R, columns=[f"a{i}" for i in range(n)])
    S = Covariance(method="pearson", check_positive_definite=False).estimate(X)
    assert list(S.index) == list(X.columns)
    assert _rel(S.to_numpy(), rp.cov_pearson(R)) <= 1e-12
    S = Covariance(method="linear_shrinkage", lambda_covmat_regularization=0.1).estimate(X).to_numpy()
    ref = rp.cov_linear_shrinkage(R, 0.1)
    assert rp.is_pd(ref) and _rel(S, ref) <= 1e-12


def test_covariance_estimate_with_repair_at_config3_size(device):
    """The default spec at n = 1000 > T: the sample covariance has rank T - 1, K2's isPD
    fails and nearestPD repairs it on the device (Jacobi eigensolver + shift loop); the
    reference-restated repair adds ~1e-18 to the spectrum, so the repaired matrix stays
    within the covariance bar of the oracle's."""
    n = 1000
    dates, R, _, _ = factor_panel(T, n, seed=7)
    X = pd.DataFrame(R)
    S = Covariance().estimate(X).to_numpy()
    ref = rp.covariance_estimate(R)
    assert not rp.is_pd(rp.cov_pearson(R))
    assert _rel(S, ref) <= 1e-12, _rel(S, ref)
    assert rp.is_pd(S)


def test_pairwise_nan_covariance_at_config3_size(device):
    n = 1000
    dates, R, _, _ = factor_panel(T + 10, n, seed=11)
    rng = np.random.default_rng(11)
    R = R.copy()
    R[rng.random(R.shape) < 0.02] = np.nan                        # 2 % of the returns missing
    R[:40, :25] = np.nan                                          # late listings
    rows, tlen = engine.window_rows(dates, dates[[T - 1, T + 9]], T)
    pan = engine.Panel(R, device=device)
    r_d, t_d = pan.rows_to_device(rows, tlen)
    S = pan.cov_pairwise(r_d, t_d).cpu().numpy()
    for b in range(2):
        ref = rp.cov_pairwise_rows(R[rows[b]])
        got = S[b, :n, :n]
        assert np.array_equal(np.isnan(got), np.isnan(ref))
        ok = ~np.isnan(ref)
        assert np.linalg.norm(got[ok] - ref[ok]) <= 1e-12 * np.linalg.norm(ref[ok])
