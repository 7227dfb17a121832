# Host-side API restatement of PorQua (part of the GeomScale project; reference tree
# amolrpatil21/PorQua): src/covariance.py.  PorQua is Copyright (c) 2024 Cyril Bachelard and
# Minh Ha Ho and licensed under the GNU LGPL v3; this module keeps that API and its
# behaviour (quirks included) so that the MI355X engine is a drop-in, and is distributed
# under the same licence terms.
"""Covariance estimation on the device (mirror of src/covariance.py:21-84).

``Covariance.estimate(X)`` keeps the reference signature (T x n DataFrame in, n x n
DataFrame out) and computes the two-pass np.cov / DataFrame.cov() result with K1
(window mean + FP64-MFMA SYRK; windows with NaN: pandas' pairwise-complete covariance from
four masked MFMA Grams), the PD check with K2's Cholesky info and the repair with
``helper_functions.nearestPD``.  ``estimate_batch`` is the batched backtest entry: all
rebalance dates of a device-resident panel at once, results left on the device.
"""
from __future__ import annotations

import numpy as np
import pandas as pd

from .helper_functions import isPD, nearestPD


class CovarianceSpecification(dict):
    """Defaults: method 'pearson', check_positive_definite True (src/covariance.py:21-28)."""

    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self.__dict__ = self
        self.setdefault("method", "pearson")
        if self.get("method") is None:
            self["method"] = "pearson"
        if self.get("check_positive_definite") is None:
            self["check_positive_definite"] = True


def _shrink_lambda(lam):
    if lam is None or np.isnan(lam) or lam < 0:
        return 0.0
    return float(lam)


class Covariance:

    def __init__(self, spec: CovarianceSpecification = None, *args, **kwargs):
        self.spec = CovarianceSpecification(*args, **kwargs) if spec is None else spec

    def set_ctrl(self, *args, **kwargs) -> None:
        self.spec = CovarianceSpecification(*args, **kwargs)

    def estimate(self, X: pd.DataFrame):
        method = self.spec["method"]
        if method == "pearson":
            covmat = cov_pearson(X)
        elif method == "duv":
            covmat = cov_duv(X)
        elif method == "linear_shrinkage":
            covmat = cov_linear_shrinkage(X, self.spec.get("lambda_covmat_regularization"))
        else:
            raise NotImplementedError("This method is not implemented yet")
        if self.spec.get("check_positive_definite") and not isPD(covmat):
            fixed = nearestPD(covmat)
            covmat = pd.DataFrame(fixed, index=covmat.index, columns=covmat.columns) \
                if isinstance(covmat, pd.DataFrame) else fixed
        return covmat

    def _estimate_batch_pairwise(self, panel, rows, tlen, out, method):
        r = _pairwise_batch(panel, rows, tlen, out, method, self.spec.get("lambda_covmat_regularization"),
                            bool(self.spec.get("check_positive_definite")))
        return (None, None, None, None) if r is None else r

    # -- batched (backtest) entry --------------------------------------------------------
    def estimate_batch(self, panel, rows, tlen, out=None, plan=None, lower_only=False):
        """All dates at once on the device.  Returns (S, p_diag): S is the (B, ld, ld)
        device tensor of raw sample covariances; p_diag (B,) is the diagonal term the spec
        adds (linear shrinkage: lam * mean(diag S)); 'duv' returns (None, None)."""
        S, pdiag, _, _ = self.estimate_batch_lr(panel, rows, tlen, out=out, plan=plan, lower_only=lower_only)
        return S, pdiag

    def estimate_batch_lr(self, panel, rows, tlen, out=None, plan=None, lower_only=False,
                          materialise=True, groups=None):
        """estimate_batch plus the window means (the centring of the factored form
        S = Xc'Xc / (T-1) that the low-rank solver uses) -> (S, p_diag, mu, dg).
        ``plan``: an engine.SlidePlan for overlapping windows; ``lower_only``: lower-triangle
        storage.  ``materialise=False`` (the window-form solver, which never reads an n x n
        S): S is None and dg = diag(Xc'Xc) per date carries what the shrinkage term needs."""
        import torch
        method = self.spec["method"]
        if method == "duv":
            return None, None, None, None
        if method not in ("pearson", "linear_shrinkage"):
            raise NotImplementedError("This method is not implemented yet")
        B, n = int(rows.shape[0]), panel.n
        if panel.has_nan:
            return self._estimate_batch_pairwise(panel, rows, tlen, out, method)
        S = dg = None
        if not materialise and groups is not None and groups.ok:
            # the window form with slide groups (engine.GroupPlan): means and diag(Xc'Xc) of
            # every window in one sliding pass per group instead of two passes per window
            ld = ((n + 63) // 64) * 64
            mu = torch.zeros((B, ld), dtype=torch.float64, device=panel.device)
            dg = torch.zeros((B, ld), dtype=torch.float64, device=panel.device)
            panel.window_moments_grouped(groups, tlen, mu, dg)
        else:
            mu = panel.window_means(rows, tlen)
            if materialise:
                S = panel.cov(rows, tlen, mode=0, out=out, mu=mu, plan=plan,
                              lower_only=lower_only and plan is not None)
            else:
                dg = panel.window_sumsq(rows, tlen, mu)
        pdiag = torch.zeros(B, dtype=torch.float64, device=mu.device)
        if method == "linear_shrinkage":
            lam = _shrink_lambda(self.spec.get("lambda_covmat_regularization"))
            if lam > 0:
                if S is not None:
                    pdiag = lam * torch.diagonal(S, dim1=1, dim2=2)[:, :n].mean(dim=1)
                else:   # mean(diag S) = mean(diag Xc'Xc) / (T - 1)
                    pdiag = lam * dg[:, :n].mean(dim=1) / (tlen.to(torch.float64) - 1.0)
        return S, pdiag, mu, dg


def _pairwise_batch(panel, rows, tlen, out, method, lam_raw, check_pd):
    """Windows with missing values, all dates at once: pairwise-complete covariance
    (pq_cov_pairwise_batched), the linear-shrinkage term, then Covariance.estimate's PD check
    and nearestPD repair for the dates that need it (src/covariance.py:50-54) -> (S, 0, None,
    None); None when some pair has fewer than 2 common rows (the reference fails there too)."""
    import torch
    from .helper_functions import nearestPD_device, pd_info_device
    S = panel.cov_pairwise(rows, tlen, out=out)
    n = panel.n
    if bool(torch.isnan(S[:, :n, :n]).any().item()):
        return None
    B = S.shape[0]
    idx = torch.arange(n, device=S.device)
    if method == "linear_shrinkage":
        lam = _shrink_lambda(lam_raw)
        if lam > 0:
            md = torch.diagonal(S, dim1=1, dim2=2)[:, :n].mean(dim=1)
            S[:, idx, idx] += (lam * md)[:, None]
    if check_pd:   # on the device: K2 info for every date, the repair for the failing ones only
        bad = torch.nonzero(pd_info_device(S, n) != 0).flatten()
        if bad.numel():
            S[bad, :n, :n] = nearestPD_device(S[bad], n)[:, :n, :n]
    return S, torch.zeros(B, dtype=torch.float64, device=S.device), None, None


def _device_cov(X, mode=0):
    from . import engine
    Xv = np.ascontiguousarray(X.to_numpy() if hasattr(X, "to_numpy") else X, dtype=np.float64)
    T, n = Xv.shape
    pan = engine.Panel(Xv)
    rows, tlen = pan.rows_to_device(np.arange(T, dtype=np.int32)[None], np.array([T], dtype=np.int32))
    if mode == 0 and np.isnan(Xv).any():
        # missing values: pandas' pairwise-complete DataFrame.cov() (pq_cov_pairwise_batched)
        S = pan.cov_pairwise(rows, tlen)
    else:
        S = pan.cov(rows, tlen, mode=mode)
    return S[0, :n, :n].cpu().numpy()


def cov_pearson(X):
    """X.cov() (src/covariance.py:65-66) on the device."""
    S = _device_cov(X, mode=0)
    if isinstance(X, pd.DataFrame):
        return pd.DataFrame(S, index=X.columns, columns=X.columns)
    return S


def cov_duv(X):
    """Identity, returned as an ndarray like the reference (src/covariance.py:68-69)."""
    return np.identity(X.shape[1])


def cov_linear_shrinkage(X, lambda_covmat_regularization=None):
    """Sigma + lambda * mean(diag Sigma) * I (src/covariance.py:71-84); the reference's
    unused correlation loop (:78-82) is not reproduced (it has no effect on the result)."""
    lam = _shrink_lambda(lambda_covmat_regularization)
    S = cov_pearson(X)
    if lam > 0:
        vals = S.to_numpy() if isinstance(S, pd.DataFrame) else S
        d = vals.shape[0]
        vals = vals + lam * np.mean(np.diag(vals)) * np.eye(d)
        S = pd.DataFrame(vals, index=S.index, columns=S.columns) if isinstance(S, pd.DataFrame) else vals
    return S
