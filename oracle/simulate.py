"""CPU oracle for the strategy-simulation row -- TEST
INFRASTRUCTURE ONLY (see ``oracle/__init__.py``).

numpy restatement of ``floating_weights`` (``src/portfolio.py:259-296``),
``Strategy.simulate`` (``src/portfolio.py:209-248``, vc = 0) and the pairwise
``Portfolio.turnover`` (``src/portfolio.py:111-123``).  Pinned by
``tests/golden/msci_simulate.npz`` (``tools/capture_simulate.py`` ran the reference's own
``portfolio.py`` on the msci panel).
"""
from __future__ import annotations

import numpy as np


def period_rows(days: np.ndarray, start_day: int, end_day: int):
    """Rows of ``X.loc[start_date:end_date]`` (src/portfolio.py:283) on a sorted day index,
    with the range checks of src/portfolio.py:262-265."""
    if start_day < days[0]:
        raise ValueError("start_date must be contained in dataset")
    if end_day > days[-1]:
        raise ValueError("end_date must be contained in dataset")
    s = int(np.searchsorted(days, start_day, side="left"))
    e = int(np.searchsorted(days, end_day, side="right"))
    return s, e


def floating_weights(R: np.ndarray, w: np.ndarray, s: int, e: int, rescale: bool) -> np.ndarray:
    """src/portfolio.py:283-296: rows s..e-1 of the panel, NaN -> 0, row 0 replaced by the
    weights, cumulative product; optional rescale of the long and short books."""
    xm = 1.0 + np.nan_to_num(R[s:e], nan=0.0)
    xm[0] = w
    wf = np.cumprod(xm, axis=0)
    if rescale:
        pos = np.where(wf >= 0, wf, 0.0)
        neg = np.where(wf < 0, -wf, 0.0)
        sp = pos.sum(axis=1, keepdims=True)
        sn = neg.sum(axis=1, keepdims=True)
        with np.errstate(invalid="ignore", divide="ignore"):
            lo = np.where(wf >= 0, np.nan_to_num(wf / sp, nan=0.0), 0.0)
            sh = np.where(wf < 0, wf / sn, 0.0)
        wf = lo + sh
    return wf


def simulate(R: np.ndarray, days: np.ndarray, reb_days: np.ndarray, W: np.ndarray,
             fc: float = 0.0, n_days_per_year: int = 252):
    """src/portfolio.py:209-248 with vc = 0: returns (days, returns) of the concatenated
    level percentage changes, NaNs dropped, fixed cost on every return after the first."""
    out_d, out_r = [], []
    for i, d in enumerate(reb_days):
        nxt = reb_days[i + 1] if i + 1 < len(reb_days) else days[-1]
        s, e = period_rows(days, d, nxt)
        w = W[i]
        wf = floating_weights(R, w, s, e, rescale=False)
        L = w[w >= 0].sum()
        S = w[w < 0].sum()
        margin = abs(S)
        cash = max(min(1 - L, 1), 0)
        loan = 1 - (L + cash) - (S + margin)
        level = wf.sum(axis=1) + (loan + cash + margin)
        r = level[1:] / level[:-1] - 1.0
        keep = ~np.isnan(r)
        out_d.append(days[s + 1:e][keep])
        out_r.append(r[keep])
    dd = np.concatenate(out_d)
    rr = np.concatenate(out_r)
    if fc != 0:
        nd = np.diff(dd).astype(np.float64)
        rr[1:] -= (1 + fc) ** (nd / n_days_per_year) - 1
    return dd, rr


def turnover_pairs(R: np.ndarray, days: np.ndarray, reb_days: np.ndarray, W: np.ndarray,
                   rescale: bool):
    """Portfolio.turnover(previous) for every date after the first (src/portfolio.py:111-123):
    the previous weights floated to the current date (initial_weights, :88-109) minus the
    *previous* weights (the reference subtracts ``portfolio.weights``, the argument)."""
    ends, tos = [], []
    for i in range(1, len(reb_days)):
        s, e = period_rows(days, reb_days[i - 1], reb_days[i])
        we = floating_weights(R, W[i - 1], s, e, rescale)[-1]
        ends.append(we)
        tos.append(np.abs(we - W[i - 1]).sum())
    return np.array(ends), np.array(tos)
