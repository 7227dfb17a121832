# Host-side API restatement of PorQua (part of the GeomScale project; reference tree
# amolrpatil21/PorQua): src/portfolio.py.  PorQua is Copyright (c) 2024 Cyril Bachelard and
# Minh Ha Ho and licensed under the GNU LGPL v3; this module keeps that API and its
# behaviour (quirks included) so that the MI355X engine is a drop-in, and is distributed
# under the same licence terms.
"""Portfolio / Strategy containers (mirror of src/portfolio.py:20-296).

The rebalance loop fills these; ``Strategy.simulate`` and ``Strategy.turnover_pairs`` float
every holding period on the device in one launch (``engine.simulate_periods`` ->
``pq_simulate_periods``).  ``Portfolio.float_weights`` /
``initial_weights`` / ``turnover`` are the reference's single-pair helpers and stay on the
host (pandas, one period at a time), as does ``floating_weights``.
"""
from __future__ import annotations

import numpy as np
import pandas as pd


class Portfolio:

    def __init__(self, rebalancing_date: str = None, weights: dict = None, name: str = None,
                 init_weights: dict = None):
        self.rebalancing_date = rebalancing_date
        self.weights = {} if weights is None else weights
        self.name = name
        self.init_weights = {} if init_weights is None else init_weights

    @staticmethod
    def empty() -> "Portfolio":
        return Portfolio()

    @classmethod
    def _from_row(cls, rebalancing_date: str, keys: list, row: np.ndarray) -> "Portfolio":
        """A portfolio of the batched backtest: the weights stay a row of the solved weight
        panel until first read, then become the reference's {asset: float} dict (cached)."""
        p = cls.__new__(cls)
        p.rebalancing_date = rebalancing_date
        p._name = None
        p.init_weights = {}
        p._weights = None
        p._row = (keys, row)
        return p

    @property
    def weights(self):
        if self._weights is None and getattr(self, "_row", None) is not None:
            keys, row = self._row
            self._weights = dict(zip(keys, row.tolist()))
            self._row = None
        return self._weights

    @weights.setter
    def weights(self, new_weights):
        if not isinstance(new_weights, dict):
            if hasattr(new_weights, "to_dict"):
                new_weights = new_weights.to_dict()
            else:
                raise TypeError("weights must be a dictionary")
        self._weights = new_weights
        self._row = None

    @property
    def rebalancing_date(self):
        return self._rebalancing_date

    @rebalancing_date.setter
    def rebalancing_date(self, new_date):
        if new_date and not isinstance(new_date, str):
            raise TypeError("date must be a string")
        self._rebalancing_date = new_date

    @property
    def name(self):
        return self._name

    @name.setter
    def name(self, new_name):
        if new_name is not None and not isinstance(new_name, str):
            raise TypeError("name must be a string")
        self._name = new_name

    def get_weights_series(self) -> pd.Series:
        return pd.Series(self.weights)

    def __repr__(self):
        return f"Portfolio(rebalancing_date={self.rebalancing_date}, weights={self.weights})"

    def float_weights(self, return_series: pd.DataFrame, end_date: str, rescale: bool = False):
        """src/portfolio.py:74-86."""
        if self.weights is not None:
            return floating_weights(X=return_series, w=self.weights, start_date=self.rebalancing_date,
                                    end_date=end_date, rescale=rescale)
        return None

    def initial_weights(self, selection, return_series: pd.DataFrame, end_date: str,
                        rescale: bool = True):
        """src/portfolio.py:88-109, including its cache: the first answer is kept."""
        if not hasattr(self, "_initial_weights"):
            if self.rebalancing_date is not None and self.weights is not None:
                w_init = dict.fromkeys(selection, 0)
                w_floated = self.float_weights(return_series=return_series, end_date=end_date,
                                               rescale=rescale).iloc[-1]
                w_init.update({k: w_floated[k] for k in w_init.keys() & w_floated.keys()})
                self._initial_weights = w_init
            else:
                self._initial_weights = None
        return self._initial_weights

    def turnover(self, portfolio: "Portfolio", return_series: pd.DataFrame, rescale=True):
        """src/portfolio.py:111-123 (the floated weights are compared with the *argument's*
        weights, as in the reference)."""
        if portfolio.rebalancing_date is not None and portfolio.rebalancing_date < self.rebalancing_date:
            w_init = portfolio.initial_weights(selection=self.weights.keys(), return_series=return_series,
                                               end_date=self.rebalancing_date, rescale=rescale)
        else:
            w_init = self.initial_weights(selection=portfolio.weights.keys(), return_series=return_series,
                                          end_date=portfolio.rebalancing_date, rescale=rescale)
        return pd.Series(w_init).sub(pd.Series(portfolio.weights), fill_value=0).abs().sum()


class Strategy:

    def __init__(self, portfolios: list):
        self.portfolios = portfolios

    @property
    def portfolios(self):
        return self._portfolios

    @portfolios.setter
    def portfolios(self, new_portfolios):
        if not isinstance(new_portfolios, list):
            raise TypeError("portfolios must be a list")
        if not all(isinstance(p, Portfolio) for p in new_portfolios):
            raise TypeError("all elements in portfolios must be of type Portfolio")
        self._portfolios = new_portfolios

    def get_rebalancing_dates(self):
        return [p.rebalancing_date for p in self.portfolios]

    def get_weights(self, rebalancing_date: str):
        for p in self.portfolios:
            if p.rebalancing_date == rebalancing_date:
                return p.weights
        return None

    def get_weights_df(self) -> pd.DataFrame:
        ps = self.portfolios
        rows = [getattr(p, "_row", None) for p in ps]
        if ps and all(r is not None for r in rows) and all(r[0] is rows[0][0] for r in rows) \
                and len({p.rebalancing_date for p in ps}) == len(ps):
            # batched backtest, weights not yet materialised: the same frame straight from the
            # weight panel (dates x assets, float64)
            return pd.DataFrame(np.stack([r[1] for r in rows]), index=[p.rebalancing_date for p in ps],
                                columns=list(rows[0][0]))
        return pd.DataFrame({p.rebalancing_date: p.weights for p in ps}).T

    def clear(self) -> None:
        self.portfolios.clear()

    def get_portfolio(self, rebalancing_date: str) -> Portfolio:
        dates = self.get_rebalancing_dates()
        if rebalancing_date in dates:
            return self.portfolios[dates.index(rebalancing_date)]
        raise ValueError(f"No portfolio found for rebalancing date {rebalancing_date}")

    def has_previous_portfolio(self, rebalancing_date: str) -> bool:
        dates = self.get_rebalancing_dates()
        return len(dates) > 0 and dates[0] < rebalancing_date

    def get_previous_portfolio(self, rebalancing_date: str) -> Portfolio:
        if not self.has_previous_portfolio(rebalancing_date):
            return Portfolio.empty()
        yesterday = [x for x in self.get_rebalancing_dates() if x < rebalancing_date][-1]
        return self.get_portfolio(yesterday)

    def get_initial_portfolio(self, rebalancing_date: str) -> Portfolio:
        if self.has_previous_portfolio(rebalancing_date=rebalancing_date):
            return self.get_previous_portfolio(rebalancing_date)
        return Portfolio(rebalancing_date=None, weights={})

    def __repr__(self):
        return f"Strategy(portfolios={self.portfolios})"

    def number_of_assets(self, th: float = 0.0001) -> pd.Series:
        return self.get_weights_df().apply(lambda x: sum(np.abs(x) > th), axis=1)

    # ---- device-batched simulation (pq_simulate_periods) --------------------------------
    def _stage(self, return_series: pd.DataFrame, last_end: bool):
        """Host bookkeeping for one launch: the weight matrix over the union of asset names,
        the panel rows of every holding period (X.loc[start:end], src/portfolio.py:283) and
        the range / name checks of floating_weights (src/portfolio.py:262-276)."""
        dates = self.get_rebalancing_dates()
        names = []
        seen = set()
        for p in self.portfolios:
            if p.weights is None:
                raise ValueError(f"portfolio of {p.rebalancing_date} has no weights (solver failed)")
            for k in p.weights:
                if k not in seen:
                    seen.add(k)
                    names.append(k)
        if not pd.Index(names).isin(return_series.columns).all():
            raise ValueError("Not all assets in w are contained in X.")
        W = np.zeros((len(dates), len(names)), dtype=np.float64)
        col = {k: j for j, k in enumerate(names)}
        for i, p in enumerate(self.portfolios):
            for k, v in p.weights.items():
                W[i, col[k]] = v
        if np.isnan(W).any():
            raise ValueError("weights (w) contain NaN which is not allowed.")
        days = return_series.index.values.astype("datetime64[D]").astype(np.int64)
        reb = np.array([np.datetime64(str(d)[:10], "D") for d in dates]).astype(np.int64)
        ends = np.empty_like(reb)
        ends[:-1] = reb[1:]
        if len(reb):
            ends[-1] = days[-1] if last_end else reb[-1]
        if len(reb) and (reb.min() < days[0]):
            raise ValueError("start_date must be contained in dataset")
        if len(reb) and (ends.max() > days[-1]):
            raise ValueError("end_date must be contained in dataset")
        row0 = np.searchsorted(days, reb, side="left")
        nrows = np.searchsorted(days, ends, side="right") - row0
        if len(reb) and nrows.min() < 1:
            raise ValueError("a holding period has no rows in return_series")
        return names, W, days, row0, nrows

    def _device_run(self, return_series, names, W, days, row0, nrows, fc, n_days_per_year,
                    rescale, want_end):
        import torch
        from . import engine
        dev = engine.default_device()
        lo = int(row0.min())
        hi = int((row0 + nrows).max())
        X = np.ascontiguousarray(return_series[names].to_numpy(dtype=np.float64)[lo:hi])
        panel = torch.as_tensor(X, device=dev)
        Wd = torch.as_tensor(W, device=dev)
        ret_days = np.concatenate([days[r + 1:r + k] for r, k in zip(row0, nrows)]) if len(row0) else days[:0]
        ret, wend, to = engine.simulate_periods(panel, Wd, row0 - lo, nrows, ret_day=ret_days, fc=fc,
                                                days_per_year=n_days_per_year, rescale=rescale,
                                                want_end=want_end)
        return ret_days, ret, wend, to

    def turnover(self, return_series, rescale=True) -> pd.Series:
        """src/portfolio.py:194-203.  In the reference the first date always compares with
        an empty previous portfolio whose floating window ends at ``None``, which raises
        ``TypeError`` (``pd.to_datetime(None) > Timestamp``, src/portfolio.py:264;
        captured in tests/golden/msci_simulate.npz).  That behaviour is kept;
        ``turnover_pairs`` gives the per-date values of the dates after the first."""
        if len(self.portfolios) == 0:
            return pd.Series(dtype=np.float64)
        raise TypeError("'>' not supported between instances of 'NoneType' and 'Timestamp' "
                        "(reference Strategy.turnover: the first date has no previous portfolio)")

    def turnover_pairs(self, return_series: pd.DataFrame, rescale: bool = True) -> pd.Series:
        """Portfolio.turnover(previous) for every date after the first
        (src/portfolio.py:111-123), all pairs in one device launch."""
        dates = self.get_rebalancing_dates()
        if len(dates) < 2:
            return pd.Series(dtype=np.float64)
        sub = Strategy(self.portfolios[:-1])
        names, W, days, row0, nrows = sub._stage(return_series, last_end=False)
        reb_last = np.datetime64(str(dates[-1])[:10], "D").astype(np.int64)
        if reb_last > days[-1]:
            raise ValueError("end_date must be contained in dataset")
        nrows[-1] = int(np.searchsorted(days, reb_last, side="right")) - row0[-1]
        _, _, _, to = self._device_run(return_series, names, W, days, row0, nrows, 0.0, 252,
                                       rescale, True)
        return pd.Series(to.cpu().numpy(), index=dates[1:])

    def simulate(self, return_series=None, fc: float = 0, vc: float = 0,
                 n_days_per_year: int = 252) -> pd.Series:
        """src/portfolio.py:209-248 on the device: every holding period floated, levelled
        and differenced in one launch; the fixed cost is applied in the same kernel."""
        if len(self.portfolios) == 0:
            raise ValueError("No objects to concatenate")                # pd.concat([]), :235
        if vc != 0:
            self.turnover(return_series=return_series, rescale=False)   # raises as the reference
        names, W, days, row0, nrows = self._stage(return_series, last_end=True)
        ret_days, ret, _, _ = self._device_run(return_series, names, W, days, row0, nrows, fc,
                                               n_days_per_year, False, False)
        r = ret.cpu().numpy()
        keep = ~np.isnan(r)
        idx = pd.DatetimeIndex(ret_days[keep].astype("datetime64[D]"))
        return pd.Series(r[keep], index=idx)


def floating_weights(X, w, start_date, end_date, rescale=True):
    """src/portfolio.py:259-296 (host helper for single pairs)."""
    start_date = pd.to_datetime(start_date)
    end_date = pd.to_datetime(end_date)
    if start_date < X.index[0]:
        raise ValueError("start_date must be contained in dataset")
    if end_date > X.index[-1]:
        raise ValueError("end_date must be contained in dataset")
    w = pd.Series(w, index=w.keys())
    if w.isna().any():
        raise ValueError("weights (w) contain NaN which is not allowed.")
    w = w.to_frame().T
    wnames = w.columns
    if not all(wnames.isin(X.columns)):
        raise ValueError("Not all assets in w are contained in X.")
    xmat = 1 + X.loc[start_date:end_date, wnames].copy().fillna(0)
    xmat.iloc[0] = w.dropna(how="all").fillna(0)
    w_float = xmat.cumprod()
    if rescale:
        pos = w_float[w_float >= 0]
        neg = w_float[w_float < 0]
        w_long = w_float.where(w_float >= 0).div(pos.abs().sum(axis=1), axis="index").fillna(0)
        w_short = w_float.where(w_float < 0).div(neg.abs().sum(axis=1), axis="index").fillna(0)
        w_float = pd.DataFrame(w_long + w_short, index=xmat.index, columns=wnames)
    return w_float
