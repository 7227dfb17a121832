"""Portfolio / Strategy containers (mirror of the parts of src/portfolio.py:20-245 that
the rebalance loop produces; simulation helpers are a later row)."""
from __future__ import annotations

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

    @property
    def weights(self):
        return self._weights

    @weights.setter
    def weights(self, new_weights):
        if not isinstance(new_weights, dict):
            if hasattr(new_weights, "to_dict"):
                new_weights = new_weights.to_dict()
            else:
                raise TypeError("weights must be a dictionary")
        self._weights = new_weights

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
        return pd.Series(self._weights)

    def __repr__(self):
        return f"Portfolio(rebalancing_date={self.rebalancing_date}, weights={self.weights})"


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
        return pd.DataFrame({p.rebalancing_date: p.weights for p in self.portfolios}).T
