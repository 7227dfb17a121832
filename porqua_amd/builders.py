# Host-side API restatement of PorQua (part of the GeomScale project; reference tree
# amolrpatil21/PorQua): src/builders.py.  PorQua is Copyright (c) 2024 Cyril Bachelard and
# Minh Ha Ho and licensed under the GNU LGPL v3; this module keeps that API and its
# behaviour (quirks included) so that the MI355X engine is a drop-in, and is distributed
# under the same licence terms.
"""Backtest item builders (mirror of src/builders.py:35-287, the hot-path subset).

Selection / optimization items are built per date by callable builders exactly as in the
reference.  The batched engine (backtest.Backtest.run with solver 'mi355x') recognises the
standard builders below and replaces their per-date pandas slicing by window row-index
lists on a device-resident panel; custom builders still run per date on the host.
"""
from __future__ import annotations

from abc import ABC, abstractmethod
from typing import Any

import numpy as np
import pandas as pd


class BacktestItemBuilder(ABC):

    def __init__(self, **kwargs):
        self._arguments = dict(kwargs)

    @property
    def arguments(self) -> dict[str, Any]:
        return self._arguments

    @arguments.setter
    def arguments(self, value: dict[str, Any]) -> None:
        self._arguments = value

    @abstractmethod
    def __call__(self, service, rebdate: str) -> None:
        raise NotImplementedError("Method '__call__' must be implemented in derived class.")


class SelectionItemBuilder(BacktestItemBuilder):

    def __call__(self, bs, rebdate: str) -> None:
        fn = self.arguments.get("bibfn")
        if fn is None or not callable(fn):
            raise ValueError("bibfn is not defined or not callable.")
        value = fn(bs=bs, rebdate=rebdate, **self.arguments)
        bs.selection.add_filtered(filter_name=self.arguments.get("item_name"), value=value)


class OptimizationItemBuilder(BacktestItemBuilder):

    def __call__(self, bs, rebdate: str) -> None:
        fn = self.arguments.get("bibfn")
        if fn is None or not callable(fn):
            raise ValueError("bibfn is not defined or not callable.")
        fn(bs=bs, rebdate=rebdate, **self.arguments)


def bibfn_selection_data(bs, rebdate: str, **kwargs) -> pd.Series:
    """All return-series columns are selected (src/builders.py:124-135)."""
    data = bs.data.get("return_series")
    if data is None:
        raise ValueError("Return series data is missing.")
    return pd.Series(np.ones(data.shape[1], dtype=int), index=data.columns, name="binary")


def _upto(data, rebdate, width):
    """data[data.index <= rebdate].tail(width): on a sorted index the rows up to the date are a
    prefix, so the window is one positional slice (no copy of the whole prefix first)."""
    idx = data.index
    if isinstance(idx, pd.DatetimeIndex) and idx.is_monotonic_increasing:
        end = int(idx.searchsorted(pd.Timestamp(rebdate), side="right"))
        return data.iloc[max(0, end - width) if width is not None else 0:end]
    out = data[idx <= rebdate]
    return out.tail(width) if width is not None else out


def _trailing(data: pd.DataFrame, rebdate, width):
    out = _upto(data, rebdate, width)
    return out[out.index.dayofweek < 5]


def bibfn_return_series(bs, rebdate: str, **kwargs) -> None:
    """data[index <= rebdate].tail(width)[selected], weekends dropped (src/builders.py:188-215)."""
    data = bs.data.get("return_series")
    if data is None:
        raise ValueError("Return series data is missing.")
    ids = bs.selection.selected
    out = _upto(data, rebdate, kwargs.get("width"))[ids]
    bs.optimization_data["return_series"] = out[out.index.dayofweek < 5]


def bibfn_bm_series(bs, rebdate: str, **kwargs) -> None:
    """Benchmark window (src/builders.py:218-251); align=True aligns it with the returns."""
    data = bs.data.get("bm_series")
    if data is None:
        raise ValueError("Benchmark return series data is missing.")
    bs.optimization_data["bm_series"] = _trailing(data, rebdate, kwargs.get("width"))
    if kwargs.get("align"):
        bs.optimization_data.align_dates(variable_names=["bm_series", "return_series"], dropna=True)


def bibfn_budget_constraint(bs, rebdate: str, **kwargs) -> None:
    """src/builders.py:258-269."""
    bs.optimization.constraints.add_budget(rhs=kwargs.get("budget", 1), sense="=")


def bibfn_box_constraints(bs, rebdate: str, **kwargs) -> None:
    """src/builders.py:272-287 (defaults LongOnly [0, 1])."""
    bs.optimization.constraints.add_box(box_type=kwargs.get("box_type", "LongOnly"),
                                        lower=kwargs.get("lower", 0), upper=kwargs.get("upper", 1))


# builders whose output the batched engine can stage without per-date pandas work
STANDARD_BIBFNS = {bibfn_selection_data, bibfn_return_series, bibfn_bm_series,
                   bibfn_budget_constraint, bibfn_box_constraints}
