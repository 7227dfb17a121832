# Host-side API restatement of PorQua (part of the GeomScale project; reference tree
# amolrpatil21/PorQua): src/selection.py.  PorQua is Copyright (c) 2024 Cyril Bachelard and
# Minh Ha Ho and licensed under the GNU LGPL v3; this module keeps that API and its
# behaviour (quirks included) so that the MI355X engine is a drop-in, and is distributed
# under the same licence terms.
"""Asset-universe filter bookkeeping (mirror of src/selection.py:23-113; host only)."""
from __future__ import annotations

from typing import Optional, Union

import pandas as pd


class Selection:

    def __init__(self, ids: pd.Index = pd.Index([])):
        self._filtered: dict = {}
        self.selected = ids

    @property
    def selected(self) -> pd.Index:
        return self._selected

    @selected.setter
    def selected(self, value):
        if not isinstance(value, pd.Index):
            raise ValueError("Inconsistent input type for selected.setter. Needs to be a pd.Index.")
        self._selected = value

    @property
    def filtered(self):
        return self._filtered

    def get_selected(self, filter_names: Optional[list] = None) -> pd.Index:
        names = list(self.filtered.keys()) if filter_names is None else list(filter_names)
        if len(names) == 1:   # one binary Series (the usual selection): the same rows, no frame
            v = self.filtered[names[0]]
            if isinstance(v, pd.Series) and v.name == "binary" and v.index.is_unique:
                v = v.dropna()
                return v.index[v.to_numpy() == 1]
        df = self.df_binary(filter_names)
        return df[df.eq(1).all(axis=1)].index

    def clear(self) -> None:
        self.selected = pd.Index([])
        self._filtered = {}

    def add_filtered(self, filter_name: str, value: Union[pd.Series, pd.DataFrame]) -> None:
        if not isinstance(filter_name, str) or not filter_name.strip():
            raise ValueError("Argument 'filter_name' must be a nonempty string.")
        if not isinstance(value, (pd.Series, pd.DataFrame)):
            raise ValueError("Inconsistent input type. Needs to be a pd.Series or a pd.DataFrame.")
        binary = value if isinstance(value, pd.Series) and value.name == "binary" else (
            value["binary"] if isinstance(value, pd.DataFrame) and "binary" in value.columns else None)
        if binary is not None:
            if not binary.isin([0, 1]).all():
                raise ValueError("Column 'binary' must contain only 0s and 1s.")
            if isinstance(value, pd.Series):
                value = value.astype(int)
            else:
                value = value.copy()
                value["binary"] = value["binary"].astype(int)
        self._filtered[filter_name] = value
        self.selected = self.get_selected()

    def df(self, filter_names: Optional[list] = None) -> pd.DataFrame:
        names = self.filtered.keys() if filter_names is None else filter_names
        return pd.concat({k: (pd.DataFrame(self.filtered[k]) if isinstance(self.filtered[k], pd.Series)
                              else self.filtered[k]) for k in names}, axis=1)

    def df_binary(self, filter_names: Optional[list] = None) -> pd.DataFrame:
        df = self.df(filter_names).filter(like="binary").dropna()
        df.columns = df.columns.droplevel(1)
        return df
