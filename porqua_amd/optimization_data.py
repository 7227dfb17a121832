# Host-side API restatement of PorQua (part of the GeomScale project; reference tree
# amolrpatil21/PorQua): src/optimization_data.py.  PorQua is Copyright (c) 2024 Cyril Bachelard and
# Minh Ha Ho and licensed under the GNU LGPL v3; this module keeps that API and its
# behaviour (quirks included) so that the MI355X engine is a drop-in, and is distributed
# under the same licence terms.
"""Per-date data container (mirror of src/optimization_data.py:19-49)."""
from __future__ import annotations

from typing import Optional

import pandas as pd


class OptimizationData(dict):

    def __init__(self, align=True, lags=None, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self.__dict__ = self
        for key, lag in (lags or {}).items():
            self[key] = self[key].shift(lag)
        if align:
            self.align_dates()

    def align_dates(self, variable_names: Optional[list] = None, dropna: bool = True) -> None:
        # the reference's builders call align_dates(..., dropna=True), which its signature
        # lacks (src/builders.py:246-249 vs src/optimization_data.py:30); accepted here.
        names = list(self.keys()) if variable_names is None else list(variable_names)
        index = self.intersecting_dates(variable_names=names, dropna=dropna)
        for key in names:
            self[key] = self[key].loc[index]

    def intersecting_dates(self, variable_names: Optional[list] = None, dropna: bool = True) -> pd.DatetimeIndex:
        names = list(self.keys()) if variable_names is None else list(variable_names)
        if dropna:
            for key in names:
                self[key] = self[key].dropna()
        index = self[names[0]].index
        for key in names:
            index = index.intersection(self[key].index)
        return index
