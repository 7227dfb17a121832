# Host-side API restatement of PorQua (part of the GeomScale project; reference tree
# amolrpatil21/PorQua): src/data_loader.py.  PorQua is Copyright (c) 2024 Cyril Bachelard and
# Minh Ha Ho and licensed under the GNU LGPL v3; this module keeps that API and its
# behaviour (quirks included) so that the MI355X engine is a drop-in, and is distributed
# under the same licence terms.
"""Data loading helpers (mirror of src/data_loader.py; I/O is outside the hot path).

``load_data_msci`` accepts the shipped CSV format (comma separated, dd-mm-YYYY) as well as
the ';' / dd/mm/YYYY format the reference loader expects (src/data_loader.py:39-44,
which raises on the shipped files).
"""
from __future__ import annotations

import os

import pandas as pd


def _read(path: str) -> pd.DataFrame:
    with open(path, "r", encoding="utf-8-sig") as f:
        head = f.readline()
    sep = ";" if head.count(";") > head.count(",") else ","
    df = pd.read_csv(path, sep=sep, index_col=0, header=0, encoding="utf-8-sig")
    first = str(df.index[0])
    fmt = "%d-%m-%Y" if "-" in first else "%d/%m/%Y"
    df.index = pd.to_datetime(df.index, format=fmt)
    return df.astype(float)


def load_data_msci(path: str = None, n: int = 24) -> dict:
    """MSCI country index returns (first n columns) and the NDDLWI world index."""
    path = os.path.join(os.getcwd(), "data") if path is None else path
    X = _read(os.path.join(path, "msci_country_indices.csv"))
    y = _read(os.path.join(path, "NDDLWI.csv"))
    return {"return_series": X[X.columns[:n]], "bm_series": y}
