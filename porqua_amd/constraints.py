# Host-side API restatement of PorQua (part of the GeomScale project; reference tree
# amolrpatil21/PorQua): src/constraints.py.  PorQua is Copyright (c) 2024 Cyril Bachelard and
# Minh Ha Ho and licensed under the GNU LGPL v3; this module keeps that API and its
# behaviour (quirks included) so that the MI355X engine is a drop-in, and is distributed
# under the same licence terms.
"""Constraint bookkeeping (mirror of src/constraints.py:23-219).

Pure host bookkeeping, computed once per backtest when constraints are date-invariant:
budget / box / linear / l1 constraints -> dense G, h, A, b consumed by the QP engine.
Behaviour follows the reference including its known quirk: with ``lbub_to_G=True`` and
only '=' linear rows, the box rows are stacked twice (src/constraints.py:128-133,159-161);
duplicated inequality rows leave the feasible set and the optimum unchanged.
"""
from __future__ import annotations

import warnings
from typing import Dict

import numpy as np
import pandas as pd


class Constraints:

    def __init__(self, selection="NA") -> None:
        if not all(isinstance(item, str) for item in selection):
            raise ValueError("argument 'selection' has to be a character vector.")
        self.selection = selection
        self.budget = {"Amat": None, "sense": None, "rhs": None}
        self.box = {"box_type": "NA", "lower": None, "upper": None}
        self.linear = {"Amat": None, "sense": None, "rhs": None}
        self.l1 = {}

    def __str__(self) -> str:
        return " ".join(f"\n{k}:\n\n{v}\n" for k, v in vars(self).items())

    def add_budget(self, rhs=1, sense="=") -> None:
        if self.budget.get("rhs") is not None:
            warnings.warn("Existing budget constraint is overwritten\n")
        ones = pd.Series(np.ones(len(self.selection)), index=self.selection)
        self.budget = {"Amat": ones, "sense": sense, "rhs": rhs}

    def add_box(self, box_type="LongOnly", lower=None, upper=None) -> None:
        box = box_constraint(box_type, lower, upper)
        for side in ("lower", "upper"):
            if np.isscalar(box[side]):
                box[side] = pd.Series(np.repeat(float(box[side]), len(self.selection)), index=self.selection)
        if (box["upper"] < box["lower"]).any():
            raise ValueError("Some lower bounds are higher than the corresponding upper bounds.")
        self.box = box

    def add_linear(self, Amat: pd.DataFrame = None, a_values: pd.Series = None, sense: str = "=",
                   rhs=None, name: str = None) -> None:
        if Amat is None:
            if a_values is None:
                raise ValueError("Either 'Amat' or 'a_values' must be provided.")
            Amat = pd.DataFrame(a_values).T.reindex(columns=self.selection).fillna(0)
            if name is not None:
                Amat.index = [name]
        if isinstance(sense, str):
            sense = pd.Series([sense])
        if isinstance(rhs, (int, float)):
            rhs = pd.Series([rhs])
        if self.linear["Amat"] is not None:
            Amat = pd.concat([self.linear["Amat"], Amat], axis=0, ignore_index=False)
            sense = pd.concat([self.linear["sense"], sense], axis=0, ignore_index=False)
            rhs = pd.concat([self.linear["rhs"], rhs], axis=0, ignore_index=False)
        Amat = Amat.fillna(0)
        self.linear = {"Amat": Amat, "sense": sense, "rhs": rhs}

    def add_l1(self, name: str, rhs=None, x0=None, *args, **kwargs) -> None:
        """name: 'turnover' or 'leverage'."""
        if rhs is None:
            raise TypeError("argument 'rhs' is required.")
        con = {"rhs": rhs}
        if x0:
            con["x0"] = x0
        con.update({f"arg{i}": a for i, a in enumerate(args)})
        con.update(kwargs)
        self.l1[name] = con

    def to_GhAb(self, lbub_to_G: bool = False) -> Dict[str, np.ndarray]:
        A_parts, b_parts, G_parts, h_parts = [], [], [], []
        if self.budget["Amat"] is not None:
            row = np.asarray(self.budget["Amat"], dtype=float)
            val = np.asarray(self.budget["rhs"], dtype=float)
            (A_parts if self.budget["sense"] == "=" else G_parts).append(row)
            (b_parts if self.budget["sense"] == "=" else h_parts).append(val)
        box_block = None
        if lbub_to_G:
            n = len(self.selection)
            box_block = (np.vstack([-np.eye(n), np.eye(n)]),
                         np.concatenate([-np.asarray(self.box["lower"], dtype=float),
                                         np.asarray(self.box["upper"], dtype=float)]))
            G_parts.append(box_block[0])
            h_parts.append(box_block[1])
        if self.linear["Amat"] is not None:
            M = self.linear["Amat"].to_numpy(dtype=float).copy()
            r = np.asarray(self.linear["rhs"], dtype=float).reshape(-1).copy()
            sense = np.asarray(self.linear["sense"])
            flip = sense == ">="
            M[flip] *= -1.0
            r[flip] *= -1.0
            eq = sense == "="
            if eq.any():
                A_parts.append(M[eq])
                b_parts.append(r[eq])
            extra = None
            if (~eq).any():
                extra = (M[~eq], r[~eq])
            elif box_block is not None:
                extra = box_block          # reference quirk: the box block is appended again
            if extra is not None:
                G_parts.append(extra[0])
                h_parts.append(extra[1])

        def stack(parts, vec):
            if not parts:
                return None
            if vec:
                return np.concatenate([np.atleast_1d(p) for p in parts]) if len(parts) > 1 else parts[0]
            return np.vstack(parts) if len(parts) > 1 else parts[0]

        A = stack(A_parts, False)
        b = stack(b_parts, True)
        G = stack(G_parts, False)
        h = stack(h_parts, True)
        A = A.reshape(-1, A.shape[-1]) if A is not None else None
        G = G.reshape(-1, G.shape[-1]) if G is not None else None
        return {"G": G, "h": h, "A": A, "b": b}


def match_arg(x, lst):
    return [el for el in lst if x in el][0]


def box_constraint(box_type="LongOnly", lower=None, upper=None) -> dict:
    """Default bounds per box type (src/constraints.py:178-204)."""
    box_type = match_arg(box_type, ["LongOnly", "LongShort", "Unbounded"])
    if box_type == "Unbounded":
        lower = float("-inf") if lower is None else lower
        upper = float("inf") if upper is None else upper
    elif box_type == "LongShort":
        lower = -1 if lower is None else lower
        upper = 1 if upper is None else upper
    else:
        if lower is None:
            if upper is None:
                lower, upper = 0, 1
            else:
                lower = upper * 0
        else:
            if not np.isscalar(lower) and any(v < 0 for v in lower):
                raise ValueError("Inconsistent lower bounds for box_type 'LongOnly'. "
                                 "Change box_type to LongShort or ensure that lower >= 0.")
            upper = lower * 0 + 1 if upper is None else upper
    return {"box_type": box_type, "lower": lower, "upper": upper}


def linear_constraint(Amat=None, sense="=", rhs=float("inf"), index_or_name=None, a_values=None) -> dict:
    out = {"Amat": Amat, "sense": sense, "rhs": rhs}
    if index_or_name is not None:
        out["index_or_name"] = index_or_name
    if a_values is not None:
        out["a_values"] = a_values
    return out
