"""The engine's algorithm (ADMM + active-set polish, restated in numpy by
tests/engine_model.py) reaches the oracle's optimum on the reference's golden QPs."""
import numpy as np
import pytest

from tests.conftest import load_golden
from tests.engine_model import admm, polish


@pytest.mark.parametrize("tag", ["msci_ls", "msci_mv", "msci_mv_shrink"])
def test_model_matches_golden(tag):
    g = load_golden(tag)
    for i in range(0, len(g["P"]), 15):
        P, q = g["P"][i], g["q"][i]
        n = len(q)
        C = np.vstack([g["A"][i], np.eye(n)])
        l = np.concatenate([np.atleast_1d(g["b"][i]), g["lb"][i]])
        u = np.concatenate([np.atleast_1d(g["b"][i]), g["ub"][i]])
        r = admm(P, q, C, l, u, scaling=0)
        assert r["status"] == "solved"
        sc = max(np.abs(q).max(), np.abs(np.diag(P)).max())
        x, lam, zb, rounds, ok = polish(P, q, C, l, u, r["x"], r["y"], r["z"], dual_tol=1e-9 * sc)
        assert ok
        assert np.abs(x - g["x"][i]).max() < 1e-5
