"""Parity at the headline configuration: bench.py's exact problem (BASELINE.json configs[2]:
n = 1000, T = 252, all 4749 daily dates of the seed-20240314 panel, long-only
min-variance, budget + box [0, 1]) solved through the same path the bench times (window
moments -> band Gram -> capacitance + K2 -> grouped fused ADMM -> window polish), both
eager and as the replayed HIP-graph step bench.py times (graph=True), then

  * 32 evenly spaced dates against the oracle optima in tests/golden/headline_c3.npz
    (oracle.qp_ipm, tools/capture_headline.py): weights <= 1e-5 L-inf, objective <= 1e-6
    relative, violation <= 1e-7 (the north_star bars, src/qp_problems.py:184-221,
    test/tests_quadratic_program.py:79-82 for obj = 0.5 x'Px + q'x);
  * all 4749 solutions against the size-independent KKT certificate (P x recomputed from
    the panel rows with torch): violation <= 1e-7, relative stationarity and
    complementarity <= 1e-7, every status SOLVED.
"""
import os

import numpy as np
import pytest
import torch

from oracle.ref_pipeline import cov_pearson
from porqua_amd import _lib
from porqua_amd.workloads import MinVarianceBacktest

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), "golden", "headline_c3.npz")


@pytest.fixture(scope="module", params=["eager", "graph"])
def solved(device, request):
    """``graph``: exactly what bench.py times -- graph=True, prepare() (the eager step and the
    capturing step), then a REPLAYED step: sync-free rounds capped at the first step's count,
    every stage a replayed HIP graph.  ``eager``: the host-checked solve."""
    graph = request.param == "graph"
    wl = MinVarianceBacktest(device=device, graph=graph)
    assert wl.use_lr and wl.grouped and not wl.with_cov     # the path bench.py times
    if graph:
        wl.prepare()
        assert wl.graphs is not None and wl.sf_rounds is not None
    res = wl.step()
    torch.cuda.synchronize()
    if graph:
        assert wl.graph_replays > 0, "the checked step was not a graph replay"
    return wl, res


def test_headline_matches_oracle_on_32_dates(solved):
    wl, res = solved
    g = np.load(GOLD)
    assert int(g["n"]) == wl.n and int(g["T"]) == wl.T and int(g["D"]) == wl.D
    idx = g["date_index"]
    assert len(idx) == 32
    x = res.x.cpu().numpy()[idx]
    st = res.status.cpu().numpy()[idx]
    assert np.all(st == _lib.PQ_SOLVED), st
    T = wl.T
    for i, d in enumerate(idx):
        e = wl.ends_local[d]
        P = 2.0 * cov_pearson(wl.R_rank[e - T + 1:e + 1])
        xi = x[i]
        assert np.abs(xi - g["x"][i]).max() <= 1e-5, (d, np.abs(xi - g["x"][i]).max())
        obj = 0.5 * xi @ P @ xi
        assert abs(obj - g["obj"][i]) <= 1e-6 * abs(g["obj"][i]), (d, obj, g["obj"][i])
        viol = max(abs(xi.sum() - 1.0), max(0.0, -xi.min()), max(0.0, xi.max() - 1.0))
        assert viol <= 1e-7, (d, viol)
        # the engine's own objective field agrees with 0.5 x'Px
        assert abs(res.obj[d].item() - obj) <= 1e-9 * abs(obj)


def test_headline_kkt_certificate_all_dates(solved):
    wl, res = solved
    c = wl.certificate(res)
    assert c["status_counts"] == {str(_lib.PQ_SOLVED): wl.D}, c
    assert c["max_violation"] <= 1e-7, c
    assert c["max_rel_stationarity"] <= 1e-7, c
    assert c["max_rel_complementarity"] <= 1e-7, c
