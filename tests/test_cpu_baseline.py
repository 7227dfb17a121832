"""The cpu_baseline leg's workloads (oracle/cpu_baseline.py, bench infrastructure): each
restates the reference's per-QP path on the same synthetic inputs bench.py's GPU legs solve,
and its answers are feasible optima of that problem (small sizes here)."""
import numpy as np

from oracle import cpu_baseline as cb
from oracle.ref_pipeline import cov_pearson, mean_geometric
from porqua_amd.synthetic import factor_panel


def _feasible(x, G=None, h=None):
    assert abs(x.sum() - 1.0) <= 1e-7 and x.min() >= -1e-7 and x.max() <= 1 + 1e-7
    if G is not None:
        assert (G @ x - h).max() <= 1e-7


def test_config2_replication_units_and_solution():
    wl = cb.Workload("config2", 40, 30, 0, 0, root=".")
    assert len(wl.units) == wl.R.shape[0] - 29 and wl.R.shape[1] == 40
    u = wl.sample(3)[1]
    sol = wl.solve(u)
    _feasible(sol.x)
    X, y = wl.R[u - 29:u + 1], wl.y[u - 29:u + 1]
    # stationarity of the tracking objective P = 2 X'X, q = -2 X'y at the IPM answer (tol 1e-7)
    g = 2 * X.T @ (X @ sol.x) - 2 * X.T @ y
    free = (sol.x > 1e-5) & (sol.x < 1 - 1e-5)
    if free.sum() > 1:
        assert np.ptp(g[free]) <= 1e-5 * max(1.0, np.abs(g).max())


def test_config4_sector_caps_bind():
    wl = cb.Workload("config4", 60, 30, 8, 0)
    assert wl.G.shape == (20, 60) and np.allclose(wl.G.sum(0), 1.0) and np.all(wl.h == 0.15)
    sol = wl.solve(wl.units[3])
    _feasible(sol.x, wl.G, wl.h)


def test_config5_sweep_grid_and_objective():
    wl = cb.Workload("config5", 50, 30, 3, 0)
    assert len(wl.units) == 3 * 64 and wl.lams[0] == 0.1 and abs(wl.lams[-1] - 100.0) < 1e-9
    picks = wl.sample(5)
    assert len({k for _, k in picks}) > 1                 # lambdas vary over the sample
    e, k = picks[2]
    sol = wl.solve((e, k), repair=False)
    _feasible(sol.x)
    R = factor_panel(29 + 21 * 3, 50)[1]
    X = R[e - 29:e + 1]
    assert np.array_equal(wl.R, R)
    P, q = 2 * wl.lams[k] * cov_pearson(X), -mean_geometric(X)
    assert abs(sol.obj - (0.5 * sol.x @ P @ sol.x + q @ sol.x)) <= 1e-9 * max(1.0, abs(sol.obj))
