"""The CPU oracle is pinned against golden vectors captured from the reference itself
(tools/capture_golden.py imports /root/reference/src with a capturing qpsolvers stub)."""
import numpy as np
import pytest

from oracle import ref_pipeline as rp
from oracle.qp_ipm import solve_qp
from tests.conftest import load_golden


def _panel():
    g = load_golden("msci_panel")
    return g["dates"].astype("datetime64[D]"), g["returns"], g["bm"]


def test_cov_cases_match_reference():
    g = load_golden("cov_cases")
    names = sorted({k.split("__")[0] for k in g.files})
    assert len(names) == 6
    for name in names:
        X = g[f"{name}__X"]
        spec = eval(str(g[f"{name}__spec"]))   # dict literal written by the capture script
        kw = {"method": spec.get("method", "pearson"),
              "check_positive_definite": spec.get("check_positive_definite", True),
              "lam": spec.get("lambda_covmat_regularization")}
        S = rp.covariance_estimate(X, **kw)
        ref = g[f"{name}__cov"]
        assert np.linalg.norm(S - ref) <= 1e-12 * np.linalg.norm(ref), name
        assert np.linalg.norm(rp.cov_pearson(X) - g[f"{name}__raw"]) <= 1e-13 * np.linalg.norm(g[f"{name}__raw"])


def test_nearest_pd_fires_for_singular_window():
    g = load_golden("cov_cases")
    raw, rep = g["pearson_n_gt_T__raw"], g["pearson_n_gt_T__cov"]
    assert not rp.is_pd(raw) and rp.is_pd(rep)
    assert np.linalg.norm(rep - raw) <= 1e-12 * np.linalg.norm(raw)   # repair is rounding-level


@pytest.mark.parametrize("tag", ["msci_ls", "msci_ls_l2", "msci_ls_log"])
def test_least_squares_objective_matches_reference(tag):
    dates, R, y = _panel()
    g = load_golden(tag)
    params = eval(str(g["params"]))
    for d, rb in enumerate(g["rebdates"][::11]):
        i = d * 11
        rows = rp.window_rows(dates, rb, int(g["width"]))
        assert len(rows) == g["win_len"][i]
        assert dates[rows[0]].astype(np.int64) == g["win_first"][i]
        P, q, c = rp.objective_least_squares(R[rows], y[rows], l2_penalty=params.get("l2_penalty"),
                                             log_transform=params.get("log_transform", False))
        assert np.allclose(P, g["P"][i], rtol=1e-12, atol=1e-15)
        assert np.allclose(q, g["q"][i], rtol=1e-12, atol=1e-15)
        assert abs(c - g["const"][i]) <= 1e-12 * abs(c)


@pytest.mark.parametrize("tag", ["msci_wls", "msci_wls_log"])
def test_weighted_least_squares_objective_matches_reference(tag):
    """src/optimization.py:232-256 (tools/capture_wls.py): P, q, constant of every 7th date."""
    dates, R, y = _panel()
    g = load_golden(tag)
    params = eval(str(g["params"]))
    for i in range(0, len(g["rebdates"]), 7):
        rows = rp.window_rows(dates, g["rebdates"][i], int(g["width"]))
        assert len(rows) == g["win_len"][i]
        P, q, c = rp.objective_wls(R[rows], y[rows], params["tau"], params.get("log_transform", False))
        assert np.allclose(P, g["P"][i], rtol=1e-12, atol=1e-15)
        # the reference's q is an (n, 1) column here (X' W y with y a DataFrame)
        assert np.allclose(q, g["q"][i].reshape(-1), rtol=1e-12, atol=1e-15)
        assert abs(c - g["const"][i]) <= 1e-12 * abs(c)
    assert g["kkt_primal"].max() < 1e-9 and g["kkt_dual"].max() < 1e-9


@pytest.mark.parametrize("tag", ["msci_mv", "msci_mv_shrink"])
def test_mean_variance_objective_matches_reference(tag):
    dates, R, _ = _panel()
    g = load_golden(tag)
    cov = eval(str(g["cov"]))
    for i in range(0, len(g["rebdates"]), 13):
        rows = rp.window_rows(dates, g["rebdates"][i], int(g["width"]))
        P, q, _ = rp.objective_mean_variance(R[rows], risk_aversion=float(g["risk_aversion"]),
                                             method=cov.get("method", "pearson"),
                                             lam=cov.get("lambda_covmat_regularization"))
        assert np.allclose(P, g["P"][i], rtol=1e-12, atol=1e-17)
        assert np.allclose(q, g["q"][i], rtol=1e-12, atol=1e-17)


def test_constraints_to_GhAb_matches_reference():
    g = load_golden("ghab")
    n = 24
    sub = 12
    blk = np.zeros((3, n)); blk[:, :sub] = g["blk"]
    linear = (np.vstack([g["a1"], g["a2"], g["a3"], blk]), ["<=", ">=", "=", "=", "=", "="],
              np.array([1, -1, 0.5, 1, 1, 1.0]))
    budget = (np.ones(n), "=", 1)
    box = rp.box_bounds(n, "LongOnly")
    for lbub, sfx in [(False, "0"), (True, "1")]:
        out = rp.to_GhAb(n, budget, box, linear, lbub_to_G=lbub)
        for k in "GhAb":
            assert np.allclose(out[k], g[k + sfx]), (k, sfx)
    out = rp.to_GhAb(n, budget, rp.box_bounds(n, "LongShort"),
                     (np.vstack([g["a3"], blk]), ["="] * 4, np.array([0.5, 1, 1, 1.0])), lbub_to_G=True)
    assert out["G"].shape == g["G2"].shape == (4 * n, n)      # box rows stacked twice (quirk)
    assert np.allclose(out["G"], g["G2"]) and np.allclose(out["h"], g["h2"])


@pytest.mark.parametrize("tag", ["msci_ls", "msci_mv", "msci_qeqw"])
def test_ipm_oracle_is_kkt_certified(tag):
    g = load_golden(tag)
    for i in range(0, len(g["P"]), 20):
        s = solve_qp(g["P"][i], g["q"][i], A=g["A"][i], b=np.atleast_1d(g["b"][i]), lb=g["lb"][i], ub=g["ub"][i])
        assert s.primal_residual() < 1e-12 and s.dual_residual() < 1e-12
        assert np.abs(s.x - g["x"][i]).max() < 1e-9
        assert abs(s.obj - g["obj"][i]) <= 1e-12 * max(1.0, abs(g["obj"][i]))


@pytest.mark.parametrize("tag", ["msci_lad", "msci_lad_ret"])
def test_lad_lp_matches_reference(tag):
    """oracle/lad.py restates LAD.set_objective / model_qpsolvers (src/optimization.py:271-336):
    the LP the reference hands to qpsolvers (tools/capture_lad.py) is reproduced entry for
    entry, and HiGHS reproduces the golden optimal value."""
    from oracle import lad as olad
    dates, R, y = _panel()
    g = load_golden(tag)
    params = eval(str(g["params"]))
    box = eval(str(g["box"]))
    # P = 0 reaches qpsolvers as nearestPD(0) = spacing(0) I = 5e-324 I (src/qp_problems.py:189-191)
    assert (g["P_absmax"] <= 1e-300).all()
    n = R.shape[1]
    for i in range(0, len(g["rebdates"]), 5):
        rows = rp.window_rows(dates, g["rebdates"][i], int(g["width"]))
        X = olad.levels(R[rows], params.get("use_level", True), params.get("use_log", True))
        yl = olad.levels(y[rows], params.get("use_level", True), params.get("use_log", True))
        q, A, b, G, h, lb, ub = olad.lad_lp(X, yl, A=np.ones(n), b=np.array(1.0), lb=np.zeros(n),
                                            ub=np.full(n, box.get("upper", 1.0)))
        assert np.array_equal(q, g["q"][i]) and np.allclose(A, g["A"][i], rtol=1e-13, atol=0)
        assert np.allclose(b, g["b"][i], rtol=1e-13, atol=0)
        assert np.array_equal(lb, g["lb"][i]) and np.array_equal(ub, g["ub"][i])
        s = olad.solve_lp(q, A, b, lb, ub)
        assert abs(s.fun - g["obj"][i]) <= 1e-9 * g["obj"][i]


def test_pairwise_cov_oracle_matches_reference_nan_windows():
    """oracle cov_pairwise == the reference's DataFrame.cov() on NaN-bearing windows
    (tools/capture_nan_cov.py), NaN pattern included."""
    g = load_golden("nan_cov")
    for case in ("msci_holes", "wide", "sparse"):
        S = rp.cov_pairwise(g[f"{case}__X"])
        ref = g[f"{case}__raw"]
        assert np.array_equal(np.isnan(S), np.isnan(ref)), case
        ok = ~np.isnan(ref)
        assert np.abs(S[ok] - ref[ok]).max() <= 1e-14 * np.abs(ref[ok]).max(), case


def test_vectorised_pairwise_oracle_matches_reference_and_loop():
    """oracle cov_pairwise_rows (the pair loop vectorised over one row at a time, used at the
    config sizes) == the reference's DataFrame.cov() fixtures and == cov_pairwise."""
    g = load_golden("nan_cov")
    for case in ("msci_holes", "wide", "sparse"):
        S = rp.cov_pairwise_rows(g[f"{case}__X"])
        ref = g[f"{case}__raw"]
        assert np.array_equal(np.isnan(S), np.isnan(ref)), case
        ok = ~np.isnan(ref)
        assert np.abs(S[ok] - ref[ok]).max() <= 1e-14 * np.abs(ref[ok]).max(), case
    rng = np.random.default_rng(3)
    X = rng.normal(3e-4, 0.02, size=(60, 40))
    X[rng.random(X.shape) < 0.1] = np.nan
    A, B = rp.cov_pairwise_rows(X), rp.cov_pairwise(X)
    assert np.array_equal(np.isnan(A), np.isnan(B)) and np.nanmax(np.abs(A - B)) <= 1e-15 * np.nanmax(np.abs(B))
