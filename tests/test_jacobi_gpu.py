"""The hand-written batched symmetric eigensolver (pq_sym_eig_batched, two-sided block
Jacobi) behind nearestPD (src/helper_functions.py:29-58) and the risk-aversion sweep's
eigen capacitance: eigenvalues against numpy (LAPACK syevd) to 1e-13 x (column blocks) of the
matrix norm,
eigenvectors orthonormal and reconstructing the matrix, the PSD projection
Q max(L, 0) Q' (pq_psd_form_batched) against numpy, on sizes with one, a few and many
32-column blocks (n = 24, 100, 252, 600) and on a rank-deficient covariance (n > T)."""
import numpy as np
import pytest
import torch

from porqua_amd import _lib, engine
from porqua_amd.helper_functions import sym_eig

pytestmark = pytest.mark.gpu


def _dev_batch(A, ld):
    B, n, _ = A.shape
    t = torch.zeros((B, ld, ld), dtype=torch.float64, device="cuda")
    t[:, :n, :n] = torch.from_numpy(A).cuda()
    return t


@pytest.mark.parametrize("n", [24, 100, 252, 600])
def test_sym_eig_matches_lapack(device, n):
    rng = np.random.default_rng(n)
    M = rng.normal(size=(3, n, n))
    A = 0.5 * (M + M.transpose(0, 2, 1))
    A[2] = M[2].T @ M[2] / n                                       # PSD, spread spectrum
    ld = engine.round_up(n, 64)
    W = _dev_batch(A, ld)
    ev, V = sym_eig(W, n)
    ev = ev.cpu().numpy()[:, :n]
    V = V.cpu().numpy()[:, :n, :n]
    # backward stable to the rounding of the rotations applied: ~1e-13 per round of a sweep
    # (nbk - 1 rounds, nbk = ld / 32 column blocks; LAPACK's own bound is ~n eps)
    tol = 1e-13 * (ld // 32)
    for b in range(3):
        ref = np.linalg.eigvalsh(A[b])
        nrm = np.abs(ref).max()
        assert np.abs(np.sort(ev[b]) - ref).max() <= tol * nrm, np.abs(np.sort(ev[b]) - ref).max() / nrm
        assert np.abs(V[b].T @ V[b] - np.eye(n)).max() <= tol
        assert np.abs((V[b] * ev[b]) @ V[b].T - A[b]).max() <= tol * nrm


def test_psd_projection_of_rank_deficient_covariance(device):
    rng = np.random.default_rng(7)
    n, T = 300, 120
    X = rng.normal(0, 0.02, size=(T, n))
    S = np.cov(X, rowvar=False)
    S[:5, :5] -= 1e-5 * np.eye(5)                                  # indefinite, rank-deficient
    ld = engine.round_up(n, 64)
    W = _dev_batch(S[None], ld)
    ev, V = sym_eig(W, n)
    out = torch.empty((1, ld, ld), dtype=torch.float64, device="cuda")
    _lib.check(_lib.load().pq_psd_form_batched(V.data_ptr(), V.stride(0), ev.data_ptr(), ev.stride(0), ld, n, 1,
                                                out.data_ptr(), out.stride(0), engine._stream()), "psd_form")
    L, Q = np.linalg.eigh(S)
    ref = (Q * np.maximum(L, 0)) @ Q.T
    assert np.abs(out[0, :n, :n].cpu().numpy() - ref).max() <= 5e-13 * (ld // 32) * np.abs(S).max()


def test_unconverged_sweeps_are_flagged_and_finished(device):
    """pq_sym_eig_converged: after too few sweeps the matrices are reported unconverged and
    sym_eig finishes them (never hands out unconverged eigenpairs); with enough sweeps every
    matrix converges and nothing is finished elsewhere."""
    rng = np.random.default_rng(11)
    n = 200
    M = rng.normal(size=(2, n, n))
    A = 0.5 * (M + M.transpose(0, 2, 1))
    ld = engine.round_up(n, 64)
    ev, V = sym_eig(_dev_batch(A, ld), n, max_sweeps=1)
    assert sym_eig.last_unconverged == 2
    ev, V = ev.cpu().numpy()[:, :n], V.cpu().numpy()[:, :n, :n]
    for b in range(2):
        ref = np.linalg.eigvalsh(A[b])
        nrm = np.abs(ref).max()
        assert np.abs(np.sort(ev[b]) - ref).max() <= 1e-12 * nrm
        assert np.abs((V[b] * ev[b]) @ V[b].T - A[b]).max() <= 1e-12 * nrm
    sym_eig(_dev_batch(A, ld), n)
    assert sym_eig.last_unconverged == 0
