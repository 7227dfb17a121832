# Host-side API restatement of PorQua (part of the GeomScale project; reference tree
# amolrpatil21/PorQua): src/helper_functions.py.  PorQua is Copyright (c) 2024 Cyril Bachelard and
# Minh Ha Ho and licensed under the GNU LGPL v3; this module keeps that API and its
# behaviour (quirks included) so that the MI355X engine is a drop-in, and is distributed
# under the same licence terms.
"""PD test / repair and small helpers (mirror of src/helper_functions.py:29-83).

``isPD`` is the batched device Cholesky (K2) info flag.  ``nearestPD`` is the reference's
Higham / D'Errico repair (src/helper_functions.py:29-58) on the device for a whole batch:
symmetrise, SVD polar projection onto the PSD cone, and -- while the K2 Cholesky still
fails -- the shift A3 += I (-lambda_min k^2 + spacing(||A||_F)), k = 1, 2, ...  The SVD and
the eigenvalues run on the GPU through rocSOLVER (torch.linalg; the repair is a library
factorisation, not a hot-path kernel), the PD tests on K2.  ``nearestPD_shift`` is the
cheaper repair used before (a spacing-scaled diagonal shift grown x4 until K2 succeeds);
for the covariance / Gram inputs on this path both agree to ~1e-15 relative.
"""
from __future__ import annotations

import numpy as np
import torch


def to_numpy(data):
    """src/helper_functions.py:82-83."""
    return None if data is None else data.to_numpy() if hasattr(data, "to_numpy") else data


def _as_batch(A):
    A = np.asarray(to_numpy(A), dtype=np.float64)
    return (A[None] if A.ndim == 2 else A), A.ndim == 2


def pd_info(A, device=None) -> np.ndarray:
    """Cholesky info per matrix (0 = positive definite), computed by K2 on the device."""
    from . import engine
    Ab, _ = _as_batch(A)
    n = Ab.shape[-1]
    qb = engine.QPBatch.from_dense(0.5 * (Ab + np.swapaxes(Ab, 1, 2)), np.zeros(Ab.shape[:2]), device=device)
    _, info = engine.factor_only(qb)
    return info.cpu().numpy()[: Ab.shape[0]]


def isPD(B, device=None) -> bool:
    """True when the (symmetric) matrix is positive definite (src/helper_functions.py:61-67)."""
    return bool(np.all(pd_info(B, device) == 0))


def nearestPD(A, device=None, max_attempts: int = 60):
    """src/helper_functions.py:29-58 on the device, for one matrix or a batch."""
    from . import engine
    Ab, single = _as_batch(A)
    dev = device or engine.default_device()
    At = torch.from_numpy(np.ascontiguousarray(Ab)).to(dev)
    B = 0.5 * (At + At.transpose(1, 2))
    _, s, Vh = torch.linalg.svd(B)                                   # :42
    H = Vh.transpose(1, 2) @ (s[:, :, None] * Vh)                      # :43  V' diag(s) V
    A2 = 0.5 * (B + H)                                                 # :44
    A3 = 0.5 * (A2 + A2.transpose(1, 2))                               # :45
    n = Ab.shape[-1]
    eye = torch.eye(n, dtype=torch.float64, device=dev)
    spacing = torch.from_numpy(np.array([np.spacing(np.linalg.norm(Ab[i])) for i in range(len(Ab))])).to(dev)
    todo = np.flatnonzero(pd_info(A3.cpu().numpy(), dev) != 0)         # :47 isPD
    k = 1
    while todo.size and k <= max_attempts:                             # :51-56
        t = torch.from_numpy(todo).to(dev)
        mineig = torch.linalg.eigvalsh(A3[t]).amin(1)                  # symmetric: eigvals are real
        A3[t] += eye[None] * (-mineig * k ** 2 + spacing[t])[:, None, None]
        k += 1
        ok = pd_info(A3[t].cpu().numpy(), dev) == 0
        todo = todo[~ok]
    out = A3.cpu().numpy()
    return out[0] if single else out


def nearestPD_shift(A, device=None, max_attempts: int = 60):
    """Symmetrise, then add the smallest spacing-scaled diagonal shift (x4 per attempt)
    that lets the device Cholesky succeed.  Works on one matrix or a batch."""
    from . import engine
    Ab, single = _as_batch(A)
    B = 0.5 * (Ab + np.swapaxes(Ab, 1, 2))
    out = B.copy()
    dev = device or engine.default_device()
    base = np.array([np.spacing(np.linalg.norm(Ab[i])) for i in range(len(Ab))])
    shift = np.zeros(len(Ab))
    todo = np.flatnonzero(pd_info(B, dev) != 0)
    step = base.copy()
    for _ in range(max_attempts):
        if todo.size == 0:
            break
        shift[todo] += step[todo]
        step[todo] *= 4.0
        trial = B[todo] + shift[todo, None, None] * np.eye(B.shape[-1])[None]
        ok = pd_info(trial, dev) == 0
        todo = todo[~ok]
    n = B.shape[-1]
    out = B + shift[:, None, None] * np.eye(n)[None]
    return out[0] if single else out


def nearest_pd_shift_device(P: torch.Tensor, ld: int, n: int, max_attempts: int = 60) -> torch.Tensor:
    """Device-resident variant for a (B, ld, ld) batch: returns the per-problem diagonal
    shift (tensor, B) that makes each P + shift I Cholesky-factorable."""
    from . import engine
    Bn = P.shape[0]
    dev = P.device
    fro = torch.linalg.matrix_norm(P, ord="fro").cpu().numpy()
    step = np.array([np.spacing(f) for f in fro])
    shift = np.zeros(Bn)
    qb = engine.QPBatch(n, Bn, 0, device=dev, has_box=False, P=P)
    qb.p_diag = torch.zeros(Bn, dtype=torch.float64, device=dev)
    _, info = engine.factor_only(qb)
    todo = np.flatnonzero(info.cpu().numpy() != 0)
    for _ in range(max_attempts):
        if todo.size == 0:
            break
        shift[todo] += step[todo]
        step[todo] *= 4.0
        qb.p_diag = torch.from_numpy(shift).to(dev)
        _, info = engine.factor_only(qb)
        todo = np.flatnonzero(info.cpu().numpy() != 0)
    return torch.from_numpy(shift).to(dev)
