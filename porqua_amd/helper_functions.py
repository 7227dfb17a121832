# Host-side API restatement of PorQua (part of the GeomScale project; reference tree
# amolrpatil21/PorQua): src/helper_functions.py.  PorQua is Copyright (c) 2024 Cyril Bachelard and
# Minh Ha Ho and licensed under the GNU LGPL v3; this module keeps that API and its
# behaviour (quirks included) so that the MI355X engine is a drop-in, and is distributed
# under the same licence terms.
"""PD test / repair and small helpers (mirror of src/helper_functions.py:29-83).

``isPD`` is the batched device Cholesky (K2) info flag.  ``nearestPD`` is the reference's
Higham / D'Errico repair (src/helper_functions.py:29-58) on the device for a whole batch,
entirely in hand-written kernels and without host copies of the matrices:
  * B = (A + A')/2; the SVD projection H = V' diag(s) V, A2 = (B + H)/2 equals
    Q max(L, 0) Q' for the symmetric eigendecomposition B = Q L Q' (s = |L|), computed by the
    batched block-Jacobi eigensolver (pq_sym_eig_batched) and one MFMA product
    (pq_psd_form_batched) of the negative part: A2 = B + Q max(-L, 0) Q'; A3 = (A2 + A2')/2;
  * while K2's Cholesky of A3 fails: A3 += I (-lambda_min k^2 + spacing(||A||_F)), k = 1, 2, ...
    with lambda_min the smallest eigenvalue of the formed A3 (np.linalg.eigvals in the
    reference), from the Jacobi eigensolver on Q' A3 Q (warm: nearly diagonal).
The only host traffic is the per-matrix Cholesky info vector of each loop pass.
``nearestPD_shift`` is the cheaper repair used before (a spacing-scaled diagonal shift grown
x4 until K2 succeeds).
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

F64 = torch.float64


def to_numpy(data):
    """src/helper_functions.py:82-83."""
    return None if data is None else data.to_numpy() if hasattr(data, "to_numpy") else data


def _as_batch(A):
    A = np.asarray(to_numpy(A), dtype=np.float64)
    return (A[None] if A.ndim == 2 else A), A.ndim == 2


def pd_info_device(S: torch.Tensor, n: int, chunk: int = 1024) -> torch.Tensor:
    """Cholesky info per matrix (0 = positive definite) of the device batch S (B, ld, ld)
    (symmetric, the lower triangle is read), computed by K2 in chunks of ``chunk`` matrices
    (the factor workspace is chunk x ld x ld) -> int32 device tensor (B,)."""
    from . import _lib, engine
    B = S.shape[0]
    info = torch.zeros(B, dtype=torch.int32, device=S.device)
    lib = _lib.load()
    st = engine.Settings(sigma=0.0).to_c()
    for s0 in range(0, B, chunk):
        e0 = min(B, s0 + chunk)
        qb = engine.QPBatch(n, e0 - s0, 0, device=S.device, has_box=False, P=S[s0:e0])
        if S.shape[-1] != qb.ld or S.stride(1) != qb.ld:
            Pp = torch.zeros((e0 - s0, qb.ld, qb.ld), dtype=F64, device=S.device)
            Pp[:, :n, :n] = S[s0:e0, :n, :n]
            qb.P = Pp
        ws = engine.Workspace(qb)
        pb, sw = qb.c_struct(), ws.c_struct()
        pb.lb = pb.ub = None
        strm = engine._stream()
        _lib.check(lib.pq_init_state(ctypes.byref(pb), ctypes.byref(sw), None, 0, ctypes.byref(st), strm), "init")
        _lib.check(lib.pq_factor_batched(ctypes.byref(pb), ctypes.byref(sw), None, 0, ctypes.byref(st), 0, strm),
                   "pq_factor_batched (isPD)")
        info[s0:e0] = ws.info
    return info


def pd_info(A, device=None) -> np.ndarray:
    """Cholesky info per matrix (0 = positive definite), computed by K2 on the device."""
    from . import engine
    Ab, _ = _as_batch(A)
    dev = device or engine.default_device()
    n = Ab.shape[-1]
    S = torch.from_numpy(np.ascontiguousarray(0.5 * (Ab + np.swapaxes(Ab, 1, 2)))).to(dev)
    return pd_info_device(S, n).cpu().numpy()


def isPD(B, device=None) -> bool:
    """True when the (symmetric) matrix is positive definite (src/helper_functions.py:61-67)."""
    return bool(np.all(pd_info(B, device) == 0))


def sym_eig(A: torch.Tensor, n: int, vectors: bool = True, max_sweeps: int = 30, tol: float = 1e-14):
    """Symmetric eigendecomposition of the device batch A (B, ld, ld), ld a multiple of 64,
    by the hand-written block-Jacobi kernels (pq_sym_eig_batched).  A is overwritten
    (diagonalised).  Returns (evals (B, ld): eigenvalue j of matrix b at evals[b, j], j < n,
    unsorted; V (B, ld, ld) with the eigenvectors as columns, or None).  A matrix still
    unconverged after ``max_sweeps`` (pq_sym_eig_converged) is finished by rocSOLVER's eigh
    from its partially diagonalised state; ``sym_eig.last_unconverged`` counts them."""
    from . import _lib, engine
    lib = _lib.load()
    B, ld = A.shape[0], A.shape[-1]
    if ld % 64 or A.stride(2) != 1 or A.stride(1) != ld:
        raise ValueError("sym_eig: contiguous (B, ld, ld) with ld a multiple of 64 expected")
    dev = A.device
    w = int(lib.pq_sym_eig_work_doubles(ld))
    work = torch.empty((B, w), dtype=F64, device=dev)
    V = torch.empty((B, ld, ld), dtype=F64, device=dev) if vectors else None
    ev = torch.empty((B, ld), dtype=F64, device=dev)
    for s0 in range(0, B, 65535):
        e0 = min(B, s0 + 65535)
        _lib.check(lib.pq_sym_eig_batched(A[s0:].data_ptr(), ld, A.stride(0), n, e0 - s0,
                                          None if V is None else V[s0:].data_ptr(), ld * ld, ev[s0:].data_ptr(),
                                          ld, work[s0:].data_ptr(), w, max_sweeps, tol, engine._stream()),
                   "pq_sym_eig_batched")
    # convergence (one host sync): a matrix whose last sweep still rotated is finished by
    # rocSOLVER from where the Jacobi sweeps left it -- A is now Q' A0 Q with Q = V, so
    # eigh(A) = (lam, W) gives A0's eigenpairs (lam, Q W) -- never used unconverged
    conv = torch.empty(B, dtype=torch.int32, device=dev)
    for s0 in range(0, B, 65535):
        e0 = min(B, s0 + 65535)
        _lib.check(lib.pq_sym_eig_converged(work[s0:].data_ptr(), ld, w, e0 - s0, max_sweeps, conv[s0:].data_ptr(),
                                            engine._stream()), "pq_sym_eig_converged")
    bad = torch.nonzero(conv == 0).flatten()
    if bad.numel():
        As = A[bad]
        As = 0.5 * (As + As.mT)
        lam, Wr = torch.linalg.eigh(As[:, :n, :n])
        ev[bad] = 0.0
        ev[bad, :n] = lam
        if V is not None:
            V[bad, :, :n] = V[bad][:, :, :n] @ Wr
        Ad = torch.zeros((len(bad), ld, ld), dtype=F64, device=dev)
        Ad[:, :n, :n] = torch.diag_embed(lam)
        A[bad] = Ad                                                    # diagonalised, as on convergence
    sym_eig.last_unconverged = int(bad.numel())
    return ev, V


def _tile_gemm(A, ta, B, tb):
    from . import _lib, engine
    C = torch.empty_like(A)
    ld = A.shape[-1]
    _lib.check(_lib.load().pq_tile_gemm_batched(A.data_ptr(), A.stride(0), int(ta), B.data_ptr(), B.stride(0),
                                                int(tb), C.data_ptr(), C.stride(0), ld, A.shape[0],
                                                engine._stream()), "pq_tile_gemm_batched")
    return C


def _spacing(x: torch.Tensor) -> torch.Tensor:
    """np.spacing for positive finite FP64 values, on the device."""
    _, e = torch.frexp(x)
    return torch.ldexp(torch.ones_like(x), (e - 53).to(torch.int32))


def nearestPD_device(A: torch.Tensor, n: int, max_attempts: int = 60) -> torch.Tensor:
    """src/helper_functions.py:29-58 for the device batch A (B, n, n) or (B, ld, ld) (entries
    beyond n ignored) -> (B, ld, ld) device tensor, ld = round_up(n, 64), zero padded."""
    from . import _lib, engine
    B = A.shape[0]
    ld = engine.round_up(n, 64)
    dev = A.device
    An = A[:, :n, :n]
    Bm = torch.zeros((B, ld, ld), dtype=F64, device=dev)
    Bm[:, :n, :n] = 0.5 * (An + An.transpose(1, 2))                       # :40
    spacing = _spacing(torch.linalg.matrix_norm(An, ord="fro"))          # :48 np.spacing(norm(A))
    W = Bm.clone()
    ev, V = sym_eig(W, n)                                                # :42 (B = Q L Q')
    # :43-44 (B + H)/2 = Q max(L, 0) Q' = B - Q min(L, 0) Q': formed as B plus the (tiny)
    # negative part, so the eigensolver's rounding (~n eps of the whole spectrum for the
    # Jacobi sweeps) only touches that correction and the result keeps B's own accuracy
    # (numpy's SVD form and this one agree to ~1e-15 at n = 1000; the product of the full
    # spectrum left 4e-12, profiles/r04c_pytest.txt)
    nev = -ev
    E = torch.empty_like(Bm)
    _lib.check(_lib.load().pq_psd_form_batched(V.data_ptr(), V.stride(0), nev.data_ptr(), nev.stride(0), ld, n, B,
                                                E.data_ptr(), E.stride(0), engine._stream()),
               "pq_psd_form_batched")                                    # Q max(-L, 0) Q'
    A2 = Bm + E
    A3 = 0.5 * (A2 + A2.transpose(1, 2))                                 # :45
    todo = torch.nonzero(pd_info_device(A3, n) != 0).flatten()          # :47 isPD
    diag = torch.arange(n, device=dev)
    k = 1
    while todo.numel() and k <= max_attempts:                            # :51-56
        At, Vt = A3[todo].contiguous(), V[todo].contiguous()
        M = _tile_gemm(Vt, 1, _tile_gemm(At, 0, Vt, 0), 0)              # Q' A3 Q: eigvals(A3)
        M = 0.5 * (M + M.transpose(1, 2))
        evm, _ = sym_eig(M, n, vectors=False)
        mineig = evm[:, :n].amin(1)
        A3[todo[:, None], diag[None, :], diag[None, :]] += (-mineig * k ** 2 + spacing[todo])[:, None]
        k += 1
        ok = pd_info_device(A3[todo], n) == 0
        todo = todo[~ok]
    return A3


def nearestPD(A, device=None, max_attempts: int = 60):
    """src/helper_functions.py:29-58 on the device, for one matrix or a batch (host arrays
    in and out; nearestPD_device keeps them on the device)."""
    from . import engine
    Ab, single = _as_batch(A)
    dev = device or engine.default_device()
    n = Ab.shape[-1]
    A3 = nearestPD_device(torch.from_numpy(np.ascontiguousarray(Ab)).to(dev), n, max_attempts)
    out = A3[:, :n, :n].cpu().numpy()
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
