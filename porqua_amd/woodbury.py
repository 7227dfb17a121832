"""Window-form normal equations for the device interior-point methods.

The LAD LP (src/optimization.py:296-345) and the QPs with both l1 linearisations
(src/qp_problems.py:40-118) are, in standard form, min c'x + (separable quadratic) s.t.
A x = b with bounds on x, where A's rows are the k = (few general rows) + T window rows over
the n assets (plus identity blocks).  An interior-point step then needs the m-space normal
matrix of a diagonally scaled A:

    M = U diag(w) U' + diag(d)        (k x k per problem, U the k x n row block, k < n)

(w = the assets' primal scaling theta_x, d = what the identity blocks contribute), not the
n x n x-space matrix: forming that costs 2 T n^2 flop and factoring it n^3 / 3 per problem and
iteration, M costs 2 k^2 n (T = 252, n = 1000: 8x fewer) and k^3 / 3.  Solving M directly,
instead of applying Woodbury to the x-space matrix, also avoids the cancellation of
Lam^-1 - Lam^-1 U'(...)^-1 U Lam^-1 once the scalings spread over 1e-12 .. 1e24 near the
optimum -- the classical normal-equations form of an LP interior-point method.

M is formed by the hand-written FP64-MFMA weighted SYRK ``pq_wgram_batched`` and factored
+ inverted by K2 (``pq_factor_batched``, invert = 2); ``apply`` multiplies by M itself
(two batched GEMVs over U), so callers refine every solve against the exact M.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib, engine

F64 = torch.float64


class NormalM:
    """M = U diag(w) U' + diag(d) for a batch; U (B, k, n) device tensor (unit column stride).
    ``factor(w, d)`` then ``solve(g)`` / ``apply(y)`` for g, y (B, k) or (B, k, m)."""

    def __init__(self, U):
        assert U.dim() == 3 and U.stride(2) == 1
        self.U = U
        self.B, self.k, self.n = U.shape
        from .lad import _NormalFactor
        self.nf = _NormalFactor(self.B, self.k, U.device)
        self.k_ld = self.nf.qb.ld
        self.w = self.d = self.Minv = None

    def _form(self, w, d):
        B, k, n = self.B, self.k, self.n
        P = self.nf.qb.P
        lib = _lib.load()
        stream = engine._stream()
        for s in range(0, B, 65535):
            c = min(B, s + 65535) - s
            U = self.U[s:s + c]
            _lib.check(lib.pq_wgram_batched(U.data_ptr(), U.stride(1), U.stride(0), k, n, c,
                                            w[s:].data_ptr(), w.stride(0), None, 0, d[s:].data_ptr(), d.stride(0),
                                            P[s:].data_ptr(), self.k_ld, P.stride(0), stream), "pq_wgram_batched")

    def factor(self, w, d, retries: int = 3):
        """w (B, n) >= 0, d (B, k) >= 0.  A problem whose Cholesky breaks down (K2 info != 0,
        e.g. equality rows that became dependent under the scaling) is refactored with a
        diagonal shift 1e-13 .. 1e-1 times its largest diagonal entry.  Returns a bool tensor
        of the problems that still failed; the caller freezes those."""
        self.w = w.contiguous()
        self.d = d.contiguous()
        nf = self.nf
        lib = _lib.load()
        dd = self.d
        bad = None
        for attempt in range(retries + 1):
            self._form(self.w, dd)
            _lib.check(lib.pq_factor_batched(ctypes.byref(nf.pb), ctypes.byref(nf.st), None, 0,
                                             ctypes.byref(nf.s), 2, engine._stream()), "pq_factor_batched (M)")
            bad = (nf.ws.info != 0) | ~torch.isfinite(self.w).all(1) | ~torch.isfinite(dd).all(1)
            if attempt == retries or not bool(bad.any()):
                break
            Md = nf.qb.P.diagonal(dim1=1, dim2=2)[:, :self.k]
            scale = Md.abs().amax(1, keepdim=True).clamp(min=1e-300)
            dd = torch.where(bad[:, None], dd + scale * 10.0 ** (-13 + 4 * attempt), dd)
        self.Minv = nf.ws.K[:, :self.k, :self.k]
        return bad

    def apply(self, y):
        """M y (exact: the unshifted diagonal)."""
        vec = y.dim() == 2
        Y = y.unsqueeze(2) if vec else y
        out = torch.bmm(self.U, torch.bmm(self.U.transpose(1, 2), Y) * self.w.unsqueeze(2)) + self.d.unsqueeze(2) * Y
        return out.squeeze(2) if vec else out

    def solve(self, g, refine: int = 2):
        """M^-1 g, refined ``refine`` times against the exact M."""
        from .lad import _mv
        vec = g.dim() == 2
        G = (g.unsqueeze(2) if vec else g).contiguous()
        Y = _mv(self.Minv, G)
        for _ in range(refine):
            Y = Y + _mv(self.Minv, (G - self.apply(Y)).contiguous())
        return Y.squeeze(2) if vec else Y
