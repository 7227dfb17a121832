#!/usr/bin/env python3
"""Batched symmetric eigendecomposition of 64 window Grams (T = 252, the config-5 EigCap
input): torch.linalg.eigh against rocSOLVER's strided-batched syevd / syevj called directly
(torch's own bundled librocsolver) and the hand-written block-Jacobi kernels
(helper_functions.sym_eig, jacobi.hip).  Experiment tool: python tools/exp_eigh.py"""
import ctypes
import json
import os
import time

import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
TL = os.path.join(os.path.dirname(torch.__file__), "lib")


def rocsolver():
    rb = ctypes.CDLL(os.path.join(TL, "librocblas.so"))
    rs = ctypes.CDLL(os.path.join(TL, "librocsolver.so"))
    h = ctypes.c_void_p()
    assert rb.rocblas_create_handle(ctypes.byref(h)) == 0
    assert rb.rocblas_set_stream(h, ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)) == 0
    return rb, rs, h


def main():
    dev = torch.device("cuda", 0)
    nb, T = 64, 252
    g = torch.Generator(device="cpu").manual_seed(1)
    X = torch.randn((nb, T, 5000), generator=g, dtype=torch.float64).to(dev) * 0.02
    X -= X.mean(1, keepdim=True)
    G = X @ X.mT
    out = {}

    def timed(fn, reps=3):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            r = fn()
        torch.cuda.synchronize()
        return r, (time.perf_counter() - t0) / reps * 1e3

    (ev, V), ms = timed(lambda: torch.linalg.eigh(G))
    out["torch_eigh_ms"] = ms
    ref = ev
    rb, rs, h = rocsolver()
    ld = T
    info = torch.zeros(nb, dtype=torch.int32, device=dev)
    D = torch.empty((nb, T), dtype=torch.float64, device=dev)
    E = torch.empty((nb, T), dtype=torch.float64, device=dev)

    def syevd():
        A = G.clone()
        st = rs.rocsolver_dsyevd_strided_batched(h, 211, 122, T, ctypes.c_void_p(A.data_ptr()), ld,
                                                 ctypes.c_int64(T * T), ctypes.c_void_p(D.data_ptr()),
                                                 ctypes.c_int64(T), ctypes.c_void_p(E.data_ptr()), ctypes.c_int64(T),
                                                 ctypes.c_void_p(info.data_ptr()), nb)
        assert st == 0, st
        return A
    A, ms = timed(syevd)
    out["rocsolver_syevd_batched_ms"] = ms
    out["syevd_max_eig_err"] = float((D - ref).abs().max())
    res = torch.empty(nb, dtype=torch.float64, device=dev)
    nsw = torch.empty(nb, dtype=torch.int32, device=dev)
    W = torch.empty((nb, T), dtype=torch.float64, device=dev)

    def syevj():
        A = G.clone()
        st = rs.rocsolver_dsyevj_strided_batched(h, 252, 211, 122, T, ctypes.c_void_p(A.data_ptr()), ld,
                                                 ctypes.c_int64(T * T), ctypes.c_double(0.0),
                                                 ctypes.c_void_p(res.data_ptr()), 100,
                                                 ctypes.c_void_p(nsw.data_ptr()), ctypes.c_void_p(W.data_ptr()),
                                                 ctypes.c_int64(T), ctypes.c_void_p(info.data_ptr()), nb)
        assert st == 0, st
        return A
    A, ms = timed(syevj)
    out["rocsolver_syevj_batched_ms"] = ms
    out["syevj_max_eig_err"] = float((W - ref).abs().max())
    out["syevj_sweeps_max"] = int(nsw.max())
    from porqua_amd.helper_functions import sym_eig
    Gp = torch.zeros((nb, 256, 256), dtype=torch.float64, device=dev)

    def jac():
        Gp.zero_()
        Gp[:, :T, :T] = G
        return sym_eig(Gp, T)
    (evj, Vj), ms = timed(jac)
    out["jacobi_sym_eig_ms"] = ms
    out["jacobi_max_eig_err"] = float((torch.sort(evj[:, :T], 1)[0] - ref).abs().max())
    Vt = Vj[:, :T, :T]
    out["jacobi_max_recon_err"] = float((Vt @ torch.diag_embed(evj[:, :T]) @ Vt.mT - G).abs().max())
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
