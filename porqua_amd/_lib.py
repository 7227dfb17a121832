"""ctypes binding of the in-tree HIP library ``libporqua_hip.so`` (see include/porqua_hip.h).

The product path has no CPU fallback: if the library is missing or no GPU is visible the
calls raise ``PorquaHipError``.  Structures mirror the C ABI field for field.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# PQ_LIB_PATH: an alternative build of the same library (e.g. the PQ_PROFILE phase-timing build)
LIB_PATH = os.environ.get("PQ_LIB_PATH") or os.path.join(_HERE, "libporqua_hip.so")

c_int32 = ctypes.c_int32
c_int64 = ctypes.c_int64
c_dp = ctypes.c_void_p   # device pointers are passed as plain integers

PQ_UNSOLVED = 0
PQ_SOLVED = 1
PQ_SOLVED_INACCURATE = 2
PQ_MAX_ITER = 3
PQ_NEED_REFACTOR = 4
PQ_PRIMAL_INFEASIBLE = -3
PQ_DUAL_INFEASIBLE = -4
PQ_NON_CONVEX = -5

PQ_PG_RECORD = 384                   # doubles per problem of the grouped polish record
PQ_PG_PASS_SCRATCH = 123537          # doubles per slide group of the split polish window passes
PQ_PG_PENDING, PQ_PG_DONE, PQ_PG_FALLBACK, PQ_PG_SKIP = range(4)
PQ_PG_STATE = 3                      # record field holding the state
PQ_PG_K, PQ_PG_SC, PQ_PG_W = 0, 5, 320   # record fields: free count, problem scale, wide round

PQ_OUT_OBJ, PQ_OUT_PRIM, PQ_OUT_DUAL, PQ_OUT_GAP, PQ_OUT_RHO, PQ_OUT_NFREE, PQ_OUT_ROUNDS = range(7)
PQ_OUT_FIELDS = 8


def work_doubles(ld: int, mg_pad: int) -> int:
    """PQ_WORK_DOUBLES of include/porqua_hip.h."""
    return (9 + mg_pad) * ld + 512


class PorquaHipError(RuntimeError):
    pass


class PQProblem(ctypes.Structure):
    _fields_ = [
        ("n", c_int32), ("ld", c_int32), ("batch", c_int32), ("mg", c_int32),
        ("P", c_dp), ("P_stride", c_int64),
        ("p_scale", c_dp), ("p_diag", c_dp),
        ("q", c_dp), ("q_stride", c_int64),
        ("Cg", c_dp), ("Cg_stride", c_int64),
        ("lg", c_dp), ("ug", c_dp), ("g_stride", c_int64),
        ("lb", c_dp), ("ub", c_dp), ("box_stride", c_int64),
    ]


class PQState(ctypes.Structure):
    _fields_ = [
        ("K", c_dp), ("K_stride", c_int64),
        ("Dt", c_dp), ("Dt_stride", c_int64),
        ("x", c_dp), ("Px", c_dp),
        ("z", c_dp), ("y", c_dp),
        ("m_ld", c_int32), ("mg_pad", c_int32),
        ("rho", c_dp),
        ("iters", c_dp), ("status", c_dp), ("info", c_dp),
        ("out", c_dp),
        ("work", c_dp), ("work_stride", c_int64),
    ]


class PQSettings(ctypes.Structure):
    _fields_ = [
        ("rho0", ctypes.c_double), ("rho0_rel", ctypes.c_double),
        ("sigma", ctypes.c_double), ("alpha", ctypes.c_double),
        ("eps_abs", ctypes.c_double), ("eps_rel", ctypes.c_double),
        ("rho_min", ctypes.c_double), ("rho_max", ctypes.c_double),
        ("adapt_tol", ctypes.c_double), ("eq_scale", ctypes.c_double),
        ("delta", ctypes.c_double), ("dual_tol", ctypes.c_double),
        ("max_iter", c_int32), ("adapt_interval", c_int32), ("polish", c_int32),
        ("polish_rounds", c_int32), ("refine_iters", c_int32),
        ("polish_fix_rel", ctypes.c_double),
        ("polish_inner", ctypes.c_int32), ("min_iter", ctypes.c_int32),
        ("polish_release_rel", ctypes.c_double),
    ]


class PQLowRank(ctypes.Structure):
    _fields_ = [
        ("panel", c_dp), ("ldp", c_int64),
        ("rows", c_dp), ("tlen", c_dp), ("tmax", c_int32),
        ("mu", c_dp), ("mu_stride", c_int64),
        ("w_scale", c_dp),
        ("dg", c_dp), ("dg_stride", c_int64),
    ]


class PQGcap(ctypes.Structure):
    _fields_ = [
        ("gdates", c_dp), ("ngroups", c_int32),
        ("urows", c_dp), ("ucnt", c_dp), ("uoff", c_dp), ("umax", c_int32),
        ("gidx", c_dp), ("grho", c_dp),
        ("M", c_dp), ("Minv", c_dp), ("k_ld", c_int32), ("M_stride", c_int64),
        ("aq", c_dp), ("aq_stride", c_int64),
        ("hinv", c_dp), ("ldh", c_int32),
        ("gmax", c_int32),
    ]


class PQPgWide(ctypes.Structure):
    """pq_pg_wide: the wide rounds of the grouped polish (include/porqua_hip.h)."""
    _fields_ = [
        ("gc", ctypes.POINTER(PQGcap)),
        ("pc", c_dp), ("ldpc", c_int64), ("r0", c_int32), ("cc", c_dp),
        ("nzr", c_dp), ("nzv", c_dp), ("nzmax", c_int32),
        ("wscr", c_dp), ("wscr_stride", c_int64),
        ("refine_steps", c_int32),
    ]


PQ_PG_WMB = 8                        # bordered rows per date of a wide round


def pg_wscr(k_ld: int) -> int:
    """PQ_PG_WSCR(k_ld): doubles per problem of the wide rounds' scratch."""
    return 2 * PQ_PG_WMB * int(k_ld)


_EXPORTS = {
    "pq_version": ([], c_int32),
    "pq_last_error": ([], ctypes.c_char_p),
    "pq_window_mean": ([c_dp, c_int64, c_int32, c_dp, c_dp, c_int32, c_int32, c_dp, c_int64, c_dp], c_int32),
    "pq_window_geomean": ([c_dp, c_int64, c_int32, c_dp, c_dp, c_int32, c_int32, c_dp, c_int64, c_dp], c_int32),
    "pq_window_geomean_grouped": ([c_dp, c_int64, c_int32, c_dp, c_int32, c_dp, c_int32, c_dp, c_dp, c_dp,
                                   c_int64, c_dp], c_int32),
    "pq_cov_batched": ([c_dp, c_int64, c_int32, c_dp, c_dp, c_int32, c_int32, c_int32, c_dp, c_int64,
                        c_dp, c_int32, c_int64, c_dp], c_int32),
    "pq_cov_slide_batched": ([c_dp, c_int64, c_int32, c_dp, c_dp, c_int32, c_int32, c_int32, c_dp, c_int64,
                              c_dp, c_int32, c_int64, c_dp, c_int32, c_dp, c_int32, c_dp], c_int32),
    "pq_window_sumsq": ([c_dp, c_int64, c_int32, c_dp, c_dp, c_int32, c_int32, c_dp, c_int64, c_dp, c_int64,
                         c_dp], c_int32),
    "pq_window_nanmean": ([c_dp, c_int64, c_int32, c_dp, c_dp, c_int32, c_int32, c_dp, c_int64, c_int32, c_dp],
                          c_int32),
    "pq_cov_pairwise_batched": ([c_dp, c_int64, c_int32, c_dp, c_dp, c_int32, c_int32, c_dp, c_int64, c_dp,
                                 c_int32, c_int64, c_dp], c_int32),
    "pq_window_moments_grouped": ([c_dp, c_int64, c_int32, c_dp, c_int32, c_dp, c_int32, c_dp, c_dp, c_dp,
                                   c_int64, c_dp, c_int64, c_dp], c_int32),
    "pq_init_state_lr": ([ctypes.POINTER(PQLowRank), ctypes.POINTER(PQProblem), ctypes.POINTER(PQState), c_dp,
                          c_int32, ctypes.POINTER(PQSettings), c_dp], c_int32),
    "pq_polish_w_batched": ([ctypes.POINTER(PQLowRank), ctypes.POINTER(PQProblem), ctypes.POINTER(PQState),
                             c_dp, c_int32, ctypes.POINTER(PQSettings), c_int32, c_int32, c_dp, c_int64,
                             c_int32, c_dp], c_int32),
    "pq_gram_xy_grouped": ([c_dp, c_int64, c_int32, c_dp, c_dp, c_int32, c_dp, c_int32, c_dp, c_dp, c_dp,
                            c_int64, c_dp, c_dp, c_int64, c_dp], c_int32),
    "pq_gram_xy_batched": ([c_dp, c_int64, c_int32, c_dp, c_dp, c_dp, c_int32, c_int32, c_dp, c_int64,
                            c_dp, c_dp], c_int32),
    "pq_init_state": ([ctypes.POINTER(PQProblem), ctypes.POINTER(PQState), c_dp, c_int32,
                       ctypes.POINTER(PQSettings), c_dp], c_int32),
    "pq_factor_batched": ([ctypes.POINTER(PQProblem), ctypes.POINTER(PQState), c_dp, c_int32,
                           ctypes.POINTER(PQSettings), c_int32, c_dp], c_int32),
    "pq_factor_large": ([ctypes.POINTER(PQProblem), ctypes.POINTER(PQState), c_dp, c_int32,
                         ctypes.POINTER(PQSettings), c_int32, c_dp, c_int64, c_dp], c_int32),
    "pq_sym_eig_work_doubles": ([c_int32], c_int64),
    "pq_sym_eig_batched": ([c_dp, c_int32, c_int64, c_int32, c_int32, c_dp, c_int64, c_dp, c_int64, c_dp, c_int64,
                            c_int32, ctypes.c_double, c_dp], c_int32),
    "pq_sym_eig_converged": ([c_dp, c_int32, c_int64, c_int32, c_int32, c_dp, c_dp], c_int32),
    "pq_psd_form_batched": ([c_dp, c_int64, c_dp, c_int64, c_int32, c_int32, c_int32, c_dp, c_int64, c_dp], c_int32),
    "pq_tile_gemm_batched": ([c_dp, c_int64, c_int32, c_dp, c_int64, c_int32, c_dp, c_int64, c_int32, c_int32,
                              c_dp], c_int32),
    "pq_admm_batched": ([ctypes.POINTER(PQProblem), ctypes.POINTER(PQState), c_dp, c_int32,
                         ctypes.POINTER(PQSettings), c_int32, c_dp], c_int32),
    "pq_polish_batched": ([ctypes.POINTER(PQProblem), ctypes.POINTER(PQState), c_dp, c_int32,
                           ctypes.POINTER(PQSettings), c_dp], c_int32),
    "pq_admm_lr_grouped": ([ctypes.POINTER(PQLowRank), ctypes.POINTER(PQProblem), ctypes.POINTER(PQState),
                            c_dp, c_int32, c_int64, c_dp, c_int32, c_dp, c_dp, c_dp, c_int32,
                            ctypes.POINTER(PQSettings), c_int32, c_dp, c_int64, c_int32, c_dp, c_dp, c_dp,
                            c_int32, c_dp], c_int32),
    "pq_admm_lr_sweep": ([ctypes.POINTER(PQLowRank), ctypes.POINTER(PQProblem), ctypes.POINTER(PQState),
                          c_dp, c_int32, c_int64, c_dp, c_int32, ctypes.POINTER(PQSettings), c_int32, c_dp,
                          c_int64, c_int32, c_dp, c_int32, c_dp, c_int64, c_dp], c_int32),
    "pq_sweep_scratch_doubles": ([c_int32, c_int32, c_int32], c_int64),
    "pq_polish_lr_batched": ([ctypes.POINTER(PQLowRank), ctypes.POINTER(PQProblem), ctypes.POINTER(PQState),
                              c_dp, c_int32, ctypes.POINTER(PQSettings), c_dp], c_int32),
    "pq_lr_capacitance": ([ctypes.POINTER(PQLowRank), ctypes.POINTER(PQProblem), ctypes.POINTER(PQState),
                           c_dp, c_int32, ctypes.POINTER(PQSettings), c_dp, c_int32, c_int64, c_dp], c_int32),
    "pq_lr_band_gram": ([c_dp, c_int64, c_int32, c_int32, c_int32, c_int32, c_dp, c_int64, c_dp, c_int32, c_int32,
                         c_dp, c_int64, c_dp], c_int32),
    "pq_lr_capacitance_band": ([ctypes.POINTER(PQLowRank), ctypes.POINTER(PQProblem), ctypes.POINTER(PQState),
                                c_dp, c_int32, ctypes.POINTER(PQSettings), c_dp, c_int64, c_int32, c_dp, c_int64,
                                c_dp, c_dp, c_int32, c_int64, c_dp], c_int32),
    "pq_admm_lr_batched": ([ctypes.POINTER(PQLowRank), ctypes.POINTER(PQProblem), ctypes.POINTER(PQState),
                            c_dp, c_int32, c_int64, c_dp, c_int32, ctypes.POINTER(PQSettings), c_int32,
                            c_dp], c_int32),
    "pq_polish_grouped_init": ([ctypes.POINTER(PQLowRank), ctypes.POINTER(PQProblem), ctypes.POINTER(PQState),
                                c_dp, ctypes.POINTER(PQSettings), c_dp], c_int32),
    "pq_polish_grouped_round": ([ctypes.POINTER(PQLowRank), ctypes.POINTER(PQProblem), ctypes.POINTER(PQState),
                                 c_dp, c_int32, c_dp, c_int32, c_dp, c_dp, c_dp, c_int32,
                                 ctypes.POINTER(PQSettings), c_dp, ctypes.POINTER(PQPgWide), c_dp], c_int32),
    "pq_gcap_assemble": ([ctypes.POINTER(PQLowRank), ctypes.POINTER(PQProblem), ctypes.POINTER(PQGcap),
                          ctypes.POINTER(PQSettings), c_dp, c_int64, c_int32, c_dp, c_int64, c_dp, c_dp], c_int32),
    "pq_gcap_prepare": ([ctypes.POINTER(PQLowRank), ctypes.POINTER(PQProblem), ctypes.POINTER(PQState),
                         ctypes.POINTER(PQGcap), ctypes.POINTER(PQSettings), c_dp, c_int32, c_dp, c_int64, c_int32,
                         c_dp, c_int64, c_dp], c_int32),
    "pq_admm_lr_gcap": ([ctypes.POINTER(PQLowRank), ctypes.POINTER(PQProblem), ctypes.POINTER(PQState),
                         ctypes.POINTER(PQGcap), ctypes.POINTER(PQSettings), c_int32, c_dp, c_int64, c_int32, c_dp,
                         c_dp, c_dp, c_int32, c_dp], c_int32),
    "pq_eigcap_form": ([ctypes.POINTER(PQLowRank), ctypes.POINTER(PQProblem), ctypes.POINTER(PQState),
                        ctypes.POINTER(PQSettings), c_dp, c_dp, c_dp, c_dp, c_dp, c_int32, c_dp, c_int32, c_dp,
                        c_int64, c_dp, c_dp], c_int32),
    "pq_gemv_batched": ([c_dp, c_int64, c_int64, c_int32, c_int32, c_int32, c_int32, c_dp, c_int64, c_dp,
                         c_int64, c_dp], c_int32),
    "pq_workspace_bytes": ([c_int32, c_int32, c_int32, c_int32, c_int32, c_int32], c_int64),
    "pq_simulate_periods": ([c_dp, c_int64, c_int32, c_dp, c_int64, c_dp, c_dp, c_int32, c_dp, c_dp,
                             ctypes.c_double, ctypes.c_double, c_dp, c_dp, c_int64, c_dp, c_int32, c_dp], c_int32),
    "pq_lad_mv_batched": ([c_dp, c_int64, c_int64, c_int32, c_int32, c_dp, c_int64, c_int32, c_dp, c_int64,
                           c_dp, c_int64, c_dp], c_int32),
    "pq_wgram_batched": ([c_dp, c_int64, c_int64, c_int32, c_int32, c_int32, c_dp, c_int64, c_dp, c_int64,
                          c_dp, c_int64, c_dp, c_int32, c_int64, c_dp], c_int32),
}

_lib = None


def load() -> ctypes.CDLL:
    """Load the HIP library (raises PorquaHipError if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise PorquaHipError(
            f"{LIB_PATH} not found: build it with `make -C porqua_amd/csrc` "
            "(or __graft_entry__.build()); there is no CPU fallback")
    lib = ctypes.CDLL(LIB_PATH)
    for name, (args, res) in _EXPORTS.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = res
    _lib = lib
    return lib


def exported_symbols():
    return list(_EXPORTS)


def check(rc: int, what: str):
    if rc != 0:
        msg = load().pq_last_error().decode(errors="replace")
        raise PorquaHipError(f"{what} failed (rc={rc}): {msg}")
