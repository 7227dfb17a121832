"""Device engine: batched covariance + batched dense QP solve on MI355X through the C ABI.

Host code only stages data (PyTorch-ROCm tensors for device memory and the current HIP
stream) and drives the kernels of ``libporqua_hip.so``:

  K1 pq_window_mean / pq_cov_batched / pq_gram_xy_batched / pq_window_geomean
  K2 pq_factor_batched   (KKT formation + Cholesky [+ inverse])
  K3 pq_admm_batched     (OSQP-style ADMM, per-problem convergence)
  K4 pq_polish_batched   (active-set polish + exact residuals)

There is deliberately no CPU fallback: without the library or a GPU every entry point
raises ``PorquaHipError``.
"""
from __future__ import annotations

import os
import ctypes
import dataclasses
from dataclasses import dataclass

import numpy as np
import torch

from . import _lib

F64 = torch.float64


def round_up(v: int, m: int) -> int:
    return ((int(v) + m - 1) // m) * m


def _ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def default_device() -> torch.device:
    if not torch.cuda.is_available():
        raise _lib.PorquaHipError("no HIP device visible: the MI355X engine has no CPU fallback")
    return torch.device("cuda", torch.cuda.current_device())


@dataclass
class Settings:
    """ADMM / polish settings.  OSQP defaults except a scale-aware initial rho (4 x mean
    diag P, adapted every 60 iterations: no refactorisation on the n = 1000 min-variance
    windows, tests/engine_model.py), the stopping tolerance and the polish settings.  ADMM
    only has to reach an approximate point whose active set the polish can correct: measured
    on config 3 (round 2 kernels, bench.py --set eps_abs=... eps_rel=...) eps 2e-3 gives 20 ADMM iterations +
    2.7 polish rounds against 21 + 2.6 at 1e-3 and 18 + 2.9 at 4e-3 (about 2 % apart; configs
    2, 4 and 5 also gain), alpha 1.7 / 1.8 trade 10 / 29 more ADMM iterations for 0.7 / 1.5
    fewer polish rounds and lose; round 1 measured 1e-3 against 1e-4 (95.7k vs 85.1k QPs/s).
    Every answer is still KKT-checked and a rejected polish resumes ADMM to eps_retry.
    Passed through ``params`` of the reference API."""
    rho0: float = 0.1
    rho0_rel: float = 4.0      # initial rho = rho0_rel * mean(diag P) (0: use rho0)
    sigma: float = 1e-6
    alpha: float = 1.6
    eps_abs: float = 2e-3      # ADMM stop before the polish (twice OSQP's default; the polish
    eps_rel: float = 2e-3      # identifies the active set and solves the reduced KKT exactly)
    eps_retry: float = 1e-7    # problems whose polish is rejected resume ADMM to this eps
    rho_min: float = 1e-6
    rho_max: float = 1e6
    adapt_tol: float = 5.0
    eq_scale: float = 1e3
    delta: float = 1e-9        # polish regularisation, relative to the problem scale
    dual_tol: float = 1e-9     # multiplier sign tolerance, relative to the problem scale
    max_iter: int = 4000
    adapt_interval: int = 60
    polish: int = 1
    polish_rounds: int = 8
    refine_iters: int = 1      # proximal refinement steps per polish round (then KKT-checked)
    # problems whose polish is rejected are polished again with this many refinement steps
    # (nearly singular P_FF, e.g. small risk aversions) before the ADMM retry (host-side)
    refine_retry: int = 4
    # window path: initial rho >= rho0_qrel * max|q| (host-side, not in pq_settings): for
    # nearly linear objectives (small risk aversion) 4 mean(diag P) is far too small a rho
    rho0_qrel: float = 10.0
    # wide rounds of the grouped polish (polish_gw.hip, host-side): refinement steps per round
    # (early exit at the 1e-13 residual) and the group capacitance's diagonal relative to the
    # problem scale (the reduced KKT system keeps delta).  Measured on config 4
    # (profiles/r03c_config4_grid.log, steps 2/4/6/10 x 1e-9/1e-7): at 1e-9 the explicit M_U^-1
    # (condition ~1e11) limits each step to ~1e-5, so 2 steps leave 2e-7 stationarity and 1.8
    # rounds; 1e-7 converges in <= 4 steps to 5e-13 (87k QPs/s, polish 40 ms, 1.0 rounds)
    refine_wide: int = 6
    delta_wide: float = 1e-7
    # centred windows (mean-variance family) on the group capacitance with the grouped polish
    # (host-side): the ADMM stops at this looser eps -- it only has to predict the active
    # set, the pipeline's rounds are cheap and every answer is certified -- and the dates the
    # pipeline hands to the per-date polish resume ADMM to eps_abs / eps_rel first (their
    # rounds are not cheap).  Measured (profiles/r03s_*, r03t_*, r03u_*): config 3 2e-3 /
    # 1e-2 / 2e-2 / 1e-1 -> 311k / 335k / 343k / 353k QPs/s (20 / 16 / 15 / 11 iterations,
    # 2.7 / 3.1 / 3.2 / 3.8 rounds); with the sparse exact-P x pass (r03y_*) 2e-2 / 3e-2 /
    # 5e-2 / 1e-1 -> 347k / 357k / 358k / 360k at 5 / 5 / 6 / 6 rounds at most (of the 8
    # allowed): 3e-2 keeps the round count of 2e-2; with polish_fix_rel = 0.05 (r03Q_grid*):
    # 3e-2 / 5e-2 -> 374k / 389k at 2.86 / 2.99 rounds, at most 5 / 5.  Round 4, with the
    # inner primal steps (polish_inner) the rounds stay cheap from a looser point
    # (profiles/r04t_eg*.log, one box, polish_inner = 1): 0.2 / 0.3 -> 461k / 466k (9 / 8
    # iterations, 2.2 / 2.3 rounds, at most 4, largest free set 88); 0.5 and 1.0 stop after 4
    # iterations -- ADMM's residuals are not monotone: they dip below 0.5 at iteration 4 and
    # stay above 0.3 until 8 -- where the free sets outgrow the LDS solve and every date takes
    # the per-date fallback (144k).  The loose stop therefore also waits for min_iter_grouped
    # iterations: 0.3 with at least 8 -> 536k (r04O_eg25*.log: 0.25, the same 8 iterations),
    # and a larger eps cannot fall off that cliff.  Tracking (uncentred) windows keep eps_abs: their free
    # sets mostly exceed the LDS solve -- config 2 53.0k at 2e-3, 45.0k at 1e-2 from the loose
    # point, 50.1k with the resume; config 4 87.9k / 91.8k / 87.6k.  0 or <= eps_abs: off.
    # Round 6, with the register-tile polish solve (profiles/r06p_*, r06q_*): (0.3, floor 8) ->
    # 676-680k QPs/s (ADMM 2.90, polish 2.52-2.61 ms); (0.5 or 1.0, floor 7) -> 694-699k (7
    # iterations: ADMM 2.56, polish 2.75 ms, 2.27 rounds, at most 4); floor 6 or 5 -> 525-560k
    # (polish 5.0-5.3 ms: free sets beyond the register solve and up to 5 rounds).  So the loose
    # stop is in effect a 7-iteration warm start of the polish for the centred windows
    eps_grouped: float = 0.5
    # (host-side) the loose stop's pq_settings.min_iter.  Round 5 (profiles/r05T_config3_miniter_grid.log):
    # 6 / 7 / 8 / 9 -> the same 8 iterations below 9 (eps 0.3 is first met at 8), 9 slower (569k);
    # round 6: 7 with eps 0.5 (above)
    min_iter_grouped: int = 7
    # (host-side) the same loose stop for uncentred (tracking) windows on the group capacitance;
    # 0: off (they stop at eps_abs / eps_rel).  Measured on config 2 (profiles/r04T_*.log): off /
    # 1e-2 / 3e-2 / 1e-1 -> 161k / 151k / 142k / 114k QPs/s (20 / 17 / 15 / 13 iterations, 2.7 /
    # 3.1 / 3.5 / 4.0 rounds): the tracking rounds (free sets of 160..220) cost more than the
    # ADMM iterations they replace
    eps_grouped_tracking: float = 0.0
    # (host-side) small batches of tracking windows (at most small_batch dates, e.g. the
    # reference notebook's 13-date monthly run) take the loose stop at this eps when it is > 0
    # and eps_grouped_tracking is 0.  Off by default: the first grid on the 13-date monthly run
    # (profiles/r05N_monthly_grid.log: off / 3e-3 / 1e-2 / 3e-2 / 0.1 / 0.3 -> 10.3 / 10.4 / 9.5 /
    # 9.6 / 10.0 / 9.5 ms) did not hold up when re-measured as medians of five
    # (profiles/r05V_monthly_grid.log: 1e-2 9.84 ms, off 9.78 ms).  The rule keys on the batch
    # of one solve call, so in a chunked backtest only a short last chunk would take it
    eps_grouped_tracking_small: float = 0.0
    small_batch: int = 64
    # (host-side) tracking windows with more than 4 general rows (the column-sparse wide form,
    # e.g. config 4's sector caps) take the loose stop at this eps when eps_grouped_tracking is
    # 0: their polish finishes in about one wide round, so ADMM iterations are the cost.
    # Measured on config 4 (profiles/r05Q_grid.log): off / 3e-3 / 1e-2 / 3e-2 -> 119-123k /
    # 124k / 129k / 113k QPs/s (20 / 19 / 17 / 15 iterations; 3e-2 hands dates to the per-date
    # polish); around it (profiles/r05U_config4_eps_wide_grid.log) 1e-2 / 1.5e-2 / 2e-2 ->
    # 130-131k / 122-124k / 128-131k (1.00 / 1.12 / 1.05 rounds: 1e-2 the steadiest); config 2
    # (one general row) keeps eps_abs (round 4: 161k off, 151k at 1e-2;
    # round 5, profiles/r05S_config2_loose_grid.log: off / 3e-3 / 1e-2 -> 227k / 226-230k /
    # 214-217k: its rounds of free sets of ~190 still cost more than the iterations saved)
    eps_grouped_tracking_wide: float = 1e-2
    # (host-side) the loose stop also on the per-problem capacitance (grouped ADMM without the
    # group capacitance: the lambda sweep, whose problems of a date differ in P's scale)
    eps_grouped_percap: bool = False
    min_iter: int = 0           # pq_settings.min_iter: no convergence test before this iteration
    # grouped polish: variables with x - lb < polish_fix_rel * max(x - lb) at the ADMM point
    # also start fixed at lb (besides OSQP's z - lb < -y): the loose ADMM point leaves small
    # positive weights that the first rounds would only fix later.  Numpy model of config 3
    # (tests/engine_model.py, eps 3e-2, 10 dates): 0 / 0.05 / 0.1 / 0.2 -> 3.0 / 2.6 / 2.3 /
    # 3.3 rounds, first free sets 79 / 71 / 62 / 47 (wrong fixes cost the rounds back); on
    # the GPU (profiles/r03N_*): 0 / 0.05 / 0.1 -> 363k / 378k / 372k QPs/s, 3.31 / 2.86 / 3.0
    # rounds on average, at most 5 / 5 / 6.  Round 4 at eps_grouped 0.2 / 0.3 with one inner
    # step: 0.05 / 0.1 -> 461k / 467k and 466k / 479k (profiles/r04t_eg*_in1{,_fr1}.log).
    # Centred windows only (k_pg_init)
    polish_fix_rel: float = 0.1
    # grouped polish, LDS solve (k_pg_solve): free variables outside their box are fixed at
    # it and the reduced system re-solved inside the round, up to this many times per round,
    # instead of one whole round (window passes, checks, setup) per such step.  Measured at
    # eps_grouped 0.3 (profiles/r04t_eg3_in{1,2}.log): 1 / 2 -> 466k / 457k QPs/s (2.29 / 2.11
    # rounds; the second step costs more in the solve buckets than the rounds it saves)
    polish_inner: int = 1
    # grouped polish: a rejected round also releases the variables at a bound whose multiplier
    # is within this fraction of the problem scale of the wrong sign (0: off; see pq_settings)
    polish_release_rel: float = 0.0

    def to_c(self) -> _lib.PQSettings:
        names = {f[0] for f in _lib.PQSettings._fields_}
        return _lib.PQSettings(**{f.name: getattr(self, f.name) for f in dataclasses.fields(self)
                                  if f.name in names})

    @classmethod
    def from_params(cls, params) -> "Settings":
        s = cls()
        if params:
            for f in dataclasses.fields(cls):
                for key in (f.name, "admm_" + f.name):
                    if key in params and params[key] is not None:
                        v, typ = params[key], type(getattr(s, f.name))
                        if typ is bool and isinstance(v, str):   # "0" / "false" from --set KEY=VALUE
                            v = v.strip().lower() not in ("0", "false", "no", "off", "")
                        setattr(s, f.name, typ(v))
        return s


# ----------------------------------------------------------------------------------------
# Problem batches
# ----------------------------------------------------------------------------------------


class QPBatch:
    """A batch of dense QPs  min 0.5 x'(ps P + pd I)x + q'x  s.t. lg <= Cg x <= ug,
    lb <= x <= ub, laid out as include/porqua_hip.h expects (ld = round_up(n, 64))."""

    def __init__(self, n: int, batch: int, mg: int, device=None, shared_constraints=True,
                 has_box=True, P=None):
        self.device = device or default_device()
        self.n, self.batch, self.mg = int(n), int(batch), int(mg)
        self.ld = round_up(max(n, 1), 64)
        self.mg_pad = round_up(max(mg, 1), 8)
        ld, dev = self.ld, self.device
        self.P = P if P is not None else torch.zeros((batch, ld, ld), dtype=F64, device=dev)
        self.q = torch.zeros((batch, ld), dtype=F64, device=dev)
        self.p_scale = None
        self.p_diag = None
        nc = 1 if shared_constraints else batch
        self.shared = shared_constraints
        self.Cg = torch.zeros((nc, max(mg, 1), ld), dtype=F64, device=dev)
        self.lg = torch.full((nc, max(mg, 1)), -np.inf, dtype=F64, device=dev)
        self.ug = torch.full((nc, max(mg, 1)), np.inf, dtype=F64, device=dev)
        self.has_box = has_box
        if has_box:
            self.lb = torch.full((nc, ld), -np.inf, dtype=F64, device=dev)
            self.ub = torch.full((nc, ld), np.inf, dtype=F64, device=dev)
        else:
            self.lb = self.ub = None

    def c_struct(self) -> _lib.PQProblem:
        ld = self.ld
        cs = 0 if self.shared else self.Cg.stride(0)
        gs = 0 if self.shared else self.lg.stride(0)
        bs = 0 if (self.shared or not self.has_box) else self.lb.stride(0)
        return _lib.PQProblem(
            n=self.n, ld=ld, batch=self.batch, mg=self.mg,
            P=None if self.P is None else self.P.data_ptr(),
            P_stride=0 if self.P is None else self.P.stride(0),
            p_scale=None if self.p_scale is None else self.p_scale.data_ptr(),
            p_diag=None if self.p_diag is None else self.p_diag.data_ptr(),
            q=self.q.data_ptr(), q_stride=self.q.stride(0),
            Cg=self.Cg.data_ptr(), Cg_stride=cs,
            lg=self.lg.data_ptr(), ug=self.ug.data_ptr(), g_stride=gs,
            lb=None if self.lb is None else self.lb.data_ptr(),
            ub=None if self.ub is None else self.ub.data_ptr(), box_stride=bs)

    @classmethod
    def from_dense(cls, P, q, A=None, b=None, G=None, h=None, lb=None, ub=None, device=None, n=None):
        """Build from host arrays: P (B,n,n), q (B,n); A (me,n)|(B,me,n), b; G, h; lb, ub
        ((n,) shared or (B,n)).  Equality rows are stored first (lg == ug).  P = None (with
        ``n``): constraints only -- one problem, P left None and q zero, for callers that set
        the objective on the device afterwards (no n x n host array or upload)."""
        if P is None:
            B, n = 1, int(n)
        else:
            P = np.asarray(P, dtype=np.float64)
            if P.ndim == 2:
                P = P[None]
            B, n, _ = P.shape
            q = np.asarray(q, dtype=np.float64).reshape(B, n)

        def per(M, rows):
            if M is None:
                return None
            M = np.asarray(M, dtype=np.float64)
            if M.ndim == 1 and rows is not None:
                M = M.reshape(rows)
            return M

        A = None if A is None else np.asarray(A, dtype=np.float64)
        G = None if G is None else np.asarray(G, dtype=np.float64)
        if A is not None and A.ndim == 1:
            A = A.reshape(1, n)
        if G is not None and G.ndim == 1:
            G = G.reshape(1, n)
        me = 0 if A is None else A.shape[-2]
        mi = 0 if G is None else G.shape[-2]
        shared = (A is None or A.ndim == 2) and (G is None or G.ndim == 2)
        b_ = None if b is None else np.asarray(b, dtype=np.float64)
        h_ = None if h is None else np.asarray(h, dtype=np.float64)
        if shared and b_ is not None and b_.size != me:
            shared = False
        if shared and h_ is not None and h_.size != mi:
            shared = False
        lb_ = None if lb is None else np.asarray(lb, dtype=np.float64)
        ub_ = None if ub is None else np.asarray(ub, dtype=np.float64)
        if shared and ((lb_ is not None and lb_.ndim == 2) or (ub_ is not None and ub_.ndim == 2)):
            shared = False
        has_box = lb_ is not None or ub_ is not None
        self = cls(n, B, me + mi, device=device, shared_constraints=shared, has_box=has_box,
                   P=None if P is not None else torch.empty(0, dtype=F64))
        nc = 1 if shared else B
        ld = self.ld
        Cg = np.zeros((nc, max(me + mi, 1), ld))
        lg = np.full((nc, max(me + mi, 1)), -np.inf)
        ug = np.full((nc, max(me + mi, 1)), np.inf)
        if me:
            Ab = np.broadcast_to(A, (nc, me, n)) if A.ndim == 2 else A
            bb = np.broadcast_to(b_.reshape(-1, me) if b_ is not None else 0.0, (nc, me))
            Cg[:, :me, :n] = Ab
            lg[:, :me] = bb
            ug[:, :me] = bb
        if mi:
            Gb = np.broadcast_to(G, (nc, mi, n)) if G.ndim == 2 else G
            hb = np.broadcast_to(h_.reshape(-1, mi), (nc, mi))
            Cg[:, me:me + mi, :n] = Gb
            ug[:, me:me + mi] = hb
        dev = self.device
        if P is None:
            self.P = None
        else:
            Pp = np.zeros((B, ld, ld))
            Pp[:, :n, :n] = P
            self.P = torch.from_numpy(Pp).to(dev)
            qp = np.zeros((B, ld))
            qp[:, :n] = q
            self.q = torch.from_numpy(qp).to(dev)
        self.Cg = torch.from_numpy(Cg).to(dev)
        self.lg = torch.from_numpy(lg).to(dev)
        self.ug = torch.from_numpy(ug).to(dev)
        if has_box:
            lo = np.full((nc, ld), -np.inf)
            up = np.full((nc, ld), np.inf)
            lo[:, n:] = 0.0
            up[:, n:] = 0.0
            if lb_ is not None:
                lo[:, :n] = np.broadcast_to(lb_, (nc, n)) if lb_.ndim == 1 else lb_
            if ub_ is not None:
                up[:, :n] = np.broadcast_to(ub_, (nc, n)) if ub_.ndim == 1 else ub_
            self.lb = torch.from_numpy(lo).to(dev)
            self.ub = torch.from_numpy(up).to(dev)
        self.me, self.mi = me, mi
        return self


LR_POLISH_LDK = 256      # first compact polish scratch of the window path (free set <= 256)


class Workspace:
    """Solver state for a QPBatch (all device memory; nothing persistent in the library).

    ``dense`` (K2/K3/K4 on P itself): K / Dt are the n x n KKT inverse and polish scratch.
    Otherwise (the window path) they are only the compact ldk x ldk polish scratch of
    pq_polish_w_batched, ldk = ``kcap`` (default min(ld, LR_POLISH_LDK))."""

    def __init__(self, qb: QPBatch, dense: bool = True, kcap: int | None = None):
        B, ld, dev = qb.batch, qb.ld, qb.device
        self.B, self.device = B, dev
        self.mg_pad = qb.mg_pad
        self.m_ld = qb.mg_pad + ld
        self.ldk = ld if dense else min(ld, 1024, round_up(kcap or LR_POLISH_LDK, 64))
        kd = self.ldk
        self.K = torch.empty((B, kd, kd), dtype=F64, device=dev)
        self.Dt = torch.empty((B, kd // 64, 64, 64), dtype=F64, device=dev)
        self._lr = None
        self.x = torch.zeros((B, ld), dtype=F64, device=dev)
        self.Px = torch.zeros((B, ld), dtype=F64, device=dev)
        self.z = torch.zeros((B, self.m_ld), dtype=F64, device=dev)
        self.y = torch.zeros((B, self.m_ld), dtype=F64, device=dev)
        self.rho = torch.zeros(B, dtype=F64, device=dev)
        self.iters = torch.zeros(B, dtype=torch.int32, device=dev)
        self.status = torch.zeros(B, dtype=torch.int32, device=dev)
        self.info = torch.zeros(B, dtype=torch.int32, device=dev)
        self.out = torch.zeros((B, _lib.PQ_OUT_FIELDS), dtype=F64, device=dev)
        self.work_stride = _lib.work_doubles(ld, qb.mg_pad)
        self.work = torch.zeros((B, self.work_stride), dtype=F64, device=dev)

    def pg_record(self):
        """Per-problem record of the grouped polish pipeline (PQ_PG_RECORD doubles each)."""
        if getattr(self, "_pg_rec", None) is None:
            self._pg_rec = torch.zeros((self.B, _lib.PQ_PG_RECORD), dtype=F64, device=self.device)
        return self._pg_rec

    def lr_buffers(self, k_ld: int):
        """Capacitance matrices M, their inverses and factor scratch (low-rank path)."""
        if self._lr is None or self._lr["k_ld"] != k_ld:
            B, dev = self.B, self.device
            self._lr = {"k_ld": k_ld,
                        "M": torch.empty((B, k_ld, k_ld), dtype=F64, device=dev),
                        "Minv": torch.empty((B, k_ld, k_ld), dtype=F64, device=dev),
                        "Dt": torch.empty((B, k_ld // 64, 64, 64), dtype=F64, device=dev),
                        "iters": torch.zeros(B, dtype=torch.int32, device=dev),
                        "status": torch.zeros(B, dtype=torch.int32, device=dev),
                        "info": torch.zeros(B, dtype=torch.int32, device=dev)}
        return self._lr

    def c_struct(self) -> _lib.PQState:
        return _lib.PQState(
            K=self.K.data_ptr(), K_stride=self.K.stride(0),
            Dt=self.Dt.data_ptr(), Dt_stride=self.Dt.stride(0),
            x=self.x.data_ptr(), Px=self.Px.data_ptr(),
            z=self.z.data_ptr(), y=self.y.data_ptr(),
            m_ld=self.m_ld, mg_pad=self.mg_pad,
            rho=self.rho.data_ptr(),
            iters=self.iters.data_ptr(), status=self.status.data_ptr(), info=self.info.data_ptr(),
            out=self.out.data_ptr(),
            work=self.work.data_ptr(), work_stride=self.work_stride)


@dataclass
class BatchResult:
    x: torch.Tensor          # (B, n) weights (device)
    y: torch.Tensor          # (B, mg) multipliers of the general rows (equalities first)
    z_box: torch.Tensor      # (B, n)
    status: torch.Tensor     # (B,) int32
    iters: torch.Tensor      # (B,) int32
    out: torch.Tensor        # (B, PQ_OUT_FIELDS)
    refactors: int = 0
    admm_launches: int = 0
    polish_fallbacks: int = 0   # dates the grouped polish handed to the per-date kernel
    capacitance: str = ""    # window path: "band" (pq_lr_capacitance_band), "group", "eig" or "direct"

    @property
    def obj(self):
        return self.out[:, _lib.PQ_OUT_OBJ]

    @property
    def found(self):
        return (self.status == _lib.PQ_SOLVED) | (self.status == _lib.PQ_SOLVED_INACCURATE)


class StageGraphs:
    """HIP graphs of the stages of a solve that is repeated on the same buffers (a backtest
    re-solved every step, the bench workloads): the first time a stage runs its launches are
    captured into a graph (torch.cuda.CUDAGraph over the caller's stream: the library's
    kernels, the side-stream forks / joins of the polish and the torch glue), every later
    time the graph is replayed -- one launch per stage instead of dozens, no host work
    between them.  Stages are keyed by name and occurrence within one solve (``begin``).

    Only sync-free stages may be captured (solve_lowrank(sync_free=True) is); kernel
    arguments -- device pointers and settings -- are frozen at capture, so the owner must
    keep the same problem, window and workspace objects alive and in place."""

    def __init__(self):
        self.graphs = {}
        self.pool = None
        self._seen = {}
        self._warm = set()
        self.replays = 0   # replays of a graph captured by an earlier step (tests, diagnostics)

    def begin(self):
        self._seen = {}

    def run(self, name, fn):
        """First call of a stage: eager (it fills the host-side caches -- plans, uniformity
        checks -- whose first evaluation synchronises); second: capture + replay; then replay."""
        k = self._seen.get(name, 0)
        self._seen[name] = k + 1
        key = (name, k)
        hit = self.graphs.get(key)
        if hit is not None:
            self.replays += 1
        if hit is None:
            if key not in self._warm:
                self._warm.add(key)
                return fn()
            # captured on the caller's (non-default) stream itself: the solve passes that
            # stream to the library explicitly, so it must be the capturing one
            cur = torch.cuda.current_stream()
            if cur == torch.cuda.default_stream(cur.device):
                raise RuntimeError("StageGraphs: run the solve on a non-default stream (torch.cuda.stream(...))")
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, pool=self.pool, stream=cur):
                r = fn()
            self.pool = g.pool()
            hit = self.graphs[key] = (g, r)
        hit[0].replay()
        return hit[1]


class _Timeline:
    """Optional per-launch HIP event pairs on the launch stream (no host syncs); with
    ``graphs`` (StageGraphs) each stage is captured once and replayed afterwards (the events
    then bracket the graph launch)."""

    def __init__(self, sink, graphs: "StageGraphs | None" = None):
        self.sink = sink
        self.graphs = graphs

    def __call__(self, name, fn):
        run = (lambda: self.graphs.run(name, fn)) if self.graphs is not None else fn
        if self.sink is None:
            return run()
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        r = run()
        e1.record()
        self.sink.append((name, e0, e1))
        return r


def solve(qb: QPBatch, settings: Settings | None = None, ws: Workspace | None = None,
          max_rounds: int = 64, events: list | None = None) -> BatchResult:
    """Solve every QP of the batch on the current device/stream (K2 -> K3 [-> K2 -> K3 ...] -> K4).

    ``events``: if a list is given, (kernel name, start, end) torch.cuda.Event triples are
    appended for every launch (recorded on the launch stream)."""
    tl = _Timeline(events)
    lib = _lib.load()
    s = (settings or Settings()).to_c()
    ws = ws or Workspace(qb)
    pb = qb.c_struct()
    st = ws.c_struct()
    strm = _stream()
    P_, S_, SS = ctypes.byref(pb), ctypes.byref(st), ctypes.byref(s)
    _lib.check(lib.pq_init_state(P_, S_, None, 0, SS, strm), "pq_init_state")
    _rho_floor_q(qb, ws, settings or Settings())
    _lib.check(tl("factor", lambda: lib.pq_factor_batched(P_, S_, None, 0, SS, 1, strm)),
               "pq_factor_batched")
    cnt = {"refactors": 0, "launches": 0}

    def admm_rounds(idx, nidx, SSx):
        for _ in range(max_rounds):
            _lib.check(tl("admm", lambda: lib.pq_admm_batched(P_, S_, _ptr(idx), nidx, SSx,
                                                              int(s.max_iter), strm)),
                       "pq_admm_batched")
            cnt["launches"] += 1
            need = torch.nonzero(ws.status == _lib.PQ_NEED_REFACTOR).flatten().to(torch.int32)
            k = int(need.numel())   # host sync: small status vector
            if k == 0:
                break
            idx, nidx = need.contiguous(), k
            _lib.check(tl("factor", lambda: lib.pq_factor_batched(P_, S_, _ptr(idx), nidx, SSx, 1, strm)),
                       "pq_factor_batched")
            cnt["refactors"] += k

    admm_rounds(None, 0, SS)
    if s.polish:
        _lib.check(tl("polish", lambda: lib.pq_polish_batched(P_, S_, None, 0, SS, strm)),
                   "pq_polish_batched")
        rp = _repolish_set(ws, settings or Settings())
        if rp is not None:      # polish rejected: polish again with more refinement steps
            pidx, pn, s3 = rp
            _lib.check(tl("polish", lambda: lib.pq_polish_batched(P_, S_, _ptr(pidx), pn, ctypes.byref(s3), strm)),
                       "pq_polish_batched (refine)")
        retry = _retry_set(ws, settings or Settings())
        if retry is not None:   # polish rejected: resume ADMM to eps_retry, polish again
            idx, nidx, s2 = retry
            # the polish used K as scratch: restore K^-1 (current rho) before resuming
            _lib.check(tl("factor", lambda: lib.pq_factor_batched(P_, S_, _ptr(idx), nidx, SS, 1, strm)),
                       "pq_factor_batched (retry)")
            admm_rounds(idx, nidx, ctypes.byref(s2))
            _lib.check(tl("polish", lambda: lib.pq_polish_batched(P_, S_, _ptr(idx), nidx, SS, strm)),
                       "pq_polish_batched (retry)")
    refactors, launches = cnt["refactors"], cnt["launches"]
    n, mg = qb.n, qb.mg
    return BatchResult(x=ws.x[:, :n], y=ws.y[:, :mg], z_box=ws.y[:, ws.mg_pad:ws.mg_pad + n],
                       status=ws.status, iters=ws.iters, out=ws.out, refactors=refactors,
                       admm_launches=launches)


def _rho_floor_q(qb: "QPBatch", ws: "Workspace", settings: Settings):
    """Initial rho >= rho0_qrel * max|q| per problem (both paths, before the first factor)."""
    if settings.rho0_qrel > 0:
        qinf = qb.q[:, :qb.n].abs().amax(1)
        torch.clamp(torch.maximum(ws.rho, settings.rho0_qrel * qinf), settings.rho_min, settings.rho_max,
                    out=ws.rho)


def _repolish_set(ws: "Workspace", settings: Settings):
    """Problems whose polish was rejected: set them back to SOLVED (their ADMM point is
    untouched by a rejected polish) and return (idx, n, settings with refine_iters =
    refine_retry) for a second polish, or None (host sync: status)."""
    if settings.refine_retry <= settings.refine_iters:
        return None
    bad = torch.nonzero(ws.status == _lib.PQ_SOLVED_INACCURATE).flatten().to(torch.int32)
    m = int(bad.numel())
    if m == 0:
        return None
    ws.status[bad.long()] = _lib.PQ_SOLVED
    s3 = settings.to_c()
    s3.refine_iters = settings.refine_retry
    return bad.contiguous(), m, s3


def _retry_set(ws: "Workspace", settings: Settings):
    """Problems whose polish was rejected at the loose ADMM eps: reset them to UNSOLVED
    and return (idx, n, settings with eps = eps_retry), or None (host sync: status)."""
    bad = torch.nonzero(ws.status == _lib.PQ_SOLVED_INACCURATE).flatten().to(torch.int32)
    m = int(bad.numel())
    if m == 0 or settings.eps_retry <= 0 or settings.eps_retry >= min(settings.eps_abs, settings.eps_rel):
        return None
    ws.status[bad.long()] = _lib.PQ_UNSOLVED
    s2 = settings.to_c()
    s2.eps_abs = s2.eps_rel = settings.eps_retry
    return bad.contiguous(), m, s2


class LowRank:
    """Device description of P_eff = p_scale w_scale Xc'Xc + p_diag I through the date
    windows (pq_lowrank): nothing n x n is formed.  ``mu`` None = uncentred Gram
    (LeastSquares).  ``dg`` = diag(Xc'Xc) per date (pq_window_sumsq; computed here when
    not given -- call refresh() after the window means change in place)."""

    def __init__(self, panel, rows, tlen, mu=None, w_scale=None, dg=None):
        self.panel, self.rows, self.tlen, self.mu, self.w_scale = panel, rows, tlen, mu, w_scale
        self.tmax = int(rows.shape[1])
        self.dg = dg if dg is not None else panel.window_sumsq(rows, tlen, mu)

    def refresh(self):
        self.panel.window_sumsq(self.rows, self.tlen, self.mu, out=self.dg)
        return self

    def span(self):
        """(r0, nrows, W): the panel rows the windows touch and the widest window span."""
        if getattr(self, "_span", None) is None:
            t = self.tlen.to(torch.int64)
            first = self.rows[:, 0].to(torch.int64)
            last = self.rows.gather(1, (t - 1).clamp(min=0)[:, None]).flatten().to(torch.int64)
            v = torch.stack([first.min(), last.max(), (last - first + 1).max()]).cpu().tolist()
            self._span = (int(v[0]), int(v[1] - v[0] + 1), int(v[2]))
        return self._span

    def c_struct(self) -> _lib.PQLowRank:
        return _lib.PQLowRank(panel=self.panel.R.data_ptr(), ldp=self.panel.R.stride(0),
                              rows=self.rows.data_ptr(), tlen=self.tlen.data_ptr(), tmax=self.tmax,
                              mu=None if self.mu is None else self.mu.data_ptr(),
                              mu_stride=0 if self.mu is None else self.mu.stride(0),
                              w_scale=None if self.w_scale is None else self.w_scale.data_ptr(),
                              dg=self.dg.data_ptr(), dg_stride=self.dg.stride(0))


class EigCap:
    """One symmetric eigendecomposition per DATE of the centred window Gram Xc Xc' (T x T),
    shared by every problem of that date (pq_eigcap_form): the risk aversions of the sweep
    (P = 2 lam Sigma_d, src/optimization.py:168-174) differ only in the scale of P and in
    rho, and each capacitance inverse M_b^-1 is formed from the date's eigenvectors for the
    problem's own scale and rho -- no per-problem factorisation, and an adaptive-rho change
    is a re-form.  The Gram and the border W = Xc Cg' come from the hand-written window Gram
    kernel (pq_lr_capacitance with D = I, unit row weights); the eigendecomposition itself
    is rocSOLVER's (torch.linalg.eigh, ``backend`` 'rocsolver', the default) or the hand-written
    block-Jacobi solver (jacobi.hip, helper_functions.sym_eig, 'jacobi'), once per date.
    Measured for the 64 window Grams of config 5 (profiles/r03k_exp_eigh.log): syevd 10.4 ms,
    the block-Jacobi kernels 64.5 ms (eigenvalues to 1.2e-12) -- the Jacobi form serves the
    nearestPD repair, whose matrices need no ordering and few sweeps.

    rows / tlen / mu: per-date device tensors (every tlen == tmax); pdate: date of each
    problem (int32, device); Cg: the shared general rows (qb.Cg, mg <= 4)."""

    MG = 4

    def __init__(self, panel, rows, tlen, mu, qb: "QPBatch", pdate, k_ld: int, backend: str = "rocsolver"):
        lib = _lib.load()
        nd, tmax = int(rows.shape[0]), int(rows.shape[1])
        mg, n, dev = qb.mg, qb.n, qb.device
        if mg > self.MG or not qb.shared:
            raise _lib.PorquaHipError("EigCap: shared general rows, at most 4")
        if not bool((tlen == tmax).all().item()):
            raise _lib.PorquaHipError("EigCap: every window must have tmax rows")
        self.k_ld, self.nd, self.tmax = int(k_ld), nd, tmax
        self.pdate = pdate.to(torch.int32).contiguous()
        lgf = torch.full((max(mg, 1),), -np.inf, dtype=F64, device=dev)
        ugf = torch.full((max(mg, 1),), np.inf, dtype=F64, device=dev)
        one = torch.ones(nd, dtype=F64, device=dev)
        pb = _lib.PQProblem(n=n, ld=qb.ld, batch=nd, mg=mg, P=None, P_stride=0, p_scale=None, p_diag=None,
                            q=qb.q.data_ptr(), q_stride=0, Cg=qb.Cg.data_ptr(), Cg_stride=0,
                            lg=lgf.data_ptr(), ug=ugf.data_ptr(), g_stride=0, lb=None, ub=None, box_stride=0)
        lr = _lib.PQLowRank(panel=panel.R.data_ptr(), ldp=panel.R.stride(0), rows=rows.data_ptr(),
                            tlen=tlen.data_ptr(), tmax=tmax, mu=mu.data_ptr(), mu_stride=mu.stride(0),
                            w_scale=None, dg=None, dg_stride=0)
        st = _lib.PQState(rho=one.data_ptr())
        s = Settings(sigma=1.0, rho_min=1.0).to_c()   # D = I, unit weight on the Cg rows: M = I + U U'
        M = torch.zeros((nd, k_ld, k_ld), dtype=F64, device=dev)
        _lib.check(lib.pq_lr_capacitance(ctypes.byref(lr), ctypes.byref(pb), ctypes.byref(st), None, 0,
                                         ctypes.byref(s), M.data_ptr(), k_ld, k_ld * k_ld, _stream()),
                   "pq_lr_capacitance (window Gram)")
        T = tmax
        Mt = M[:, :T, :T]
        G = torch.tril(Mt) + torch.tril(Mt, -1).mT - torch.eye(T, dtype=F64, device=dev)
        if backend == "jacobi":   # zero padding to a multiple of 64: its pairs never rotate
            from .helper_functions import sym_eig
            ldj = round_up(T, 64)
            Gp = torch.zeros((nd, ldj, ldj), dtype=F64, device=dev)
            Gp[:, :T, :T] = G
            evj, Vj = sym_eig(Gp, T)
            ev, V = evj[:, :T], Vj[:, :T, :T]
        elif backend == "rocsolver":
            ev, V = torch.linalg.eigh(G)
        else:
            raise ValueError("EigCap: backend must be 'jacobi' or 'rocsolver'")
        self.V = torch.zeros((nd, k_ld, k_ld), dtype=F64, device=dev)
        self.V[:, :T, :T] = V
        self.evals = torch.zeros((nd, k_ld), dtype=F64, device=dev)
        self.evals[:, :T] = ev
        self.What = torch.zeros((nd, k_ld, self.MG), dtype=F64, device=dev)
        if mg:
            W = M[:, T:T + mg, :T].mT                      # Xc Cg' (rows T.. of the lower triangle)
            self.What[:, :T, :mg] = V.mT @ W
            C = qb.Cg[0, :mg, :n]
            self.cc = (C @ C.T).contiguous()
        else:
            self.cc = torch.zeros((1, 1), dtype=F64, device=dev)
        self.scratch = torch.empty((qb.batch, 2 * self.MG * k_ld), dtype=F64, device=dev)

    def form(self, lrs, pbs, sts, ss, Minv, idx, nidx, strm):
        """M_b^-1 of problems idx[0..nidx) (None: all) into Minv (B, k_ld, k_ld)."""
        lib = _lib.load()
        k = self.k_ld
        _lib.check(lib.pq_eigcap_form(lrs, pbs, sts, ss, self.pdate.data_ptr(), self.V.data_ptr(),
                                      self.evals.data_ptr(), self.What.data_ptr(), self.cc.data_ptr(), k,
                                      _ptr(idx), nidx, Minv.data_ptr(), k * k, self.scratch.data_ptr(), strm),
                   "pq_eigcap_form")


def lowrank_shape_ok(n: int, tmax: int, mg: int) -> bool:
    """The Woodbury path applies (and pays): T + mg < n, k <= 512, and the window-form polish
    can run (even panel stride n, tmax <= 1024) so nothing needs the dense upper triangle."""
    k_ld = round_up(tmax + mg, 64)
    return (k_ld <= 512 and (k_ld + 127) // 128 <= (n + 127) // 128 and tmax + mg < n
            and n % 2 == 0 and tmax <= 1024 and mg <= 64)


def lowrank_applicable(qb: QPBatch, lr: LowRank) -> bool:
    return lowrank_shape_ok(qb.n, lr.tmax, qb.mg) and lr.panel.R.stride(0) % 2 == 0


def grouped_applicable(qb: QPBatch, lr: LowRank, groups: "GroupPlan | None", ws: "Workspace") -> bool:
    k_ld = round_up(lr.tmax + qb.mg, 64)
    return (groups is not None and groups.ok and qb.n % 2 == 0 and lr.panel.R.stride(0) % 2 == 0
            and qb.mg <= 32 and k_ld <= 384 and ws.work_stride >= 3 * qb.ld)


def _sparse_columns(qb: QPBatch, nz_limit: int = 4):
    """Column-sparse form of shared general rows (more than 4 rows, at most ``nz_limit``
    nonzeros per column: the budget row plus 0/1 group memberships, Constraints.add_linear
    for sector caps) for pq_admm_lr_grouped: (row ids int32 [ld, nzmax] -1 padded, values,
    nzmax), or (None, None, 0) when the rows are few or dense."""
    if not qb.shared or qb.mg <= 4:
        return None, None, 0
    C = qb.Cg[0, :qb.mg, :]
    nzc = (C != 0).sum(0)
    nzmax = int(nzc.max().item())
    if nzmax == 0 or nzmax > nz_limit:
        return None, None, 0
    order = torch.argsort((C == 0).to(torch.int8), dim=0, stable=True)[:nzmax]   # nonzero rows first
    vals = torch.gather(C, 0, order)
    rows = torch.where(vals != 0, order, torch.full_like(order, -1)).to(torch.int32)
    return rows.T.contiguous(), vals.T.contiguous(), nzmax


def _tkey(*ts):
    """Cache key of tensors (None allowed): storage, shape and in-place version counter, so
    it changes when a tensor is replaced or modified in place."""
    return tuple(None if t is None else (t.data_ptr(), tuple(t.shape), t._version) for t in ts)


def _cached(owner, name: str, key, fn, keep=()):
    """fn() cached on ``owner`` under ``name`` while ``key`` is unchanged (host-side checks
    with device syncs and constant tables are then paid once per batch, not per solve).

    ``keep``: the objects whose identity the key encodes (``id()``s, tensor data pointers).
    The cache entry holds strong references to them, so while the entry lives no other
    object can reuse those ids or the caching allocator those addresses, and a key match
    means the same objects (in-place changes bump ``_version``, which the key includes)."""
    hit = getattr(owner, name, None)
    if hit is not None and hit[0] == key:
        return hit[1]
    val = fn()
    setattr(owner, name, (key, val, tuple(keep)))
    return val


def _uniform_box(qb: QPBatch) -> bool:
    """Every box row of every problem gets the same ADMM rho (pq_lr_capacitance_band)."""
    if qb.lb is None:
        return True
    n = qb.n

    def check():
        lo, up = qb.lb[:, :n], qb.ub[:, :n]
        cls = torch.where(torch.isinf(lo) & torch.isinf(up), 1, torch.where(lo == up, 2, 0))
        return bool((cls == cls[:, :1]).all().item()) and (qb.lb.shape[0] == 1 or
                                                          bool((cls[:, 0] == cls[0, 0]).all().item()))
    return _cached(qb, "_c_ubox", _tkey(qb.lb, qb.ub), check, keep=(qb.lb, qb.ub))


def _band_setup(qb: QPBatch, lr: LowRank, strm, w_min: int = 0):
    """Band Gram of the panel rows + PC / CC tables for pq_lr_capacitance_band, or None when
    the band form does not apply (per-problem constraints, non-uniform box rho, tmax > 1024).
    ``w_min``: band width at least this (the group capacitance needs the widest union span)."""
    if not qb.shared or lr.tmax > 1024 or not _uniform_box(qb):
        return None
    lib = _lib.load()
    r0, nrows, W = lr.span()
    W = min(max(W, int(w_min)), nrows)
    dev, n, mg = qb.device, qb.n, qb.mg
    ldo = round_up(W, 2)
    band, pc = _cached(lr, "_c_bandbuf", (nrows, ldo, mg),
                       lambda: (torch.empty((nrows, ldo), dtype=F64, device=dev),
                                torch.empty((nrows, max(mg, 1)), dtype=F64, device=dev)))
    R = lr.panel.R
    _lib.check(lib.pq_lr_band_gram(R.data_ptr(), R.stride(0), n, r0, nrows, W, band.data_ptr(), ldo,
                                   qb.Cg.data_ptr(), mg, qb.ld, pc.data_ptr(), pc.stride(0), strm),
               "pq_lr_band_gram")
    def cgram():
        C = qb.Cg[0, :mg, :n]
        return (C @ C.T).contiguous() if mg else torch.zeros((1, 1), dtype=F64, device=dev)
    cc = _cached(qb, "_c_cc", _tkey(qb.Cg), cgram, keep=(qb.Cg,))
    return {"band": band, "ldo": ldo, "r0": r0, "pc": pc, "cc": cc, "W": W, "nrows": nrows}


def _gcap_setup(qb: QPBatch, lr: "LowRank", ws: "Workspace", groups: "GroupPlan", settings: Settings):
    """Buffers and C structs of the group capacitance (admm_gcap.hip), or None when the dates
    of some group do not share c = p_scale w_scale and p_diag.  Also sets one rho per group
    (the mean of its dates' initial rho) in ws.rho."""
    B, dev, mg = qb.batch, qb.device, qb.mg

    def uniform():
        ps = qb.p_scale if qb.p_scale is not None else torch.ones(B, dtype=F64, device=dev)
        wsc = lr.w_scale if lr.w_scale is not None else torch.ones(B, dtype=F64, device=dev)
        c = ps * wsc
        pd = qb.p_diag if qb.p_diag is not None else torch.zeros(B, dtype=F64, device=dev)
        first = groups.gdates[:-1].long()[groups.gidx.long()]
        return bool(((c == c[first]) & (pd == pd[first])).all().item())
    if not _cached(ws, "_c_gcap_uniform", (id(groups),) + _tkey(qb.p_scale, lr.w_scale, qb.p_diag), uniform,
                   keep=(groups, qb.p_scale, lr.w_scale, qb.p_diag)):
        return None
    G = groups.ngroups
    k_ld = round_up(groups.ucnt_max + mg, 64)
    ldh = min(64, round_up(groups.corr_max, 8))
    key = (B, G, k_ld, ldh)
    buf = getattr(ws, "_gcap", None)
    if buf is None or buf["key"] != key:
        buf = {"key": key,
               "M": torch.empty((G, k_ld, k_ld), dtype=F64, device=dev),
               "Minv": torch.empty((G, k_ld, k_ld), dtype=F64, device=dev),
               "Dt": torch.empty((G, k_ld // 64, 64, 64), dtype=F64, device=dev),
               "grho": torch.empty(G, dtype=F64, device=dev),
               "iters": torch.zeros(G, dtype=torch.int32, device=dev),
               "status": torch.zeros(G, dtype=torch.int32, device=dev),
               "info": torch.zeros(G, dtype=torch.int32, device=dev),
               "aq": torch.empty((B, 2 * k_ld), dtype=F64, device=dev),
               "hinv": torch.empty((B, ldh, ldh), dtype=F64, device=dev)}
        ws._gcap = buf
    # one rho per group: the mean of the dates' initial rho (scale-aware, _rho_floor_q included)
    gidx, sizes = groups.device_index()
    gr = buf["grho"]
    gr.zero_().index_add_(0, gidx, ws.rho)
    gr /= sizes
    torch.index_select(gr, 0, gidx, out=ws.rho)
    kmax = groups.ucnt_max + mg
    buf["c"] = _lib.PQGcap(gdates=groups.gdates.data_ptr(), ngroups=G, urows=groups.urows.data_ptr(),
                           ucnt=groups.ucnt.data_ptr(), uoff=groups.uoff.data_ptr(), umax=groups.umax,
                           gidx=groups.gidx.data_ptr(), grho=buf["grho"].data_ptr(), M=buf["M"].data_ptr(),
                           Minv=buf["Minv"].data_ptr(), k_ld=k_ld, M_stride=k_ld * k_ld,
                           aq=buf["aq"].data_ptr(), aq_stride=2 * k_ld, hinv=buf["hinv"].data_ptr(), ldh=ldh,
                           gmax=int(groups.sizes.max()) if G else 0)
    # the factor sees each M_U as a k x k "problem" (identity padding beyond its U + mg rows)
    buf["pb"] = _lib.PQProblem(n=kmax, ld=k_ld, batch=G, mg=0, P=buf["M"].data_ptr(), P_stride=k_ld * k_ld,
                               q=qb.q.data_ptr(), q_stride=qb.q.stride(0), Cg=qb.Cg.data_ptr(),
                               lg=qb.lg.data_ptr(), ug=qb.ug.data_ptr())
    buf["st"] = _lib.PQState(K=buf["Minv"].data_ptr(), K_stride=k_ld * k_ld, Dt=buf["Dt"].data_ptr(),
                             Dt_stride=(k_ld // 64) * 4096, x=ws.x.data_ptr(), Px=ws.Px.data_ptr(),
                             z=ws.z.data_ptr(), y=ws.y.data_ptr(), m_ld=ws.m_ld, mg_pad=ws.mg_pad,
                             rho=buf["grho"].data_ptr(), iters=buf["iters"].data_ptr(),
                             status=buf["status"].data_ptr(), info=buf["info"].data_ptr(), out=ws.out.data_ptr(),
                             work=ws.work.data_ptr(), work_stride=ws.work_stride)
    return buf


def _pg_wide_setup(qb: QPBatch, lr: "LowRank", ws: "Workspace", groups: "GroupPlan", bd: dict, rec: torch.Tensor,
                   settings: Settings, sparse_cols, strm):
    """Group capacitance of the polish matrix K = P + d I for the wide rounds of the grouped
    polish (polish_gw.hip), d = p_diag + delta_g with delta_g the geometric mean of the
    group's dates' delta (settings.delta x problem scale, record field PQ_PG_SC): the same
    assemble / factor / prepare as the ADMM's group capacitance, with no general rows in the
    capacitance and a unit box whose rho is delta_g.  Returns the pq_pg_wide argument
    (its buffers kept alive on ws), or None when the wide form does not apply."""
    lib = _lib.load()
    B, dev, mg, G = qb.batch, qb.device, qb.mg, groups.ngroups
    nzr, nzv, nzmax = sparse_cols if mg > 4 else (None, None, 0)
    # uncentred windows only (LeastSquares tracking): with a mean column the correction H_b has
    # the entry 1 - (cT/d)(mu'mu - a'q/d), which cancels catastrophically at the polish's small d
    if (lr.mu is not None or bd is None or bd["W"] < groups.span_max or not qb.shared or mg > 24
            or (mg > 4 and nzmax == 0) or groups.ucnt_max + mg > 320 or groups.corr_max > 64):
        return None
    ps = qb.p_scale if qb.p_scale is not None else torch.ones(B, dtype=F64, device=dev)
    c = ps * (lr.w_scale if lr.w_scale is not None else torch.ones(B, dtype=F64, device=dev))
    pd = qb.p_diag if qb.p_diag is not None else torch.zeros(B, dtype=F64, device=dev)
    first = groups.gdates[:-1].long()[groups.gidx.long()]
    if not bool(((c == c[first]) & (pd == pd[first])).all().item()):
        return None
    k_ld = round_up(groups.ucnt_max, 64)
    ldh = min(64, round_up(groups.corr_max, 8))
    key = (B, G, k_ld, ldh)
    buf = getattr(ws, "_pgw", None)
    if buf is None or buf["key"] != key:
        buf = {"key": key,
               "M": torch.empty((G, k_ld, k_ld), dtype=F64, device=dev),
               "Minv": torch.empty((G, k_ld, k_ld), dtype=F64, device=dev),
               "Dt": torch.empty((G, k_ld // 64, 64, 64), dtype=F64, device=dev),
               "grho": torch.empty(G, dtype=F64, device=dev),
               "iters": torch.zeros(G, dtype=torch.int32, device=dev),
               "status": torch.zeros(max(G, B), dtype=torch.int32, device=dev),
               "info": torch.zeros(G, dtype=torch.int32, device=dev),
               "aq": torch.empty((B, 2 * k_ld), dtype=F64, device=dev),
               "hinv": torch.empty((B, ldh, ldh), dtype=F64, device=dev),
               "wscr": torch.empty((B, _lib.pg_wscr(k_ld)), dtype=F64, device=dev),
               "lb": torch.zeros(2, dtype=F64, device=dev), "ub": torch.ones(2, dtype=F64, device=dev)}
        ws._pgw = buf
    gi, sizes = groups.device_index()
    ld = torch.log(torch.clamp(settings.delta_wide * rec[:, _lib.PQ_PG_SC], min=1e-300))
    gl = torch.zeros(G, dtype=F64, device=dev).index_add_(0, gi, ld)
    buf["grho"].copy_(torch.exp(gl / sizes))
    gc = _lib.PQGcap(gdates=groups.gdates.data_ptr(), ngroups=G, urows=groups.urows.data_ptr(),
                     ucnt=groups.ucnt.data_ptr(), uoff=groups.uoff.data_ptr(), umax=groups.umax,
                     gidx=groups.gidx.data_ptr(), grho=buf["grho"].data_ptr(), M=buf["M"].data_ptr(),
                     Minv=buf["Minv"].data_ptr(), k_ld=k_ld, M_stride=k_ld * k_ld, aq=buf["aq"].data_ptr(),
                     aq_stride=2 * k_ld, hinv=buf["hinv"].data_ptr(), ldh=ldh)
    # the polish matrix: no general rows in the capacitance, a unit box (rho = delta_g), sigma 0
    pbw = qb.c_struct()
    pbw.mg = 0
    pbw.lb, pbw.ub, pbw.box_stride = buf["lb"].data_ptr(), buf["ub"].data_ptr(), 0
    sw = Settings(sigma=0.0).to_c()
    stw = _lib.PQState(status=buf["status"].data_ptr())
    L_ = ctypes.byref(lr.c_struct())
    band, ldo, r0 = bd["band"].data_ptr(), bd["ldo"], bd["r0"]
    pcp, ldpc = bd["pc"].data_ptr(), bd["pc"].stride(0)
    _lib.check(lib.pq_gcap_assemble(L_, ctypes.byref(pbw), ctypes.byref(gc), ctypes.byref(sw), band, ldo, r0, pcp,
                                    ldpc, bd["cc"].data_ptr(), strm), "pq_gcap_assemble (polish)")
    pbf = _lib.PQProblem(n=groups.ucnt_max, ld=k_ld, batch=G, mg=0, P=buf["M"].data_ptr(), P_stride=k_ld * k_ld,
                         q=qb.q.data_ptr(), q_stride=qb.q.stride(0), Cg=qb.Cg.data_ptr(), lg=qb.lg.data_ptr(),
                         ug=qb.ug.data_ptr())
    stf = _lib.PQState(K=buf["Minv"].data_ptr(), K_stride=k_ld * k_ld, Dt=buf["Dt"].data_ptr(),
                       Dt_stride=(k_ld // 64) * 4096, x=ws.x.data_ptr(), Px=ws.Px.data_ptr(), z=ws.z.data_ptr(),
                       y=ws.y.data_ptr(), m_ld=ws.m_ld, mg_pad=ws.mg_pad, rho=buf["grho"].data_ptr(),
                       iters=buf["iters"].data_ptr(), status=buf["status"].data_ptr(), info=buf["info"].data_ptr(),
                       out=ws.out.data_ptr(), work=ws.work.data_ptr(), work_stride=ws.work_stride)
    _lib.check(lib.pq_factor_batched(ctypes.byref(pbf), ctypes.byref(stf), None, 0, ctypes.byref(sw), 2, strm),
               "pq_factor_batched (polish M_U)")
    buf["status"].zero_()
    _lib.check(lib.pq_gcap_prepare(L_, ctypes.byref(pbw), ctypes.byref(stw), ctypes.byref(gc), ctypes.byref(sw),
                                   None, 0, band, ldo, r0, pcp, ldpc, strm), "pq_gcap_prepare (polish)")
    # a date whose correction H_b is not SPD to rounding, or whose group's M_U failed, keeps the
    # per-date kernel (state FALLBACK before the first round)
    bad = (buf["status"][:B] == _lib.PQ_NON_CONVEX) | (buf["info"][gi] != 0)
    rec[:, _lib.PQ_PG_STATE] = torch.where(bad & (rec[:, _lib.PQ_PG_STATE] == _lib.PQ_PG_PENDING),
                                           float(_lib.PQ_PG_FALLBACK), rec[:, _lib.PQ_PG_STATE])
    buf["gc"] = gc
    buf["wide"] = _lib.PQPgWide(gc=ctypes.pointer(gc), pc=pcp, ldpc=ldpc, r0=r0, cc=bd["cc"].data_ptr(),
                                nzr=_ptr(nzr), nzv=_ptr(nzv), nzmax=nzmax, wscr=buf["wscr"].data_ptr(),
                                wscr_stride=buf["wscr"].stride(0), refine_steps=int(settings.refine_wide))
    return buf["wide"]


def loose_stop_eps(settings: Settings, centred: bool, batch: int, mg: int = 1) -> float:
    """The eps of the loose ADMM stop before the grouped polish (0: none): eps_grouped for
    centred windows, eps_grouped_tracking for uncentred ones; when that is 0,
    eps_grouped_tracking_small (when > 0; default off) for uncentred batches of at most
    small_batch dates, else eps_grouped_tracking_wide for more than 4 general rows (the wide
    form).  eps_grouped = 0 turns every loose stop off."""
    if centred:
        return settings.eps_grouped
    eps = settings.eps_grouped_tracking
    if eps <= 0.0 and settings.eps_grouped > 0.0:
        if batch <= settings.small_batch and settings.eps_grouped_tracking_small > 0.0:
            eps = settings.eps_grouped_tracking_small
        elif mg > 4:
            eps = settings.eps_grouped_tracking_wide
    return eps


def solve_lowrank(qb: QPBatch, lr: LowRank, settings: Settings | None = None,
                  ws: Workspace | None = None, max_rounds: int = 64, events: list | None = None,
                  polish: bool = True, groups: "GroupPlan | None" = None, band: bool = True,
                  fuse: bool = True, grouped_polish: bool = True, gcap: bool = True,
                  eig: "EigCap | None" = None, wide_polish: bool = True, sync_free: bool = False,
                  graphs: "StageGraphs | None" = None, sf_rounds: int | None = None,
                  host_work=None, sweep: "SweepPlan | None" = None) -> BatchResult:
    """Woodbury-form solve for T + mg < n: K2 = capacitance SYRK + Cholesky/inverse of the
    k x k matrices M, K3 = low-rank ADMM over the shared window rows (grouped over sliding
    windows when a GroupPlan is given), K4 = window-form polish.  qb.P is never read (it
    may be None): P is the window (lr) throughout.

    ``sync_free`` (group capacitance with the grouped polish, no wide rounds): the stages
    run without any host synchronisation -- one ADMM launch, ``sf_rounds`` polish rounds
    (default settings.polish_rounds) -- and one flag read at the end decides whether the
    usual host-driven repairs must run (an adaptive-rho refactorisation: the whole solve is
    redone the host-driven way; dates still pending, handed back, or rejected: the remaining
    rounds, the per-date polish and the ADMM retry, exactly as without it).  With ``graphs``
    (StageGraphs) the sync-free stages are captured once and replayed.  ``host_work`` (a
    callable, sync-free only): the caller's host work that needs no result, run while the
    device works, just before the flag read.  ``sweep`` (SweepPlan: groups of up to 64
    problems sharing one window, porqua_amd.sweep): the fused ADMM runs as pq_admm_lr_sweep
    (two chip-wide launches per iteration) instead of one workgroup per group."""
    if sync_free and not (gcap and eig is None and groups is not None and grouped_polish and polish):
        sync_free = False
    tl = _Timeline(events, graphs if sync_free else None)
    if tl.graphs is not None:
        tl.graphs.begin()
    lib = _lib.load()
    s = (settings or Settings()).to_c()
    ws = ws or Workspace(qb, dense=False)
    B, dev = qb.batch, qb.device
    ldk = ws.ldk
    k = lr.tmax + qb.mg
    k_ld = round_up(k, 64)
    if not lowrank_applicable(qb, lr):
        raise _lib.PorquaHipError(f"low-rank form not applicable (k={k}, n={qb.n})")
    M = ws.lr_buffers(k_ld)
    pb = qb.c_struct()
    st = ws.c_struct()
    lrs = lr.c_struct()
    # n = k: the padded tail of M is the identity, so the factor skips its pivot steps
    pbM = _lib.PQProblem(n=k, ld=k_ld, batch=B, mg=0, P=M["M"].data_ptr(), P_stride=k_ld * k_ld,
                         q=qb.q.data_ptr(), q_stride=qb.q.stride(0), Cg=qb.Cg.data_ptr(), lg=qb.lg.data_ptr(),
                         ug=qb.ug.data_ptr())
    stM = _lib.PQState(K=M["Minv"].data_ptr(), K_stride=k_ld * k_ld, Dt=M["Dt"].data_ptr(),
                       Dt_stride=(k_ld // 64) * 4096, x=ws.x.data_ptr(), Px=ws.Px.data_ptr(),
                       z=ws.z.data_ptr(), y=ws.y.data_ptr(), m_ld=ws.m_ld, mg_pad=ws.mg_pad,
                       rho=ws.rho.data_ptr(), iters=M["iters"].data_ptr(), status=M["status"].data_ptr(),
                       info=M["info"].data_ptr(), out=ws.out.data_ptr(), work=ws.work.data_ptr(),
                       work_stride=ws.work_stride)
    sM = (settings or Settings()).to_c()
    sM.sigma = 0.0
    strm = _stream()
    P_, S_, SS, L_ = ctypes.byref(pb), ctypes.byref(st), ctypes.byref(s), ctypes.byref(lrs)
    PM_, SM_, SSM = ctypes.byref(pbM), ctypes.byref(stM), ctypes.byref(sM)
    _lib.check(lib.pq_init_state_lr(L_, P_, S_, None, 0, SS, strm), "pq_init_state_lr")
    _rho_floor_q(qb, ws, settings or Settings())

    bd = None

    def refactor(idx, nidx):
        if eig is not None:   # from the per-date eigendecompositions: no factorisation
            eig.form(L_, P_, S_, SS, M["Minv"], idx, nidx, strm)
            return
        if bd is not None:
            _lib.check(lib.pq_lr_capacitance_band(L_, P_, S_, _ptr(idx), nidx, SS, bd["band"].data_ptr(), bd["ldo"],
                                                  bd["r0"], bd["pc"].data_ptr(), bd["pc"].stride(0),
                                                  bd["cc"].data_ptr(), M["M"].data_ptr(), k_ld, k_ld * k_ld, strm),
                       "pq_lr_capacitance_band")
        else:
            _lib.check(lib.pq_lr_capacitance(L_, P_, S_, _ptr(idx), nidx, SS, M["M"].data_ptr(), k_ld,
                                             k_ld * k_ld, strm), "pq_lr_capacitance")
        _lib.check(lib.pq_factor_batched(PM_, SM_, _ptr(idx), nidx, SSM, 1, strm), "pq_factor_batched(M)")

    grouped = grouped_applicable(qb, lr, groups, ws)
    sparse_cols = _sparse_columns(qb) if grouped else (None, None, 0)
    # group capacitance: shared rows, register-resident (mg <= 4) or column-sparse (mg <= 24,
    # <= 4 nonzeros per asset); pass 1 of admm_gcap.hip covers U + mg <= 320 rows
    # (box-only problems, mg = 0, included: k_admm_gcap<0> once read an undefined Cg register
    # and stopped every date after one iteration; fixed, tests/test_gcap_gpu.py)
    gcap_try = (gcap and eig is None and grouped and fuse and qb.shared
                and (qb.mg <= 4 or (qb.mg <= 24 and sparse_cols[2] > 0))
                and groups.ucnt_max + qb.mg <= 320 and groups.corr_max <= 64)
    # the group capacitance's own plan: up to 32 dates per group (GroupPlan.gcap_plan), for
    # register-resident general rows and (GCAP32_WIDE) the column-sparse wide form; the polish
    # keeps its 16-date groups (polish_plan)
    gplan = groups
    if gcap_try and (qb.mg <= 4 or GCAP32_WIDE):
        g32 = groups.gcap_plan()
        if g32.ucnt_max + qb.mg <= 320 and g32.corr_max <= 64:
            gplan = g32
    if band:
        # the band must cover every union the capacitances read: the ADMM's groups and the
        # polish's (wide rounds)
        wmin = (max(gplan.span_max, groups.polish_plan().span_max) if (gcap_try or (grouped and wide_polish))
                else 0)
        bd = tl("gram", lambda: _band_setup(qb, lr, strm, w_min=wmin))
        ws.band_shape = (bd["nrows"], bd["W"]) if bd is not None else None   # (the bench's gram rate)
    gc = _gcap_setup(qb, lr, ws, gplan, settings or Settings()) if (gcap_try and bd is not None) else None
    ws.gcap_groups = gplan if gc is not None else None   # (the bench's roofline reads the plan used)

    def refactor_groups():
        """Group capacitance: one M_U per group (current group rho), its inverse, and every
        date's a_b, q_b, H_b^-1."""
        g = gc
        GC_ = ctypes.byref(g["c"])
        _lib.check(lib.pq_gcap_assemble(L_, P_, GC_, SS, bd["band"].data_ptr(), bd["ldo"], bd["r0"],
                                        bd["pc"].data_ptr(), bd["pc"].stride(0), bd["cc"].data_ptr(), strm),
                   "pq_gcap_assemble")
        if GCAP_FACTOR == "large":   # (experiment) many workgroups per M_U: K2L, one tile each
            if g.get("W") is None:
                g["W"] = torch.empty_like(g["M"])
            _lib.check(lib.pq_factor_large(ctypes.byref(g["pb"]), ctypes.byref(g["st"]), None, 0, SSM, 2,
                                           g["W"].data_ptr(), g["W"].stride(0), strm), "pq_factor_large(M_U)")
        else:
            _lib.check(lib.pq_factor_batched(ctypes.byref(g["pb"]), ctypes.byref(g["st"]), None, 0, SSM, 2, strm),
                       "pq_factor_batched(M_U)")
        _lib.check(lib.pq_gcap_prepare(L_, P_, S_, GC_, SS, None, 0, bd["band"].data_ptr(), bd["ldo"], bd["r0"],
                                       bd["pc"].data_ptr(), bd["pc"].stride(0), strm), "pq_gcap_prepare")

    if gc is not None:
        tl("factor", refactor_groups)
    else:
        tl("factor", lambda: refactor(None, 0))

    def admm(idx, nidx):
        if gc is not None:   # group capacitance (admm_gcap.hip)
            nzr, nzv, nzmax = sparse_cols if qb.mg > 4 else (None, None, 0)
            return lib.pq_admm_lr_gcap(L_, P_, S_, ctypes.byref(gc["c"]), SS, int(s.max_iter), bd["pc"].data_ptr(),
                                       bd["pc"].stride(0), bd["r0"], bd["cc"].data_ptr(), _ptr(nzr), _ptr(nzv),
                                       nzmax, strm)
        if grouped:   # every group relaunches; solved dates are skipped inside
            fz = bd is not None and fuse and qb.mg <= 32   # uniform D + shared Cg: the fused form
            if fz and sweep is not None and sweep.applicable(qb, lr, k_ld):
                ws.sweep_admm = sweep   # (the bench's roofline reads which kernel ran)
                scr = sweep.buffer(qb, lib)
                return lib.pq_admm_lr_sweep(L_, P_, S_, M["Minv"].data_ptr(), k_ld, k_ld * k_ld,
                                            _ptr(sweep.gdates), sweep.ngroups, SS, int(s.max_iter),
                                            bd["pc"].data_ptr(), bd["pc"].stride(0), bd["r0"], bd["cc"].data_ptr(),
                                            int(sweep.q_shared), scr.data_ptr(), scr.numel(), strm)
            nzr, nzv, nzmax = sparse_cols
            return lib.pq_admm_lr_grouped(L_, P_, S_, M["Minv"].data_ptr(), k_ld, k_ld * k_ld,
                                          _ptr(groups.gdates), groups.ngroups, _ptr(groups.urows),
                                          _ptr(groups.ucnt), _ptr(groups.uoff), groups.umax, SS,
                                          int(s.max_iter), bd["pc"].data_ptr() if fz else None,
                                          bd["pc"].stride(0) if fz else 0, bd["r0"] if fz else 0,
                                          bd["cc"].data_ptr() if fz else None, _ptr(nzr), _ptr(nzv), nzmax,
                                          strm)
        return lib.pq_admm_lr_batched(L_, P_, S_, M["Minv"].data_ptr(), k_ld, k_ld * k_ld, _ptr(idx),
                                      nidx, SS, int(s.max_iter), strm)

    cnt = {"refactors": 0, "launches": 0, "pg_fallback": 0}
    if sync_free and gc is None:   # the group capacitance did not apply: host-driven solve
        sync_free = False
        tl.graphs = None

    def admm_rounds(idx, nidx, SSx, name="admm"):
        nonlocal SS
        SS0, SS = SS, SSx   # admm() reads SS
        for _ in range(max_rounds):
            _lib.check(tl(name, lambda: admm(idx, nidx)), "pq_admm_lr")
            cnt["launches"] += 1
            if sync_free:   # NEED_REFACTOR is caught by the flag at the end
                break
            need = torch.nonzero(ws.status == _lib.PQ_NEED_REFACTOR).flatten().to(torch.int32)
            kk = int(need.numel())
            if kk == 0:
                break
            idx, nidx = need.contiguous(), kk
            if gc is not None:    # the kernel agreed a new rho per group: rebuild every M_U
                tl("factor", refactor_groups)
            else:
                tl("factor", lambda: refactor(idx, nidx))
            cnt["refactors"] += kk
        SS = SS0

    def polish_w(idx, nidx, SSp=None, name="polish"):
        SS = SSp if SSp is not None else SS_main
        kmax = min(qb.ld, 1024)
        final = ldk >= kmax
        bk = (bd["band"].data_ptr(), bd["ldo"], bd["r0"]) if bd is not None else (None, 0, 0)
        _lib.check(tl(name, lambda: lib.pq_polish_w_batched(L_, P_, S_, _ptr(idx), nidx, SS, ldk, int(final),
                                                                *bk, strm)), "pq_polish_w_batched")
        if not final:   # free sets larger than the compact scratch: relaunch those with ldk = kmax
            over = torch.nonzero(ws.out[:, _lib.PQ_OUT_ROUNDS] < 0).flatten().to(torch.int32)
            m = int(over.numel())   # host sync: small vector
            if m:
                K2 = torch.empty((m, kmax, kmax), dtype=F64, device=dev)
                D2 = torch.empty((m, kmax // 64, 64, 64), dtype=F64, device=dev)
                st2 = ws.c_struct()
                st2.K, st2.K_stride = K2.data_ptr(), K2.stride(0)
                st2.Dt, st2.Dt_stride = D2.data_ptr(), D2.stride(0)
                over = over.contiguous()
                _lib.check(tl(name, lambda: lib.pq_polish_w_batched(L_, P_, ctypes.byref(st2), _ptr(over), m,
                                                                        SS, kmax, 1, *bk, strm)),
                           "pq_polish_w_batched (relaunch)")

    pg = {}

    def pg_start(allow_wide: bool):
        """k_pg_init (classification from the ADMM point) + the wide rounds' capacitance."""
        rec = ws.pg_record()
        g = groups.polish_plan()
        _lib.check(lib.pq_polish_grouped_init(L_, P_, S_, rec.data_ptr(), SS_main, strm), "pq_polish_grouped_init")
        scr = getattr(ws, "_pg_pass", None)
        if scr is None or scr.numel() < g.ngroups * _lib.PQ_PG_PASS_SCRATCH:
            scr = torch.empty(g.ngroups * _lib.PQ_PG_PASS_SCRATCH, dtype=F64, device=dev)
            ws._pg_pass = scr
        # free sets beyond the LDS solve (k_pg_init left each date's free count in PQ_PG_K): the
        # wide rounds' group capacitance, built once for the whole polish
        wide = None
        if allow_wide and wide_polish and bool((rec[:, _lib.PQ_PG_K] > min(ldk, 128)).any()):   # host sync
            wide = _pg_wide_setup(qb, lr, ws, g, bd, rec, settings or Settings(), sparse_cols, strm)
        cnt["pg_wide"] = wide is not None
        pg.update(rec=rec, g=g, scr=scr, wide=wide, wide_p=ctypes.byref(wide) if wide is not None else None,
                  rounds=0)

    def pg_round():
        g, rec = pg["g"], pg["rec"]
        _lib.check(lib.pq_polish_grouped_round(L_, P_, S_, rec.data_ptr(), ldk, _ptr(g.gdates), g.ngroups,
                                               _ptr(g.urows), _ptr(g.ucnt), _ptr(g.uoff), g.umax, SS_main,
                                               pg["scr"].data_ptr(), pg["wide_p"], strm), "pq_polish_grouped_round")
        pg["rounds"] += 1

    def pg_rounds_host():
        """The remaining rounds, each followed by a host check for dates still pending."""
        rec = pg["rec"]
        while pg["rounds"] < int(s.polish_rounds):
            if pg["rounds"] >= 2 and not bool((rec[:, _lib.PQ_PG_STATE] == _lib.PQ_PG_PENDING).any()):   # sync
                break
            pg_round()

    def polish_grouped():
        """Grouped polish pipeline (polish_g.hip) for every date; the dates it hands back
        (FALLBACK) go through pq_polish_w_batched from their ADMM point."""
        pg_start(True)
        pg_round()
        pg_rounds_host()
        pg_finish()

    def polish_sync_free():
        """The grouped polish with a fixed number of rounds and no host check (dates done
        early skip the later rounds' kernels), then one device flag: anything left for the
        host-driven repairs (dates pending, handed back or rejected, or an ADMM refactor)."""
        pg_start(False)
        for _ in range(min(int(sf_rounds or s.polish_rounds), int(s.polish_rounds))):
            pg_round()
        st_pg = pg["rec"][:, _lib.PQ_PG_STATE]
        flag = ((st_pg == _lib.PQ_PG_PENDING) | (st_pg == _lib.PQ_PG_FALLBACK) |
                (ws.status == _lib.PQ_NEED_REFACTOR) | (ws.status == _lib.PQ_SOLVED_INACCURATE) |
                (ws.status == _lib.PQ_UNSOLVED)).any()
        if getattr(ws, "_sf_flag", None) is None:
            ws._sf_flag = torch.zeros((), dtype=torch.bool, device=dev)
        ws._sf_flag.copy_(flag)
        return dict(pg)   # the pipeline state (a replayed graph does not run this function)

    def pg_finish():
        rec = pg["rec"]
        fb = torch.nonzero(rec[:, _lib.PQ_PG_STATE] == _lib.PQ_PG_FALLBACK).flatten().to(torch.int32)
        m = int(fb.numel())
        cnt["pg_fallback"] = m
        if m:
            ws.pg_fallback = fb   # the dates handed to the per-date kernel (diagnostics)
            if SS_admm is not SS_main:   # stopped at eps_grouped: resume those to eps first
                ws.status[fb.long()] = _lib.PQ_UNSOLVED
                admm_rounds(fb.contiguous(), m, SS_main, name="admm (resume, inside polish)")
            # two refinement steps per round for the hand-offs (vertex cycling, failed
            # factorisations): config 5's fallback polish 31.3 -> 7.5 ms
            # (profiles/r02k_bench_config5_qrel30.log -> r02l_bench_config5_fallback_refine2.log)
            sfb = type(s).from_buffer_copy(s)
            sfb.refine_iters = max(sfb.refine_iters, 2)
            polish_w(fb.contiguous(), m, ctypes.byref(sfb), name="polish (fallback, inside polish)")

    SS_main = SS
    SS_admm = SS
    st_ = settings or Settings()
    eps_loose = loose_stop_eps(st_, lr.mu is not None, qb.batch, qb.mg)
    if ((gc is not None or (st_.eps_grouped_percap and grouped and eig is None)) and polish and s.polish
            and grouped_polish and ldk >= 64 and eps_loose > max(st_.eps_abs, st_.eps_rel)):
        sl = st_.to_c()
        sl.eps_abs = sl.eps_rel = eps_loose
        sl.min_iter = max(int(st_.min_iter), int(st_.min_iter_grouped))
        SS_admm = ctypes.byref(sl)
    if sync_free and not (grouped and ldk >= 64 and s.polish):
        sync_free = False
        tl.graphs = None
    admm_rounds(None, 0, SS_admm)
    if sync_free:
        pg.update(tl("polish", polish_sync_free))
        if host_work is not None:
            host_work()
        if not bool(ws._sf_flag.item()):   # the one host sync of the step: nothing left to repair
            return _lowrank_result(qb, ws, cnt, "group")
        if bool((ws.status == _lib.PQ_NEED_REFACTOR).any() | (ws.status == _lib.PQ_UNSOLVED).any()):
            # an adaptive-rho refactorisation was requested: redo the whole solve host-driven
            return solve_lowrank(qb, lr, settings, ws, max_rounds, events, polish, groups, band, fuse,
                                 grouped_polish, gcap, eig, wide_polish)
        tl.graphs = None   # the repairs below are host-driven
        sync_free = False  # (admm_rounds checks for refactorisations again)
        pg_rounds_host()   # dates still pending: the remaining rounds
        pg_finish()        # dates handed back: the per-date polish
        polished = True
    else:
        polished = False
    if s.polish and polish:
        if not polished:
            if grouped and grouped_polish and ldk >= 64:
                tl("polish", polish_grouped)
            else:
                polish_w(None, 0)
        # one host sync: nothing rejected (the usual case) skips both repairs
        rejected = bool((ws.status == _lib.PQ_SOLVED_INACCURATE).any().item())
        rp = _repolish_set(ws, settings or Settings()) if rejected else None
        if rp is not None:      # polish rejected: polish again with more refinement steps
            pidx, pn, s3 = rp
            polish_w(pidx, pn, ctypes.byref(s3))
        retry = _retry_set(ws, settings or Settings()) if rejected else None
        if retry is not None:   # polish rejected: resume ADMM to eps_retry, polish again
            ridx, rn, s2 = retry
            admm_rounds(ridx, rn, ctypes.byref(s2))
            s4 = (settings or Settings()).to_c()
            s4.refine_iters = max(s4.refine_iters, (settings or Settings()).refine_retry)
            polish_w(ridx, rn, ctypes.byref(s4))
    return _lowrank_result(qb, ws, cnt, "group" if gc is not None else ("eig" if eig is not None else
                                                                       ("band" if bd is not None else "direct")))


def _lowrank_result(qb: QPBatch, ws: Workspace, cnt: dict, capacitance: str) -> BatchResult:
    n, mg = qb.n, qb.mg
    return BatchResult(x=ws.x[:, :n], y=ws.y[:, :mg], z_box=ws.y[:, ws.mg_pad:ws.mg_pad + n],
                       status=ws.status, iters=ws.iters, out=ws.out, refactors=cnt["refactors"],
                       admm_launches=cnt["launches"], polish_fallbacks=cnt["pg_fallback"], capacitance=capacitance)


def factor_only(qb: QPBatch, invert: bool = False, sigma: float = 0.0):
    """Batched Cholesky of P_eff (mg = 0, no box): returns (Workspace, info) -- the isPD
    test of src/helper_functions.py:61-67 on the device."""
    lib = _lib.load()
    s = Settings(sigma=sigma).to_c()
    ws = Workspace(qb)
    pb = qb.c_struct()
    pb.mg = 0
    pb.lb = pb.ub = None
    st = ws.c_struct()
    strm = _stream()
    _lib.check(lib.pq_init_state(ctypes.byref(pb), ctypes.byref(st), None, 0, ctypes.byref(s), strm), "init")
    _lib.check(lib.pq_factor_batched(ctypes.byref(pb), ctypes.byref(st), None, 0, ctypes.byref(s),
                                     2 if invert else 0, strm), "pq_factor_batched")
    return ws, ws.info


# ----------------------------------------------------------------------------------------
# Windows and K1
# ----------------------------------------------------------------------------------------


def window_rows(dates: np.ndarray, rebdates, width: int):
    """Per-date row lists of ``data[data.index <= rebdate].tail(width)`` minus weekends
    (src/builders.py:208-211).  Returns (rows int32 [B, Tmax], tlen int32 [B])."""
    dates = np.asarray(dates, dtype="datetime64[D]")
    reb = np.asarray(rebdates, dtype="datetime64[D]")
    ends = np.searchsorted(dates, reb, side="right")
    starts = np.maximum(0, ends - int(width))
    B = len(ends)
    weekday = (dates.astype("int64") + 3) % 7 < 5
    # the weekdays of [s, e) are the positions wpos[cw[s] .. cw[e]) (prefix counts)
    wpos = np.flatnonzero(weekday).astype(np.int32)
    cw = np.concatenate([[0], np.cumsum(weekday)]).astype(np.int64)
    first = cw[starts]
    tlen = (cw[ends] - first).astype(np.int32)
    tmax = max(1, int(tlen.max())) if B else 1
    if not len(wpos):
        return np.zeros((B, tmax), dtype=np.int32), tlen
    # int32 index arithmetic; a calendar without weekend rows (the usual return panel) needs
    # no position lookup at all (wpos is the identity)
    j = np.arange(tmax, dtype=np.int32)[None, :]
    idx = first.astype(np.int32)[:, None] + j
    if len(wpos) != len(dates):
        idx = wpos[np.minimum(idx, len(wpos) - 1)]
    if int(tlen.min()) == tmax:   # every window full (the usual backtest): nothing to mask
        return idx.astype(np.int32, copy=False), tlen
    rows = idx * (j < tlen[:, None])
    return rows.astype(np.int32, copy=False), tlen


def slide_plan(rows, tlen, group: int = 32, smax: int = 64, smin: int = 1):
    """Host plan for pq_cov_slide_batched: ``(gstart int32 [G+1], shift int32 [B])``.

    Date d joins the group of date d-1 when its window is that window shifted by
    smin <= s <= smax rows (same length, rows[d][:T-s] == rows[d-1][s:T]) and the group
    holds fewer than ``group`` dates; otherwise d starts a new group (a full-SYRK anchor).
    smin = 0 also joins identical windows (several problems of one date, e.g. a
    risk-aversion sweep) -- the grouped ADMM accepts that, the sliding K1 does not."""
    rows = np.asarray(rows)
    tlen = np.asarray(tlen)
    B, tmax = rows.shape
    shift = np.zeros(B, dtype=np.int32)
    if B > 1:
        col = np.arange(tmax)
        prev, cur = rows[:-1], rows[1:]
        tp, tc = tlen[:-1], tlen[1:]
        # s = #rows of the previous window before the current window's first row; only
        # s <= smax can join, so the first smax + 1 columns decide it
        h = min(tmax, int(smax) + 1)
        # windows that are one contiguous run of panel rows (no gap: last - first = T - 1)
        # of the same length, the current one starting exactly s rows after the previous one,
        # are that window shifted by s -- no element compare needed.  (Without the start check
        # a later window starting EARLIER -- descending or shuffled dates -- counts s = 0 and
        # would pass as identical.)
        last = rows[np.arange(B), np.maximum(tlen - 1, 0)]
        contig = (last - rows[:, 0]) == (tlen - 1)
        if contig.all():   # (the same count from the window starts alone)
            s = np.minimum(np.clip(cur[:, 0].astype(np.int64) - prev[:, 0], 0, tp), h)
        else:
            s = ((prev[:, :h] < cur[:, :1]) & (col[None, :h] < tp[:, None])).sum(1)
        cand = (tp == tc) & (tc > 1) & (s >= smin) & (s <= smax)
        match = cand & contig[:-1] & contig[1:] & ((cur[:, 0] - prev[:, 0]) == s)
        need = cand & ~match
        for sv in np.unique(s[need]).tolist():   # rows[d][:T-s] == rows[d-1][s:T], per shift value
            sel = np.flatnonzero(need & (s == sv))
            w = tmax - sv
            ok = ((prev[sel, sv:] == cur[sel, :w]) | (col[None, :w] >= (tc[sel] - sv)[:, None])).all(1)
            match[sel[ok]] = True
        good = cand & match
        shift[1:] = np.where(good, s, 0)
    else:
        good = np.zeros(0, dtype=bool)
    joins = np.concatenate([[False], good])
    # runs of joined dates, cut every ``group`` dates: d starts a group when it does not
    # join its predecessor or sits at a multiple of ``group`` inside its run
    run_start = np.maximum.accumulate(np.where(~joins, np.arange(B), 0)) if B else np.zeros(0, np.int64)
    starts = np.flatnonzero((np.arange(B) - run_start) % max(int(group), 1) == 0)
    return np.concatenate([starts, [B]]).astype(np.int32), shift


class SlidePlan:
    """Device copy of a slide_plan (see pq_cov_slide_batched)."""

    def __init__(self, rows, tlen, device, group: int = 32, smax: int = 64):
        gs, sh = slide_plan(rows, tlen, group, smax)
        self.ngroups = len(gs) - 1
        self.gstart = torch.from_numpy(gs).to(device)
        self.shift = torch.from_numpy(sh).to(device)


GROUP_MAX_DATES = 16     # MFMA N of the grouped ADMM (admm_grp.hip GMAX)
# dates per group of the group-capacitance ADMM with its two MFMA column blocks (admm_gcap.hip,
# NB = 2: one 512-thread workgroup per CU); PQ_GCAP_GMAX=16 keeps the 16-date groups (A/B)
GCAP_MAX_DATES = int(os.environ.get("PQ_GCAP_GMAX", "32"))
# the 32-date groups also for the wide form (column-sparse general rows, config 4's sector
# caps); PQ_GCAP32_WIDE=0: 16-date groups there (A/B)
GCAP32_WIDE = os.environ.get("PQ_GCAP32_WIDE", "1") != "0"
GCAP_FACTOR = os.environ.get("PQ_GCAP_FACTOR", "batched")   # (A/B) "large": K2L for the group factor
GROUP_MAX_UNION = 320    # union rows per group (admm_grp.hip UMAXG)


SWEEP_ADMM = os.environ.get("PQ_SWEEP_ADMM", "1") != "0"   # (A/B) 0: the sweep's groups on k_admm_grp


class SweepPlan:
    """Problem groups for pq_admm_lr_sweep (admm_sweep.hip): runs of up to 64 consecutive
    problems that share one window and its centring (the risk-aversion row of a rebalance
    date, porqua_amd.sweep), with the kernel's scratch (per-problem records, per-chunk
    partials, the pass-2 operand).  ``q_shared``: the problems of a group share q as well."""

    GMAX = 64

    def __init__(self, counts, device, q_shared: bool = False):
        self.q_shared = bool(q_shared)
        starts, b = [], 0
        for c in counts:
            starts.extend(range(b, b + int(c), self.GMAX))
            b += int(c)
        starts.append(b)
        self.gdates = torch.tensor(starts, dtype=torch.int32, device=device)
        self.ngroups = len(starts) - 1
        self.scratch = None

    def applicable(self, qb: "QPBatch", lr: "LowRank", k_ld: int) -> bool:
        return (SWEEP_ADMM and self.ngroups > 0 and lr.tmax <= 256 and k_ld <= 256 and qb.mg <= 4
                and qb.lb is not None and qb.ub is not None and qb.shared)

    def buffer(self, qb: "QPBatch", lib) -> torch.Tensor:
        need = int(lib.pq_sweep_scratch_doubles(qb.n, qb.batch, self.ngroups))
        if self.scratch is None or self.scratch.numel() < need:
            self.scratch = torch.empty(need, dtype=F64, device=qb.device)
        return self.scratch


class GroupPlan:
    """Date groups for pq_admm_lr_grouped: runs of consecutive dates whose windows slide
    (slide_plan), at most ``gmax`` dates and ``umax`` union rows each.  ``ok`` is False
    when some window cannot be grouped (the per-date kernel is used then)."""

    def __init__(self, rows, tlen, device, gmax: int = GROUP_MAX_DATES, umax: int = GROUP_MAX_UNION,
                 smax: int = 64, cus: int = 256, gmin: int = 4, breaks=None, polish_full: bool = False):
        """``breaks`` (bool per problem, optional): True starts a new group at that problem
        (e.g. the risk-aversion buckets of porqua_amd.sweep, whose problems may share a
        capacitance only within a rho bucket).  ``polish_full``: polish_plan() builds a second plan
        of full 16-date groups for the grouped polish (a second host pass over the windows: worth
        it for a batch solved repeatedly, e.g. the bench workloads)."""
        rows = np.asarray(rows)
        tlen = np.asarray(tlen)
        B = len(tlen)
        self._host = (rows, tlen, device, umax, smax, breaks, cus, gmax)
        self._polish_full = polish_full
        self._polish_plan = None
        self._gcap_plan = None
        self._gmin = gmin
        # balance: one group per CU per round (one 512-thread workgroup fits a CU), as few
        # rounds as gmax allows, groups as even as possible within them
        rounds = max(1, -(-B // (gmax * cus)))
        gmax = max(1, min(gmax, max(gmin, -(-B // (rounds * cus)))))
        self.ok = B > 0 and int(tlen.min()) >= 2 and int(tlen.max()) <= umax
        gs, sh = slide_plan(rows, tlen, group=gmax, smax=smax, smin=0)
        # windows that are runs of consecutive panel rows, each joined one starting exactly its
        # shift after its predecessor: every union is then a run too (the fast path below; a
        # shift of a whole window or more joins disjoint windows, whose union has gaps)
        contig_all = bool(B) and bool(((rows[np.arange(B), np.maximum(tlen - 1, 0)] - rows[:, 0]) == (tlen - 1)).all()
                                      and ((sh[1:] == 0) | (rows[1:, 0] - rows[:-1, 0] == sh[1:])).all())
        groups = []
        # a slide group whose whole union fits (first window + every later shift <= umax) is
        # one date group; only the others are cut greedily, date by date
        cs = np.concatenate([[0], np.cumsum(sh[1:], dtype=np.int64)]) if B else np.zeros(1, np.int64)
        fits = (tlen[gs[:-1]] + cs[gs[1:] - 1] - cs[gs[:-1]]) <= umax if B else np.zeros(0, bool)
        tl_l, sh_l = tlen.tolist(), sh.tolist()
        for a, b, f in zip(gs[:-1].tolist(), gs[1:].tolist(), fits.tolist()):
            if f:
                groups.append((a, b))
                continue
            start, U = a, tl_l[a]
            for d in range(a + 1, b):
                if U + sh_l[d] > umax:
                    groups.append((start, d))
                    start, U = d, tl_l[d]
                else:
                    U += sh_l[d]
            groups.append((start, b))
        if breaks is not None:
            brk = np.flatnonzero(np.asarray(breaks, dtype=bool))
            split = []
            for a, b in groups:
                cut = [a] + [int(c) for c in brk if a < c < b] + [b]
                split += list(zip(cut[:-1], cut[1:]))
            groups = split
        self.ngroups = len(groups)
        self.umax = umax
        gdates = np.array([a for a, _ in groups] + [B], dtype=np.int32)
        urows = np.zeros((max(1, self.ngroups), umax), dtype=np.int32)
        ucnt = np.zeros(max(1, self.ngroups), dtype=np.int32)
        uoff = np.zeros(B, dtype=np.int32)
        if B and self.ngroups:
            # a group's union = its first window, then the rows each later date adds (its last
            # sh[d] window rows); every (date, column) entry gathered at once
            sizes = np.diff(gdates)
            gof = np.repeat(np.arange(self.ngroups), sizes)                 # group of each date
            isfirst = np.zeros(B, dtype=bool)
            isfirst[gdates[:-1]] = True
            shd = np.where(isfirst, 0, sh).astype(np.int64)
            cnt = np.where(isfirst, tlen, shd).astype(np.int64)             # entries per date
            col0 = np.where(isfirst, 0, tlen - shd)
            cum = np.cumsum(shd)
            uoff[:] = cum - cum[gdates[:-1]][gof]                           # sum of shifts since the group start
            cnts = np.add.reduceat(cnt, gdates[:-1]) if self.ngroups else np.zeros(0, np.int64)
            over = cnts > umax
            if over.any():
                self.ok = False
            g0 = gdates[:-1]
            if contig_all:
                # every window one run of consecutive panel rows (daily / monthly calendars
                # without gaps): a group's union is the run from its first window's first row
                u = np.arange(umax)[None, :]
                urows[:] = np.where((u < cnts[:, None]) & ~over[:, None], rows[g0, 0][:, None] + u, 0)
            else:
                estart = np.concatenate([[0], np.cumsum(cnt)])
                tot = int(estart[-1])
                dte = np.repeat(np.arange(B), cnt)
                k = np.arange(tot) - estart[dte]
                vals = rows[dte, col0[dte] + k]
                gstart_e = estart[g0]                                       # first entry of each group
                pos = np.arange(tot) - gstart_e[gof[dte]]
                keep = ~over[gof[dte]]
                urows[gof[dte][keep], pos[keep]] = vals[keep]
            ucnt[:] = np.where(over, 0, cnts)
        self.sizes = np.diff(gdates)
        gidx = np.repeat(np.arange(max(self.ngroups, 0), dtype=np.int32), self.sizes) if B else np.zeros(0, np.int32)
        # widest union span in panel rows (the band Gram must cover it for the group capacitance)
        if self.ngroups and ucnt.max() > 0:
            valid = np.arange(umax)[None, :] < ucnt[:, None]
            hi = np.where(valid, urows, np.iinfo(np.int32).min).max(1)
            lo = np.where(valid, urows, np.iinfo(np.int32).max).min(1)
            self.span_max = int((hi - lo + 1)[ucnt > 0].max())
        else:
            self.span_max = 0
        self.ucnt_max = int(ucnt.max()) if self.ngroups else 0
        # rank of the Woodbury correction of a date: union rows outside its window + the mean
        self.corr_max = int((ucnt[gidx] - tlen).max()) + 1 if B else 1
        self.gdates = torch.from_numpy(gdates).to(device)
        self.urows = torch.from_numpy(urows).to(device)
        self.ucnt = torch.from_numpy(ucnt).to(device)
        self.uoff = torch.from_numpy(uoff).to(device)
        self.gidx = torch.from_numpy(gidx).to(device)
        self._dev_index = None

    def polish_plan(self) -> "GroupPlan":
        """The plan of the grouped polish: full 16-date groups (its window passes run split
        over 4 workgroups per group, so fewer, fuller groups read fewer union rows; measured at
        the config-3 shape, profiles/r03i_bench_gmin*.log: polish 5.26 -> 4.92 ms at 16 dates per
        group, while the ADMM wants the CU-balanced size: 8.06 -> 8.51 ms)."""
        if not self._polish_full:
            return self
        if self._polish_plan is None:
            rows, tlen, device, umax, smax, breaks, cus, gmax0 = self._host
            full = self.ngroups == 0 or int(self.sizes.max()) >= min(gmax0, GROUP_MAX_DATES)
            # same breaks (e.g. rho buckets) and CU count: polish groups never straddle a break
            self._polish_plan = None if full else GroupPlan(rows, tlen, device, umax=umax, smax=smax, cus=cus,
                                                            gmax=gmax0, gmin=gmax0, breaks=breaks)
            if full:
                self._polish_full = False
        return self._polish_plan if self._polish_plan is not None else self

    def gcap_plan(self) -> "GroupPlan":
        """The plan of the group-capacitance ADMM (admm_gcap.hip) for register-resident general
        rows (mg <= 4): CU-balanced groups of up to GCAP_MAX_DATES dates (its 32-date form: one
        workgroup per CU streams one union for all of them -- half the union traffic and half the
        group factorisations of two 16-date groups; config 3: 475 groups of 10 -> 250 of 19).
        This plan itself when that changes nothing (small batches, GCAP_MAX_DATES <= 16)."""
        if self._gcap_plan is None:
            rows, tlen, device, umax, smax, breaks, cus, gmax0 = self._host
            g = self
            if GCAP_MAX_DATES > gmax0 and self.ngroups > 0:
                g32 = GroupPlan(rows, tlen, device, gmax=min(GCAP_MAX_DATES, 32), umax=umax, smax=smax, cus=cus,
                                gmin=self._gmin, breaks=breaks)
                if g32.ok and g32.ngroups < self.ngroups and int(g32.sizes.max()) > gmax0:
                    g = g32
            self._gcap_plan = g
        return self._gcap_plan

    def device_index(self):
        """(group of each date as int64, dates per group as FP64) on the device, built once."""
        if self._dev_index is None:
            self._dev_index = (self.gidx.long(), torch.from_numpy(self.sizes.astype(np.float64)).to(self.gidx.device))
        return self._dev_index


class Panel:
    """A device-resident return panel (D_total x n, row-major) with optional benchmark."""

    def __init__(self, returns, bm=None, device=None):
        self.device = device or default_device()
        R = returns if isinstance(returns, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(returns, dtype=np.float64))
        self.R = R.to(self.device, dtype=F64).contiguous()
        self.D, self.n = self.R.shape
        self.bm = None
        if bm is not None:
            y = bm if isinstance(bm, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(bm, dtype=np.float64).reshape(-1))
            self.bm = y.to(self.device, dtype=F64).contiguous()

    def window_sumsq(self, rows, tlen, mu=None, out=None):
        """diag(Xc'Xc) of every window (mu None: diag X'X) -> (B, round_up(n, 64))."""
        lib = _lib.load()
        B, tmax = rows.shape
        if out is None:
            out = torch.zeros((B, round_up(self.n, 64)), dtype=F64, device=self.device)
        _lib.check(lib.pq_window_sumsq(_ptr(self.R), self.R.stride(0), self.n, _ptr(rows), _ptr(tlen), tmax, B,
                                       _ptr(mu), 0 if mu is None else mu.stride(0), _ptr(out), out.stride(0),
                                       _stream()), "pq_window_sumsq")
        return out

    def window_moments_grouped(self, groups: "GroupPlan", tlen, mu, dg):
        """Window means and diag(Xc'Xc) of every date of a GroupPlan in one sliding pass over
        each group's union rows (pq_window_moments_grouped), into ``mu`` and ``dg``."""
        lib = _lib.load()
        _lib.check(lib.pq_window_moments_grouped(_ptr(self.R), self.R.stride(0), self.n, _ptr(groups.gdates),
                                                 groups.ngroups, _ptr(groups.urows), groups.umax,
                                                 _ptr(groups.uoff), _ptr(tlen), _ptr(mu), mu.stride(0), _ptr(dg),
                                                 dg.stride(0), _stream()), "pq_window_moments_grouped")
        return mu, dg

    def window_geomeans_grouped(self, groups: "GroupPlan", tlen, out=None):
        """Geometric window means (MeanEstimator.estimate_geometric) of every date of a
        GroupPlan in one sliding pass per group (pq_window_geomean_grouped) -> (B, round_up(n, 64))."""
        lib = _lib.load()
        B = int(tlen.shape[0])
        mu = out if out is not None else torch.zeros((B, round_up(self.n, 64)), dtype=F64, device=self.device)
        _lib.check(lib.pq_window_geomean_grouped(_ptr(self.R), self.R.stride(0), self.n, _ptr(groups.gdates),
                                                 groups.ngroups, _ptr(groups.urows), groups.umax,
                                                 _ptr(groups.uoff), _ptr(tlen), _ptr(mu), mu.stride(0),
                                                 _stream()), "pq_window_geomean_grouped")
        return mu

    def rows_to_device(self, rows, tlen):
        r = torch.from_numpy(np.ascontiguousarray(rows, dtype=np.int32)).to(self.device)
        t = torch.from_numpy(np.ascontiguousarray(tlen, dtype=np.int32)).to(self.device)
        return r, t

    def window_means(self, rows, tlen, geometric=False, out=None):
        lib = _lib.load()
        B, tmax = rows.shape
        mu = out if out is not None else torch.zeros((B, round_up(self.n, 64)), dtype=F64, device=self.device)
        fn = lib.pq_window_geomean if geometric else lib.pq_window_mean
        _lib.check(fn(_ptr(self.R), self.n, self.n, _ptr(rows), _ptr(tlen), tmax, B, _ptr(mu),
                      mu.stride(0), _stream()), "window means")
        return mu

    def window_nanmeans(self, rows, tlen, geometric=False, out=None):
        """Column means over the present rows of every window (NaN-aware; pandas skipna),
        arithmetic or geometric -> (B, round_up(n, 64))."""
        lib = _lib.load()
        B, tmax = rows.shape
        mu = out if out is not None else torch.zeros((B, round_up(self.n, 64)), dtype=F64, device=self.device)
        _lib.check(lib.pq_window_nanmean(_ptr(self.R), self.R.stride(0), self.n, _ptr(rows), _ptr(tlen), tmax, B,
                                         _ptr(mu), mu.stride(0), int(geometric), _stream()), "pq_window_nanmean")
        return mu

    @property
    def has_nan(self) -> bool:
        if getattr(self, "_has_nan", None) is None:
            self._has_nan = bool(torch.isnan(self.R).any().item())
        return self._has_nan

    def cov_pairwise(self, rows, tlen, out=None):
        """Pairwise-complete covariance of windows with missing values (pandas
        DataFrame.cov() with NaN, src/covariance.py:65-66) -> (B, ld, ld); NaN where a pair
        has fewer than 2 common rows."""
        lib = _lib.load()
        B, tmax = rows.shape
        ld = round_up(self.n, 64)
        c = torch.nan_to_num(self.window_nanmeans(rows, tlen), nan=0.0)   # all-missing column: no shift
        if out is None:
            out = torch.empty((B, ld, ld), dtype=F64, device=self.device)
        _lib.check(lib.pq_cov_pairwise_batched(_ptr(self.R), self.R.stride(0), self.n, _ptr(rows), _ptr(tlen), tmax,
                                               B, _ptr(c), c.stride(0), _ptr(out), ld, out.stride(0), _stream()),
                   "pq_cov_pairwise_batched")
        return out

    def cov(self, rows, tlen, mode=0, out=None, mu=None, plan: SlidePlan | None = None,
            lower_only: bool = False):
        """K1: per-date centred covariance (mode 0, ddof=1) or Gram X'X (mode 1) -> (B, ld, ld).
        With a SlidePlan, overlapping windows are built by rank-2s updates (same result);
        ``lower_only`` (SlidePlan only) leaves the strictly-upper off-diagonal tiles unwritten."""
        lib = _lib.load()
        B, tmax = rows.shape
        ld = round_up(self.n, 64)
        if mode == 0 and mu is None:
            mu = self.window_means(rows, tlen)
        if out is None:
            out = torch.empty((B, ld, ld), dtype=F64, device=self.device)
        mp = _ptr(mu) if mode == 0 else None
        ms = mu.stride(0) if mode == 0 else 0
        if plan is not None:
            _lib.check(lib.pq_cov_slide_batched(_ptr(self.R), self.R.stride(0), self.n, _ptr(rows), _ptr(tlen),
                                                tmax, B, mode, mp, ms, _ptr(out), ld, out.stride(0),
                                                _ptr(plan.gstart), plan.ngroups, _ptr(plan.shift),
                                                1 if lower_only else 0, _stream()),
                       "pq_cov_slide_batched")
            return out
        _lib.check(lib.pq_cov_batched(_ptr(self.R), self.R.stride(0), self.n, _ptr(rows), _ptr(tlen), tmax, B,
                                      mode, mp, ms, _ptr(out), ld, out.stride(0), _stream()), "pq_cov_batched")
        return out

    def gram_xy(self, rows, tlen):
        lib = _lib.load()
        if self.bm is None:
            raise ValueError("Benchmark return series data is missing.")
        B, tmax = rows.shape
        ld = round_up(self.n, 64)
        xty = torch.zeros((B, ld), dtype=F64, device=self.device)
        yty = torch.zeros(B, dtype=F64, device=self.device)
        _lib.check(lib.pq_gram_xy_batched(_ptr(self.R), self.n, self.n, _ptr(self.bm), _ptr(rows),
                                          _ptr(tlen), tmax, B, _ptr(xty), xty.stride(0), _ptr(yty),
                                          _stream()), "pq_gram_xy_batched")
        return xty, yty

    def gram_xy_grouped(self, groups: "GroupPlan", tlen, dg=None, xty=None):
        """gram_xy for the dates of a GroupPlan in one sliding pass per group
        (pq_gram_xy_grouped: O(n) per date after each group's first window); ``dg`` (optional,
        (B, >= n)) receives diag(X'X) of every window from the same pass."""
        lib = _lib.load()
        if self.bm is None:
            raise ValueError("Benchmark return series data is missing.")
        B = int(tlen.shape[0])
        ld = round_up(self.n, 64)
        if xty is None:
            xty = torch.zeros((B, ld), dtype=F64, device=self.device)
        yty = torch.zeros(B, dtype=F64, device=self.device)
        _lib.check(lib.pq_gram_xy_grouped(_ptr(self.R), self.R.stride(0), self.n, _ptr(self.bm), _ptr(groups.gdates),
                                          groups.ngroups, _ptr(groups.urows), groups.umax, _ptr(groups.uoff),
                                          _ptr(tlen), _ptr(xty), xty.stride(0), _ptr(yty), _ptr(dg),
                                          0 if dg is None else dg.stride(0), _stream()), "pq_gram_xy_grouped")
        return xty, yty



class PeriodPlan:
    """Device tables of one simulation launch: first panel row and row count of every
    holding period, the offset of its returns in the flattened series and (for the fixed
    cost) the calendar day of every return.  Built once, reusable across launches."""

    def __init__(self, row0, nrows, ret_day=None, device=None, panel_rows=None):
        row0 = np.asarray(row0, dtype=np.int64)
        nrows = np.asarray(nrows, dtype=np.int64)
        if len(row0) != len(nrows):
            raise ValueError("PeriodPlan: one (row0, nrows) per period")
        if len(row0) and (row0.min() < 0 or nrows.min() < 1 or
                          (panel_rows is not None and (row0 + nrows).max() > panel_rows)):
            raise ValueError("PeriodPlan: period rows outside the panel")
        self.nper = len(row0)
        self.rows_end = int((row0 + nrows).max()) if self.nper else 0
        nret = np.maximum(nrows - 1, 0)
        off = np.concatenate([[0], np.cumsum(nret)[:-1]]) if self.nper else np.zeros(0, np.int64)
        self.total = int(nret.sum())
        dev = device or default_device()
        self.row0 = torch.as_tensor(row0.astype(np.int32), device=dev)
        self.nrows = torch.as_tensor(nrows.astype(np.int32), device=dev)
        self.off = torch.as_tensor(off.astype(np.int64), device=dev)
        self.ret_day = None
        if ret_day is not None:
            if len(ret_day) != self.total:
                raise ValueError("PeriodPlan: one calendar day per return")
            self.ret_day = torch.as_tensor(np.asarray(ret_day, dtype=np.int32), device=dev)


def simulate_periods(panel: torch.Tensor, W: torch.Tensor, plan, nrows=None, ret_day=None,
                     fc: float = 0.0, days_per_year: float = 252.0, rescale: bool = False,
                     want_end: bool = False):
    """Float each period's weights over its panel rows on the device (pq_simulate_periods;
    Strategy.simulate / floating_weights / Portfolio.turnover, src/portfolio.py:111-123,
    209-296).  ``panel`` (rows x n) and ``W`` (periods x n) are FP64 device tensors;
    ``plan`` is a PeriodPlan (or the row0 array, with ``nrows`` / ``ret_day`` given).
    Returns (ret [sum(nrows - 1)], wend [periods x n] or None, turnover [periods] or None),
    all on the device."""
    dev = panel.device
    nper, n = int(W.shape[0]), int(W.shape[1])
    if panel.dtype != F64 or W.dtype != F64 or panel.dim() != 2 or panel.shape[1] != n:
        raise ValueError("simulate_periods: FP64 panel (rows x n) and W (periods x n) expected")
    if not isinstance(plan, PeriodPlan):
        plan = PeriodPlan(plan, nrows, ret_day, dev, panel_rows=panel.shape[0])
    if plan.nper != nper or plan.rows_end > panel.shape[0]:
        raise ValueError("simulate_periods: plan does not match the weights / panel")
    if fc != 0.0 and plan.ret_day is None:
        raise ValueError("simulate_periods: fc needs one calendar day per return")
    if panel.stride(1) != 1:
        panel = panel.contiguous()
    if W.stride(1) != 1:
        W = W.contiguous()
    total = plan.total
    ret = torch.empty(max(total, 1), dtype=F64, device=dev)
    wend = torch.empty((nper, n), dtype=F64, device=dev) if want_end else None
    to = torch.empty(max(nper, 1), dtype=F64, device=dev) if want_end else None
    _lib.check(_lib.load().pq_simulate_periods(
        _ptr(panel), panel.stride(0), n, _ptr(W), W.stride(0), _ptr(plan.row0), _ptr(plan.nrows), nper,
        _ptr(plan.off), _ptr(plan.ret_day), float(fc), float(days_per_year), _ptr(ret), _ptr(wend),
        n, _ptr(to), int(bool(rescale)), _stream()), "pq_simulate_periods")
    return ret[:total], wend, (to[:nper] if to is not None else None)
