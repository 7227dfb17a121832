// K3: batched OSQP-style ADMM, one 512-thread workgroup per QP, iterations inside the
// kernel with per-problem convergence (a converged problem's workgroup simply exits).
//
// Per iteration the only O(n^2) work is x~ = K^-1 rhs.  K^-1 is symmetric, so only its
// lower triangle (8 B x n(n+1)/2) is streamed from HBM, once per iteration, with 16-byte
// coalesced loads: wave w takes rows j = w (mod 8); row j adds K[j][c] rhs[j] to x~[c]
// for c < j in register accumulators (lane l owns columns 128 q + 2 l, 2 l + 1) and
// sum_{c<=j} K[j][c] rhs[c] to x~[j] through one wave reduction.  The eight partial
// vectors are combined by a fixed-order LDS tree (bit-reproducible).  Everything else is
// O(n + mg n) and lives in LDS: x, Px, z, y, rhs, q, bounds.
//
// P x is never formed with another mat-vec: K x~ = rhs gives P x~ = rhs - sigma x~ -
// C'R C x~, and P x_{k+1} = alpha P x~ + (1 - alpha) P x_k, so the OSQP residuals and
// the adaptive-rho estimate are evaluated every iteration for O(n).
//
// Replaces qpsolvers.solve_problem(...) (src/qp_problems.py:211-214) for the dense QPs
// PorQua builds in Optimization.model_qpsolvers (src/optimization.py:91-143).
#include "common.h"
#include "capi_util.h"

namespace pq {

constexpr int AT = 512;   // threads per ADMM workgroup
constexpr int AW = AT / 64;

// Optional per-phase timing (build with -DPQ_PROFILE): wall-clock ticks per phase summed
// over iterations, added into doubles [16, 24) after each problem's polish work layout.
struct PhaseClock {
#ifdef PQ_PROFILE
  long long a[8];
  long long t;
  __device__ void init() {
    for (int i = 0; i < 8; ++i) a[i] = 0;
    t = wall_clock64();
  }
  __device__ void stamp(int k) {
    __syncthreads();
    if (threadIdx.x == 0) {
      const long long now = wall_clock64();
      a[k] += now - t;
      t = now;
    }
  }
  __device__ void flush(double* dst) {
    if (threadIdx.x == 0)
      for (int i = 0; i < 8; ++i) dst[i] += (double)a[i];
  }
#else
  __device__ void init() {}
  __device__ void stamp(int) {}
  __device__ void flush(double*) {}
#endif
};

__device__ __forceinline__ double rho_row(double l, double u, double rho, const pq_settings& s) {
  if (l == u) return rho * s.eq_scale;
  if (isinf(l) && isinf(u)) return s.rho_min;
  return rho;
}

// multi-value workgroup max: v[0..NV) per thread -> out[0..NV) for every thread
template <int NV>
__device__ __forceinline__ void block_maxv(double (&v)[NV], double* red) {
#pragma unroll
  for (int k = 0; k < NV; ++k) v[k] = wave_max(v[k]);
  __syncthreads();
  if (lane_id() == 0) {
#pragma unroll
    for (int k = 0; k < NV; ++k) red[k * AW + wave_id()] = v[k];
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    double m = red[k * AW];
    for (int w = 1; w < AW; ++w) m = fmax(m, red[k * AW + w]);
    v[k] = m;
  }
}

// dot products of the mg general rows with an LDS vector: out[r] = Cg[r] . v
__device__ void rows_dot(const double* Cg, int64_t ld, int mg, int n, const double* v, double* out) {
  const int w = wave_id(), l = lane_id();
  for (int r = w; r < mg; r += AW) {
    const double* c = Cg + (int64_t)r * ld;
    double s = 0.0;
    for (int i = l; i < n; i += 64) s += c[i] * v[i];
    s = wave_sum(s);
    if (l == 0) out[r] = s;
  }
}

// fixed-order combination of the AW waves' register vectors into wave 0's acc:
// waves 4-7 -> 0-3 -> 0-1 -> 0 through LDS (tree: 4 * NQ*128 doubles)
template <int NQ>
__device__ __forceinline__ void tree_reduce(double2 (&acc)[NQ], double* tree) {
  constexpr int LM = NQ * 128;
  const int w = wave_id(), l = lane_id();
#pragma unroll
  for (int half = AW / 2; half >= 1; half >>= 1) {
    if (w >= half && w < 2 * half) {
      double2* dst = reinterpret_cast<double2*>(tree + (w - half) * LM) + l;
#pragma unroll
      for (int qq = 0; qq < NQ; ++qq) dst[64 * qq] = acc[qq];
    }
    __syncthreads();
    if (w < half) {
      const double2* src = reinterpret_cast<const double2*>(tree + w * LM) + l;
#pragma unroll
      for (int qq = 0; qq < NQ; ++qq) {
        const double2 vv = src[64 * qq];
        acc[qq].x += vv.x;
        acc[qq].y += vv.y;
      }
    }
    __syncthreads();
  }
}

// y = A v for a symmetric A of which only the lower triangle (rows j < n, leading
// dimension ld) is read: row j adds A[j][c] v[j] to y[c] for c < j (axpy, register
// accumulators; lane l owns columns 128 q + 2 l, 2 l + 1) and sum_{c<=j} A[j][c] v[c] to
// y[j] (one wave reduction per row).  Partial vectors of the AW waves are combined by a
// fixed-order LDS tree (bit-reproducible).  v, y, dotv: LDS, >= NQ*128 entries (v zero
// beyond n); tree: 4 * NQ*128 doubles.  RU rows per wave are in flight at a time (their
// loads are issued together; the accumulation order is fixed).  All threads must call.
template <int NQ, int RU>
PQ_DEVFN void symv_lower(const double* A, int64_t ld, int n, const double* v, double* y,
                           double* dotv, double* tree) {
  const int w = wave_id(), l = lane_id();
  double2 acc[NQ];
  double2 rv[NQ];
#pragma unroll
  for (int qq = 0; qq < NQ; ++qq) {
    acc[qq] = double2{0.0, 0.0};
    rv[qq] = reinterpret_cast<const double2*>(v)[64 * qq + l];
  }
  // process RU rows j0, j0 + AW, ... (rows >= n are skipped)
  auto rows = [&](int j0) {
    double2 r[RU][NQ];
#pragma unroll
    for (int u = 0; u < RU; ++u) {
      const int j = j0 + u * AW;
      const double2* rp = reinterpret_cast<const double2*>(A + (int64_t)(j < n ? j : 0) * ld) + l;
#pragma unroll
      for (int qq = 0; qq < NQ; ++qq) {
        const int c = 128 * qq + 2 * l;
        r[u][qq] = (j < n && c <= j) ? rp[64 * qq] : double2{0.0, 0.0};
      }
    }
    double d[RU];
#pragma unroll
    for (int u = 0; u < RU; ++u) {
      const int j = j0 + u * AW;
      const double a = j < n ? v[j] : 0.0;
      double s = 0.0;
#pragma unroll
      for (int qq = 0; qq < NQ; ++qq) {
        const int c = 128 * qq + 2 * l;
        const double yy = (c + 1 <= j) ? r[u][qq].y : 0.0;
        s = fma(r[u][qq].x, rv[qq].x, fma(yy, rv[qq].y, s));
        acc[qq].x = fma(a, (c < j) ? r[u][qq].x : 0.0, acc[qq].x);
        acc[qq].y = fma(a, (c + 1 < j) ? yy : 0.0, acc[qq].y);
      }
      d[u] = s;
    }
#pragma unroll
    for (int u = 0; u < RU; ++u) d[u] = wave_sum(d[u]);
    if (l == 0) {
#pragma unroll
      for (int u = 0; u < RU; ++u)
        if (j0 + u * AW < n) dotv[j0 + u * AW] = d[u];
    }
  };
  for (int j0 = w; j0 < n; j0 += RU * AW) rows(j0);
  tree_reduce<NQ>(acc, tree);
  if (w == 0) {
    double2* dst = reinterpret_cast<double2*>(y) + l;
    const double2* dv = reinterpret_cast<const double2*>(dotv) + l;
#pragma unroll
    for (int qq = 0; qq < NQ; ++qq) {
      const int c = 128 * qq + 2 * l;
      const double2 d = dv[64 * qq];
      dst[64 * qq] = double2{c < n ? acc[qq].x + d.x : 0.0, c + 1 < n ? acc[qq].y + d.y : 0.0};
    }
  }
  __syncthreads();
}

// Low-rank x~ = K^-1 rhs with K = D + U'U (see include/porqua_hip.h, pq_lowrank):
//   v = D^-1 rhs;  w = U v (T window-row dots + mg general rows);  u = M^-1 w (lower
//   symv);  x~ = v - D^-1 U' u (one axpy pass over the window rows).
// The window rows are read straight from the shared panel (2 passes per iteration).
template <int NQ, int NQK>
__device__ void lr_apply(const pq_lowrank& lr, int b, const pq_problem& pb, const pq_settings& s,
                         double rho, const double* rhs, double* xt, double* vv, double* kw,
                         double* ku, double* kdot, double* tree, double* red, const double* lo,
                         const double* up, const double* rg, const double* Cg, const double* Minv,
                         int k_ld, PhaseClock& pc) {
  constexpr int LDMAX = NQ * 128;
  constexpr int KMAX = NQK * 128;
  const int n = pb.n, ld = pb.ld, mg = pb.mg;
  const int t = threadIdx.x, w = wave_id(), l = lane_id();
  const bool has_box = pb.lb != nullptr;
  const double ps = (pb.p_scale ? pb.p_scale[b] : 1.0) * (lr.w_scale ? lr.w_scale[b] : 1.0);
  const double pd = pb.p_diag ? pb.p_diag[b] : 0.0;
  const double sps = sqrt(fmax(ps, 0.0));
  const int T = lr.tlen[b], tmax = lr.tmax, k = tmax + mg;
  const int32_t* rws = lr.rows + (int64_t)b * tmax;
  const double* mu = lr.mu ? lr.mu + (int64_t)b * lr.mu_stride : nullptr;
  const bool vec2 = (lr.ldp & 1) == 0;
  // (1) v = D^-1 rhs
  for (int i = t; i < LDMAX; i += AT) {
    double d = 0.0;
    if (i < n) d = rhs[i] / (s.sigma + pd + (has_box ? rho_row(lo[i], up[i], rho, s) : 0.0));
    vv[i] = d;
  }
  __syncthreads();
  double muv = 0.0;
  if (mu) {
    double a = 0.0;
    for (int i = t; i < n; i += AT) a += mu[i] * vv[i];
    muv = block_sum(a, red);
  }
  pc.stamp(1);
  // (2) w = U v: RU window rows per wave in flight (16-B loads, v in registers)
  constexpr int RU = 3;
  if (vec2) {
    double2 vr[NQ];
#pragma unroll
    for (int qq = 0; qq < NQ; ++qq) vr[qq] = reinterpret_cast<const double2*>(vv)[64 * qq + l];
    for (int t0 = w; t0 < tmax; t0 += RU * AW) {
      double2 r[RU][NQ];
#pragma unroll
      for (int u = 0; u < RU; ++u) {
        const int tt = t0 + u * AW;
        const int64_t ri = tt < T ? (int64_t)rws[tt] : 0;
        const double2* rp = reinterpret_cast<const double2*>(lr.panel + ri * lr.ldp) + l;
#pragma unroll
        for (int qq = 0; qq < NQ; ++qq)
          r[u][qq] = (tt < T && 128 * qq + 2 * l < n) ? rp[64 * qq] : double2{0.0, 0.0};
      }
      double d[RU];
#pragma unroll
      for (int u = 0; u < RU; ++u) {
        double s0 = 0.0;
#pragma unroll
        for (int qq = 0; qq < NQ; ++qq) s0 = fma(r[u][qq].x, vr[qq].x, fma(r[u][qq].y, vr[qq].y, s0));
        d[u] = s0;
      }
#pragma unroll
      for (int u = 0; u < RU; ++u) d[u] = wave_sum(d[u]);
      if (l == 0) {
#pragma unroll
        for (int u = 0; u < RU; ++u) {
          const int tt = t0 + u * AW;
          if (tt < tmax) kw[tt] = (tt < T) ? sps * (d[u] - muv) : 0.0;
        }
      }
    }
  } else {
    for (int tt = w; tt < tmax; tt += AW) {
      double d = 0.0;
      if (tt < T) {
        const double* row = lr.panel + (int64_t)rws[tt] * lr.ldp;
        for (int c = l; c < n; c += 64) d = fma(row[c], vv[c], d);
        d = wave_sum(d);
      }
      if (l == 0) kw[tt] = (tt < T) ? sps * (d - muv) : 0.0;
    }
  }
  for (int r = w; r < mg; r += AW) {
    const double* c = Cg + (int64_t)r * ld;
    double d = 0.0;
    for (int i = l; i < n; i += 64) d = fma(c[i], vv[i], d);
    d = wave_sum(d);
    if (l == 0) kw[tmax + r] = sqrt(rg[r]) * d;
  }
  for (int i = k + t; i < KMAX; i += AT) kw[i] = 0.0;
  __syncthreads();
  pc.stamp(2);
  // (3) u = M^-1 w
  symv_lower<NQK, 4>(Minv, k_ld, k, kw, ku, kdot, tree);
  pc.stamp(3);
  // (4) x~ = v - D^-1 U' u
  double su = 0.0;
  if (mu) {
    double a = 0.0;
    for (int tt = t; tt < T; tt += AT) a += ku[tt];
    su = block_sum(a, red);
  }
  double2 acc[NQ];
#pragma unroll
  for (int qq = 0; qq < NQ; ++qq) acc[qq] = double2{0.0, 0.0};
  if (vec2) {
    for (int t0 = w; t0 < T; t0 += RU * AW) {
      double2 r[RU][NQ];
      double a[RU];
#pragma unroll
      for (int u = 0; u < RU; ++u) {
        const int tt = t0 + u * AW;
        const int64_t ri = tt < T ? (int64_t)rws[tt] : 0;
        a[u] = tt < T ? ku[tt] : 0.0;
        const double2* rp = reinterpret_cast<const double2*>(lr.panel + ri * lr.ldp) + l;
#pragma unroll
        for (int qq = 0; qq < NQ; ++qq)
          r[u][qq] = (tt < T && 128 * qq + 2 * l < n) ? rp[64 * qq] : double2{0.0, 0.0};
      }
#pragma unroll
      for (int u = 0; u < RU; ++u)
#pragma unroll
        for (int qq = 0; qq < NQ; ++qq) {
          acc[qq].x = fma(a[u], r[u][qq].x, acc[qq].x);
          acc[qq].y = fma(a[u], r[u][qq].y, acc[qq].y);
        }
    }
  } else {
    for (int tt = w; tt < T; tt += AW) {
      const double a = ku[tt];
      const double* row = lr.panel + (int64_t)rws[tt] * lr.ldp;
#pragma unroll
      for (int qq = 0; qq < NQ; ++qq) {
        const int c = 128 * qq + 2 * l;
        if (c < n) acc[qq].x = fma(a, row[c], acc[qq].x);
        if (c + 1 < n) acc[qq].y = fma(a, row[c + 1], acc[qq].y);
      }
    }
  }
  tree_reduce<NQ>(acc, tree);
  if (w == 0) {
    double2* dst = reinterpret_cast<double2*>(xt) + l;
#pragma unroll
    for (int qq = 0; qq < NQ; ++qq) dst[64 * qq] = acc[qq];
  }
  __syncthreads();
  for (int i = t; i < n; i += AT) {
    double corr = sps * (xt[i] - (mu ? su * mu[i] : 0.0));
    for (int r = 0; r < mg; ++r) corr = fma(sqrt(rg[r]) * ku[tmax + r], Cg[(int64_t)r * ld + i], corr);
    const double D = s.sigma + pd + (has_box ? rho_row(lo[i], up[i], rho, s) : 0.0);
    xt[i] = vv[i] - corr / D;
  }
  __syncthreads();
  pc.stamp(4);
}

// Grid position -> problem slot so that the blocks sharing an XCD (g = x mod 8) take a
// contiguous range of dates: neighbouring windows overlap in T-1 rows, so the low-rank
// kernels then find the panel rows in that XCD's L2 (speed only, bijective for any N).
template <int NQ, int NQK, int MODE>
__global__ __launch_bounds__(AT) void k_admm(pq_problem pb, pq_state st, const int32_t* idx,
                                             int nidx, pq_settings s, int iters_call, pq_lowrank lr,
                                             const double* Minv_all, int k_ld, int64_t M_stride) {
  constexpr int LDMAX = NQ * 128;
  constexpr int KMAX = NQK * 128;
  __shared__ __attribute__((aligned(16))) double sm[10 * LDMAX + 4 * LDMAX + 8 * 64 + 16 * AW + 3 * KMAX];
  double* x = sm;
  double* Px = x + LDMAX;
  double* zb = Px + LDMAX;
  double* yb = zb + LDMAX;
  double* q = yb + LDMAX;
  double* rhs = q + LDMAX;
  double* xt = rhs + LDMAX;
  double* lo = xt + LDMAX;
  double* up = lo + LDMAX;
  double* dotv = up + LDMAX;       // per-row dot products of the lower-triangle mat-vec
  double* tree = dotv + LDMAX;     // 4 * LDMAX partial-vector scratch
  double* zg = tree + 4 * LDMAX;   // mg <= 64 each
  double* yg = zg + 64;
  double* rg = yg + 64;
  double* wg = rg + 64;            // rho z - y for the general rows
  double* ztg = wg + 64;
  double* cgx = ztg + 64;
  double* lgs = cgx + 64;
  double* ugs = lgs + 64;
  double* red = ugs + 64;          // 16 * AW
  double* kw = red + 16 * AW;      // low-rank: U D^-1 rhs (k)
  double* ku = kw + KMAX;          // low-rank: M^-1 kw
  double* kdot = ku + KMAX;        // low-rank: symv scratch

  const int gslot = MODE == 1 ? xcd_slot(blockIdx.x, gridDim.x) : (int)blockIdx.x;
  const int b = idx ? idx[gslot] : gslot;
  if (st.status[b] != PQ_UNSOLVED && st.status[b] != PQ_NEED_REFACTOR) return;
  const int n = pb.n, ld = pb.ld, mg = pb.mg;
  const int t = threadIdx.x, w = wave_id(), l = lane_id();
  const double* Kinv = st.K + (int64_t)b * st.K_stride;
  const double* Cg = pb.Cg ? pb.Cg + (int64_t)b * pb.Cg_stride : nullptr;
  const bool has_box = pb.lb != nullptr;
  double rho = st.rho[b];
  const double sigma = s.sigma, alpha = s.alpha;

  // ---- load state -----------------------------------------------------------------
  {
    const double* gq = pb.q + (int64_t)b * pb.q_stride;
    const double* gx = st.x + (int64_t)b * ld;
    const double* gpx = st.Px + (int64_t)b * ld;
    const double* gz = st.z + (int64_t)b * st.m_ld + st.mg_pad;
    const double* gy = st.y + (int64_t)b * st.m_ld + st.mg_pad;
    const double* glb = has_box ? pb.lb + (int64_t)b * pb.box_stride : nullptr;
    const double* gub = has_box ? pb.ub + (int64_t)b * pb.box_stride : nullptr;
    for (int i = t; i < LDMAX; i += AT) {
      const bool v = i < n;
      x[i] = v ? gx[i] : 0.0;
      Px[i] = v ? gpx[i] : 0.0;
      zb[i] = v && has_box ? gz[i] : 0.0;
      yb[i] = v && has_box ? gy[i] : 0.0;
      q[i] = v ? gq[i] : 0.0;
      lo[i] = v && has_box ? glb[i] : -INFINITY;
      up[i] = v && has_box ? gub[i] : INFINITY;
    }
    if (t < mg) {
      const double* gzg = st.z + (int64_t)b * st.m_ld;
      const double* gyg = st.y + (int64_t)b * st.m_ld;
      const double lgv = pb.lg[(int64_t)b * pb.g_stride + t];
      const double ugv = pb.ug[(int64_t)b * pb.g_stride + t];
      zg[t] = gzg[t];
      yg[t] = gyg[t];
      lgs[t] = lgv;
      ugs[t] = ugv;
      rg[t] = rho_row(lgv, ugv, rho, s);
    }
  }
  __syncthreads();
  if (mg) rows_dot(Cg, ld, mg, n, x, cgx);
  __syncthreads();

  int it = st.iters[b];
  int status = PQ_UNSOLVED;
  const int it_end = min(s.max_iter, it + iters_call);
  PhaseClock pc;
  pc.init();
  while (it < it_end) {
    ++it;
    // ---- rhs = sigma x - q + C'(R z - y) ------------------------------------------
    if (t < mg) wg[t] = rg[t] * zg[t] - yg[t];
    __syncthreads();
    for (int i = t; i < n; i += AT) {
      double r = sigma * x[i] - q[i];
      if (has_box) r += rho_row(lo[i], up[i], rho, s) * zb[i] - yb[i];
      for (int k = 0; k < mg; ++k) r += Cg[(int64_t)k * ld + i] * wg[k];
      rhs[i] = r;
    }
    for (int i = n + t; i < LDMAX; i += AT) rhs[i] = 0.0;
    __syncthreads();
    pc.stamp(0);
    if constexpr (MODE == 0) {
      symv_lower<NQ, 2>(Kinv, ld, n, rhs, xt, dotv, tree);
    } else {
      lr_apply<NQ, NQK>(lr, b, pb, s, rho, rhs, xt, dotv, kw, ku, kdot, tree, red, lo, up, rg, Cg,
                        Minv_all + (int64_t)b * M_stride, k_ld, pc);
    }
    // ---- z~ for the general rows ----------------------------------------------------
    if (mg) rows_dot(Cg, ld, mg, n, xt, ztg);
    __syncthreads();
    // ---- updates and residual terms --------------------------------------------------
    double mv[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    // mv: 0 |Cx - z|, 1 |Cx|, 2 |z|, 3 |Px + q + C'y|, 4 |Px|, 5 |C'y|, 6 |q|
    for (int i = t; i < n; i += AT) {
      const double xti = xt[i];
      double pxt = rhs[i] - sigma * xti;
      double rb = 0.0;
      if (has_box) {
        rb = rho_row(lo[i], up[i], rho, s);
        pxt -= rb * xti;
      }
      for (int k = 0; k < mg; ++k) pxt -= Cg[(int64_t)k * ld + i] * rg[k] * ztg[k];
      const double xn = alpha * xti + (1.0 - alpha) * x[i];
      const double pxn = alpha * pxt + (1.0 - alpha) * Px[i];
      x[i] = xn;
      Px[i] = pxn;
      double cty = 0.0;
      if (has_box) {
        const double zh = alpha * xti + (1.0 - alpha) * zb[i];
        const double zn = fmin(fmax(zh + yb[i] / rb, lo[i]), up[i]);
        const double yn = yb[i] + rb * (zh - zn);
        zb[i] = zn;
        yb[i] = yn;
        cty = yn;
        mv[0] = fmax(mv[0], fabs(xn - zn));
        mv[1] = fmax(mv[1], fabs(xn));
        mv[2] = fmax(mv[2], fabs(zn));
      }
      mv[4] = fmax(mv[4], fabs(pxn));
      mv[6] = fmax(mv[6], fabs(q[i]));
      // general-row part of C'y is added below once yg is updated
      rhs[i] = pxn + q[i] + cty;   // reuse rhs as the dual-residual accumulator
      xt[i] = cty;                 // reuse xt as C'y accumulator
    }
    __syncthreads();
    if (t < mg) {
      const double zh = alpha * ztg[t] + (1.0 - alpha) * zg[t];
      const double zn = fmin(fmax(zh + yg[t] / rg[t], lgs[t]), ugs[t]);
      yg[t] = yg[t] + rg[t] * (zh - zn);
      zg[t] = zn;
      cgx[t] = alpha * ztg[t] + (1.0 - alpha) * cgx[t];
    }
    __syncthreads();
    if (t < mg) {
      mv[0] = fmax(mv[0], fabs(cgx[t] - zg[t]));
      mv[1] = fmax(mv[1], fabs(cgx[t]));
      mv[2] = fmax(mv[2], fabs(zg[t]));
    }
    for (int i = t; i < n; i += AT) {
      double cy = xt[i];
      for (int k = 0; k < mg; ++k) cy += Cg[(int64_t)k * ld + i] * yg[k];
      const double dres = rhs[i] + (cy - xt[i]);
      mv[3] = fmax(mv[3], fabs(dres));
      mv[5] = fmax(mv[5], fabs(cy));
    }
    block_maxv<8>(mv, red);
    pc.stamp(5);
    const double eps_p = s.eps_abs + s.eps_rel * fmax(mv[1], mv[2]);
    const double eps_d = s.eps_abs + s.eps_rel * fmax(mv[4], fmax(mv[5], mv[6]));
    if (it >= s.min_iter && mv[0] <= eps_p && mv[3] <= eps_d) {
      status = PQ_SOLVED;
      break;
    }
    if (s.adapt_interval > 0 && it % s.adapt_interval == 0) {
      const double rp = mv[0] / (fmax(mv[1], mv[2]) + 1e-30);
      const double rd = mv[3] / (fmax(mv[4], fmax(mv[5], mv[6])) + 1e-30);
      double rn = rho * sqrt(rp / (rd + 1e-30));
      rn = fmin(fmax(rn, s.rho_min), s.rho_max);
      if (rn > rho * s.adapt_tol || rn < rho / s.adapt_tol) {
        rho = rn;
        status = PQ_NEED_REFACTOR;
        break;
      }
    }
    __syncthreads();
  }
  if (status == PQ_UNSOLVED && it >= s.max_iter) status = PQ_MAX_ITER;
  __syncthreads();
  pc.flush(st.work + (int64_t)b * st.work_stride + PQ_WORK_PROF(ld, st.mg_pad) + 16);
  // ---- save state --------------------------------------------------------------------
  {
    double* gx = st.x + (int64_t)b * ld;
    double* gpx = st.Px + (int64_t)b * ld;
    double* gz = st.z + (int64_t)b * st.m_ld;
    double* gy = st.y + (int64_t)b * st.m_ld;
    for (int i = t; i < n; i += AT) {
      gx[i] = x[i];
      gpx[i] = Px[i];
      if (has_box) {
        gz[st.mg_pad + i] = zb[i];
        gy[st.mg_pad + i] = yb[i];
      }
    }
    if (t < mg) {
      gz[t] = zg[t];
      gy[t] = yg[t];
    }
    if (t == 0) {
      st.iters[b] = it;
      st.status[b] = status;
      st.rho[b] = rho;
    }
  }
}

// dg: diag of the unscaled window Gram (pq_lowrank.dg) when P is given in window form
__global__ void k_init_state(pq_problem pb, pq_state st, const int32_t* idx, pq_settings s,
                             const double* dg, int64_t dg_stride, const double* w_scale) {
  const int b = idx ? idx[blockIdx.x] : (int)blockIdx.x;
  const int ld = pb.ld;
  for (int i = threadIdx.x; i < ld; i += blockDim.x) {
    st.x[(int64_t)b * ld + i] = 0.0;
    st.Px[(int64_t)b * ld + i] = 0.0;
  }
  for (int i = threadIdx.x; i < st.m_ld; i += blockDim.x) {
    st.z[(int64_t)b * st.m_ld + i] = 0.0;
    st.y[(int64_t)b * st.m_ld + i] = 0.0;
  }
  double rho0 = s.rho0;
  if (s.rho0_rel > 0.0) {
    __shared__ double red[16];
    const double* P = pb.P + (int64_t)b * pb.P_stride;
    const double ps = pb.p_scale ? pb.p_scale[b] : 1.0;
    const double pd = pb.p_diag ? pb.p_diag[b] : 0.0;
    double sdiag = 0.0;
    if (dg) {
      const double psw = ps * (w_scale ? w_scale[b] : 1.0);
      for (int i = threadIdx.x; i < pb.n; i += blockDim.x) sdiag += psw * dg[(int64_t)b * dg_stride + i] + pd;
    } else {
      for (int i = threadIdx.x; i < pb.n; i += blockDim.x) sdiag += ps * P[(int64_t)i * ld + i] + pd;
    }
    sdiag = block_sum(sdiag, red);
    const double md = sdiag / pb.n;
    rho0 = (md > 0.0 && isfinite(md)) ? fmin(fmax(s.rho0_rel * md, s.rho_min), s.rho_max) : s.rho0;
  }
  if (threadIdx.x == 0) {
    st.rho[b] = rho0;
    st.iters[b] = 0;
    st.status[b] = PQ_UNSOLVED;
    st.info[b] = 0;
    for (int k = 0; k < PQ_OUT_FIELDS; ++k) st.out[(int64_t)b * PQ_OUT_FIELDS + k] = 0.0;
  }
}

}  // namespace pq

extern "C" int pq_init_state(const pq_problem* pb, pq_state* st, const int32_t* idx, int32_t nidx,
                             const pq_settings* s, void* stream) {
  PQ_CHECK_ARG(pb && st && s, "pq_init_state: null argument");
  PQ_CHECK_ARG(st->x && st->Px && st->z && st->y && st->rho && st->iters && st->status &&
                   st->info && st->out, "pq_init_state: state buffers missing");
  PQ_CHECK_ARG(st->m_ld >= st->mg_pad + pb->ld && st->mg_pad >= pb->mg, "pq_init_state: bad m_ld / mg_pad");
  const int grid = idx ? nidx : pb->batch;
  if (grid <= 0) return 0;
  PQ_CHECK_ARG(pb->P || s->rho0_rel <= 0.0, "pq_init_state: rho0_rel > 0 needs P (pq_init_state_lr for the window form)");
  hipLaunchKernelGGL(pq::k_init_state, dim3(grid), dim3(256), 0, (hipStream_t)stream, *pb, *st, idx, *s,
                     nullptr, 0, nullptr);
  PQ_CHECK_LAUNCH("pq_init_state");
  return 0;
}

extern "C" int pq_init_state_lr(const pq_lowrank* lr, const pq_problem* pb, pq_state* st, const int32_t* idx,
                                int32_t nidx, const pq_settings* s, void* stream) {
  PQ_CHECK_ARG(lr && pb && st && s, "pq_init_state_lr: null argument");
  PQ_CHECK_ARG(lr->dg || s->rho0_rel <= 0.0, "pq_init_state_lr: rho0_rel > 0 needs lr->dg (pq_window_sumsq)");
  PQ_CHECK_ARG(st->x && st->Px && st->z && st->y && st->rho && st->iters && st->status &&
                   st->info && st->out, "pq_init_state_lr: state buffers missing");
  PQ_CHECK_ARG(st->m_ld >= st->mg_pad + pb->ld && st->mg_pad >= pb->mg, "pq_init_state_lr: bad m_ld / mg_pad");
  const int grid = idx ? nidx : pb->batch;
  if (grid <= 0) return 0;
  hipLaunchKernelGGL(pq::k_init_state, dim3(grid), dim3(256), 0, (hipStream_t)stream, *pb, *st, idx, *s,
                     lr->dg, lr->dg_stride, lr->w_scale);
  PQ_CHECK_LAUNCH("pq_init_state_lr");
  return 0;
}

extern "C" int pq_admm_batched(const pq_problem* pb, pq_state* st, const int32_t* idx, int32_t nidx,
                               const pq_settings* s, int32_t iters_this_call, void* stream) {
  PQ_CHECK_ARG(pb && st && s, "pq_admm_batched: null argument");
  PQ_CHECK_ARG(pb->ld % 128 == 0 || pb->ld % 64 == 0, "pq_admm_batched: bad ld");
  PQ_CHECK_ARG(pb->mg <= 64, "pq_admm_batched: mg must be <= 64");
  PQ_CHECK_ARG(pb->mg == 0 || (pb->Cg && pb->lg && pb->ug), "pq_admm_batched: Cg/lg/ug missing");
  const int grid = idx ? nidx : pb->batch;
  if (grid <= 0) return 0;
  const int nq = (pb->n + 127) / 128;
  hipStream_t str = (hipStream_t)stream;
  pq_lowrank nolr = {};
#define PQ_ADMM_CASE(NQV) \
  case NQV: hipLaunchKernelGGL((pq::k_admm<NQV, 1, 0>), dim3(grid), dim3(pq::AT), 0, str, *pb, *st, idx, nidx, *s, iters_this_call, nolr, nullptr, 0, 0); break;
  switch (nq) {
    PQ_ADMM_CASE(1)
    PQ_ADMM_CASE(2)
    PQ_ADMM_CASE(3)
    PQ_ADMM_CASE(4)
    PQ_ADMM_CASE(5)
    PQ_ADMM_CASE(6)
    PQ_ADMM_CASE(7)
    PQ_ADMM_CASE(8)
    default:
      pq::set_error("pq_admm_batched: n=%d exceeds the LDS-resident limit of 1024", pb->n);
      return -1;
  }
#undef PQ_ADMM_CASE
  PQ_CHECK_LAUNCH("pq_admm_batched");
  return 0;
}

extern "C" int pq_admm_lr_batched(const pq_lowrank* lr, const pq_problem* pb, pq_state* st,
                                  const double* Minv, int32_t k_ld, int64_t M_stride,
                                  const int32_t* idx, int32_t nidx, const pq_settings* s,
                                  int32_t iters_this_call, void* stream) {
  PQ_CHECK_ARG(lr && pb && st && s && Minv, "pq_admm_lr_batched: null argument");
  PQ_CHECK_ARG(lr->panel && lr->rows && lr->tlen && lr->tmax > 0, "pq_admm_lr_batched: window missing");
  PQ_CHECK_ARG(pb->mg <= 64 && (pb->mg == 0 || (pb->Cg && pb->lg && pb->ug)), "pq_admm_lr_batched: bad general rows");
  const int k = lr->tmax + pb->mg;
  PQ_CHECK_ARG(k_ld % 64 == 0 && k_ld >= k && k_ld <= 512, "pq_admm_lr_batched: need k <= k_ld <= 512 (k=%d k_ld=%d)", k, k_ld);
  const int grid = idx ? nidx : pb->batch;
  if (grid <= 0) return 0;
  const int nq = (pb->n + 127) / 128;
  const int nqk = (k_ld + 127) / 128;
  PQ_CHECK_ARG(nqk <= nq, "pq_admm_lr_batched: the low-rank form needs k <= n");
  hipStream_t str = (hipStream_t)stream;
#define PQ_LR_CASE(NQV, NQKV) \
  if (nq == NQV && nqk == NQKV) { hipLaunchKernelGGL((pq::k_admm<NQV, NQKV, 1>), dim3(grid), dim3(pq::AT), 0, str, *pb, *st, idx, nidx, *s, iters_this_call, *lr, Minv, k_ld, M_stride); PQ_CHECK_LAUNCH("pq_admm_lr_batched"); return 0; }
  PQ_LR_CASE(2, 1) PQ_LR_CASE(2, 2)
  PQ_LR_CASE(3, 1) PQ_LR_CASE(3, 2) PQ_LR_CASE(3, 3)
  PQ_LR_CASE(4, 1) PQ_LR_CASE(4, 2) PQ_LR_CASE(4, 3) PQ_LR_CASE(4, 4)
  PQ_LR_CASE(5, 1) PQ_LR_CASE(5, 2) PQ_LR_CASE(5, 3) PQ_LR_CASE(5, 4)
  PQ_LR_CASE(6, 1) PQ_LR_CASE(6, 2) PQ_LR_CASE(6, 3) PQ_LR_CASE(6, 4)
  PQ_LR_CASE(7, 1) PQ_LR_CASE(7, 2) PQ_LR_CASE(7, 3) PQ_LR_CASE(7, 4)
  PQ_LR_CASE(8, 1) PQ_LR_CASE(8, 2) PQ_LR_CASE(8, 3) PQ_LR_CASE(8, 4)
#undef PQ_LR_CASE
  pq::set_error("pq_admm_lr_batched: unsupported sizes n=%d k_ld=%d", pb->n, k_ld);
  return -1;
}
