// Low-rank K2: capacitance matrices M_b = I + U D^-1 U' of the Woodbury form of the ADMM
// system (include/porqua_hip.h, pq_lowrank), for windows with T + mg < n.
//
// U has k = tmax + mg rows: sqrt(p_scale) (X_t - mu) for the window rows of date b and
// sqrt(rho_r) Cg_r for the general constraint rows; D = sigma + p_diag + rho_box.  Each
// 256-thread workgroup computes one lower 64x64 tile of one M_b as an MFMA (f64
// 16x16x4) product contracted over the n assets in 16-column chunks; rows are gathered
// from the panel through the date's row list and scaled / centred / weighted by
// 1/sqrt(D_c) while they are staged into LDS.  2 k^2 n flop per date (k ~ 253, n = 1000:
// 1.3e8) instead of the n^3 of the dense KKT factorisation.
#include "common.h"
#include "capi_util.h"

namespace pq {

__device__ __forceinline__ double lr_rho(double l, double u, double rho, const pq_settings& s) {
  if (l == u) return rho * s.eq_scale;
  if (isinf(l) && isinf(u)) return s.rho_min;
  return rho;
}

struct URow {
  const double* src;   // nullptr: zero row
  const double* mu;    // centring (window rows only)
  double scale;
};

__device__ __forceinline__ URow urow(const pq_lowrank& lr, const pq_problem& pb, int b, int gi,
                                     double sps, double rho, const pq_settings& s) {
  URow r{nullptr, nullptr, 0.0};
  const int T = lr.tlen[b];
  if (gi < lr.tmax) {
    if (gi < T) {
      r.src = lr.panel + (int64_t)lr.rows[(int64_t)b * lr.tmax + gi] * lr.ldp;
      r.mu = lr.mu ? lr.mu + (int64_t)b * lr.mu_stride : nullptr;
      r.scale = sps;
    }
  } else if (gi < lr.tmax + pb.mg) {
    const int k = gi - lr.tmax;
    const double l = pb.lg[(int64_t)b * pb.g_stride + k], u = pb.ug[(int64_t)b * pb.g_stride + k];
    r.src = pb.Cg + (int64_t)b * pb.Cg_stride + (int64_t)k * pb.ld;
    r.scale = sqrt(lr_rho(l, u, rho, s));
  }
  return r;
}

__device__ __forceinline__ void load_u(double (&v)[4], const URow& r, int c0, int n,
                                       const double* wD) {
  const int cc = (threadIdx.x & 3) * 4;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int c = c0 + cc + e;
    double x = 0.0;
    if (r.src && c < n) {
      x = r.src[c];
      if (r.mu) x -= r.mu[c];
      x *= r.scale * wD[cc + e];
    }
    v[e] = x;
  }
}

__device__ __forceinline__ void store_u(const double (&v)[4], double* S) {
  const int i = threadIdx.x >> 2, cc = (threadIdx.x & 3) * 4;
#pragma unroll
  for (int e = 0; e < 4; ++e) S[(cc + e) * LDW + i] = v[e];
}

__device__ __forceinline__ int tri_row(int t) {
  int I = (int)((sqrt(8.0 * t + 1.0) - 1.0) * 0.5);
  while ((I + 1) * (I + 2) / 2 <= t) ++I;
  while (I * (I + 1) / 2 > t) --I;
  return I;
}

__global__ __launch_bounds__(256) void k_lr_gram(pq_lowrank lr, pq_problem pb, const double* rho_all,
                                                 const int32_t* idx, pq_settings s, double* M_all,
                                                 int k_ld, int64_t M_stride) {
  __shared__ __attribute__((aligned(16))) double smem[4 * STAGE + 2 * KC];
  double* wD = smem + 4 * STAGE;   // 1/sqrt(D_c) of the current (and next) column chunk
  const int b = idx ? idx[blockIdx.y] : (int)blockIdx.y;
  const int I = tri_row(blockIdx.x), J = blockIdx.x - I * (I + 1) / 2;
  const int n = pb.n;
  const double rho = rho_all[b];
  const double ps = (pb.p_scale ? pb.p_scale[b] : 1.0) * (lr.w_scale ? lr.w_scale[b] : 1.0);
  const double pd = pb.p_diag ? pb.p_diag[b] : 0.0;
  const double sps = sqrt(fmax(ps, 0.0));
  const double* lb = pb.lb ? pb.lb + (int64_t)b * pb.box_stride : nullptr;
  const double* ub = pb.ub ? pb.ub + (int64_t)b * pb.box_stride : nullptr;
  const int i = threadIdx.x >> 2;
  const URow ra = urow(lr, pb, b, I * TB + i, sps, rho, s);
  const URow rb = urow(lr, pb, b, J * TB + i, sps, rho, s);
  auto weights = [&](int c0, double* dst) {
    if (threadIdx.x < KC) {
      const int c = c0 + threadIdx.x;
      double d = s.sigma + pd;
      if (lb && c < n) d += lr_rho(lb[c], ub[c], rho, s);
      dst[threadIdx.x] = c < n ? 1.0 / sqrt(d) : 0.0;
    }
  };
  Acc acc;
  acc.zero();
  double va[4], vb[4];
  weights(0, wD);
  __syncthreads();
  load_u(va, ra, 0, n, wD);
  load_u(vb, rb, 0, n, wD);
  store_u(va, smem);
  store_u(vb, smem + STAGE);
  __syncthreads();
  int buf = 0;
  for (int c0 = 0; c0 < n; c0 += KC) {
    const bool more = c0 + KC < n;
    double* wn = wD + ((c0 / KC + 1) & 1) * KC;
    if (more) weights(c0 + KC, wn);
    __syncthreads();
    if (more) {
      load_u(va, ra, c0 + KC, n, wn);
      load_u(vb, rb, c0 + KC, n, wn);
    }
    mma_lds(acc, smem + buf * 2 * STAGE, smem + buf * 2 * STAGE + STAGE, KC);
    if (more) {
      store_u(va, smem + (buf ^ 1) * 2 * STAGE);
      store_u(vb, smem + (buf ^ 1) * 2 * STAGE + STAGE);
    }
    __syncthreads();
    buf ^= 1;
  }
  double* M = M_all + (int64_t)b * M_stride;
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int nn = 0; nn < 2; ++nn)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int gi = I * TB + acc_row(m, r), gj = J * TB + acc_col(nn);
        M[(int64_t)gi * k_ld + gj] = acc.c[m][nn][r] + (gi == gj ? 1.0 : 0.0);
      }
}

// ---- band Gram path (uniform D): M from the panel's row-by-row Gram ----------------------
//
// When D = c I (every box row has the same rho: all finite distinct bounds, or all free,
// or all fixed), M = I + U U' / c needs only inner products of panel ROWS: consecutive
// windows share T - 1 rows, so the products x_r . x_r' with 0 <= r - r' < W (W = widest
// window span) are formed once per backtest -- k_band_gram, an MFMA SYRK over the
// assets -- instead of T^2 n per date.  Centring uses the window's own mean:
//   Xc Xc' = B - r 1' - 1 r' + s 11',  r_a = (1/T) sum_b B_ab,  s = (1/T) sum_a r_a,
// which needs mu == the mean of exactly the window's rows (pq_window_mean), or mu == NULL.
// The general rows enter through PC[r][g] = x_r . Cg_g (shared Cg) and CC = Cg Cg'.

__global__ __launch_bounds__(256) void k_band_gram(const double* panel, int64_t ldp, int n, int r0,
                                                   int nrows, int W, int JB, double* out, int64_t ldo) {
  __shared__ __attribute__((aligned(16))) double smem[4 * STAGE];
  const int I = blockIdx.x / JB, Jd = blockIdx.x % JB;
  const int J = I - Jd;
  if (J < 0 || TB * Jd - (TB - 1) >= W) return;   // uniform: no lag of this tile in [0, W)
  const int t = threadIdx.x, i = t >> 2, cc = (t & 3) * 4;
  const int ra = I * TB + i, rb = J * TB + i;
  // unconditional loads from clamped rows / columns, zeroed when staged, and a ring of four
  // chunks in registers: each chunk's loads are issued four chunks ahead of its MFMAs (one
  // chunk ahead under lane conditions waited for every load, a round trip per 16 columns)
  const bool aok = ra < nrows, bok = rb < nrows;
  const double* pa = panel + (int64_t)(r0 + (aok ? ra : 0)) * ldp;
  const double* pq_ = panel + (int64_t)(r0 + (bok ? rb : 0)) * ldp;
  auto load = [&](double (&v)[4], const double* p, int c0) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int c = c0 + cc + e;
      v[e] = p[c < n ? c : 0];
    }
  };
  auto store = [&](const double (&v)[4], double* S, bool ok, int c0) {
#pragma unroll
    for (int e = 0; e < 4; ++e) S[(cc + e) * LDW + i] = (ok && c0 + cc + e < n) ? v[e] : 0.0;
  };
  constexpr int D = 4;
  const int nc = (n + KC - 1) / KC;
  Acc acc;
  acc.zero();
  double va[D][4], vb[D][4];
  load(va[0], pa, 0);
  load(vb[0], pq_, 0);
#pragma unroll
  for (int s2 = 1; s2 < D; ++s2)
    if (s2 < nc) {   // (uniform)
      load(va[s2], pa, s2 * KC);
      load(vb[s2], pq_, s2 * KC);
    }
  store(va[0], smem, aok, 0);
  store(vb[0], smem + STAGE, bok, 0);
  if (D < nc) {
    load(va[0], pa, D * KC);
    load(vb[0], pq_, D * KC);
  }
  __syncthreads();
  int buf = 0;
  for (int c = 0; c < nc; c += D) {
#pragma unroll
    for (int s2 = 0; s2 < D; ++s2) {
      const int cur = c + s2;
      if (cur >= nc) break;   // (uniform)
      mma_lds(acc, smem + buf * 2 * STAGE, smem + buf * 2 * STAGE + STAGE, KC);
      const int nx = cur + 1;   // chunk nx lives in slot nx % D = (s2 + 1) % D
      if (nx < nc) {
        store(va[(s2 + 1) % D], smem + (buf ^ 1) * 2 * STAGE, aok, nx * KC);
        store(vb[(s2 + 1) % D], smem + (buf ^ 1) * 2 * STAGE + STAGE, bok, nx * KC);
        if (nx + D < nc) {   // refill the slot with chunk nx + D
          load(va[(s2 + 1) % D], pa, (nx + D) * KC);
          load(vb[(s2 + 1) % D], pq_, (nx + D) * KC);
        }
      }
      __syncthreads();
      buf ^= 1;
    }
  }
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int nn = 0; nn < 2; ++nn)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int gr = I * TB + acc_row(m, r), gc = J * TB + acc_col(nn);
        const int lag = gr - gc;
        if (gr < nrows && lag >= 0 && lag < W) out[(int64_t)gr * ldo + lag] = acc.c[m][nn][r];
      }
}

// PC[r][g] = x_{r0 + r} . Cg_g : one wave per panel row
__global__ __launch_bounds__(64) void k_panel_cg(const double* panel, int64_t ldp, int n, int r0, int nrows,
                                                 const double* Cg, int mg, int ld_cg, double* pc, int64_t ldpc) {
  const int r = blockIdx.x, l = threadIdx.x;
  if (r >= nrows) return;
  const double* x = panel + (int64_t)(r0 + r) * ldp;
  for (int g = 0; g < mg; ++g) {
    double a = 0.0;
    for (int c = l; c < n; c += 64) a = fma(x[c], Cg[(int64_t)g * ld_cg + c], a);
    a = wave_sum(a);
    if (l == 0) pc[(int64_t)r * ldpc + g] = a;
  }
}

// M (lower 64x64 tiles, diagonal tiles in full) of one date per 256-thread workgroup
__global__ __launch_bounds__(256) void k_lr_cap_band(pq_lowrank lr, pq_problem pb, const double* rho_all,
                                                     const int32_t* idx, pq_settings s, const double* band,
                                                     int64_t ldo, int r0, const double* pc, int64_t ldpc,
                                                     const double* cc, double* M_all, int k_ld, int64_t M_stride) {
  __shared__ int s_w[1024];
  __shared__ double s_r[1024];
  __shared__ double s_pcm[64], s_sr[64];
  __shared__ double red[16];
  const int slot = xcd_slot(blockIdx.x, gridDim.x);
  const int b = idx ? idx[slot] : slot;
  const int T = lr.tlen[b], tmax = lr.tmax, mg = pb.mg;
  const int t = threadIdx.x, w = wave_id(), l = lane_id();
  for (int a = t; a < T; a += 256) s_w[a] = lr.rows[(int64_t)b * tmax + a] - r0;
  __syncthreads();
  auto Bat = [&](int ia, int ib) -> double {
    int x = s_w[ia], y = s_w[ib];
    if (x < y) { const int z = x; x = y; y = z; }
    return band[(int64_t)x * ldo + (x - y)];
  };
  const bool cen = lr.mu != nullptr;
  double ss = 0.0;
  if (cen) {
    for (int a = w; a < T; a += 4) {
      double sum = 0.0;
      for (int bb = l; bb < T; bb += 64) sum += Bat(a, bb);
      sum = wave_sum(sum);
      if (l == 0) s_r[a] = sum / T;
    }
    for (int g = w; g < mg; g += 4) {
      double sum = 0.0;
      for (int a = l; a < T; a += 64) sum += pc[(int64_t)s_w[a] * ldpc + g];
      sum = wave_sum(sum);
      if (l == 0) s_pcm[g] = sum / T;
    }
    __syncthreads();
    double a0 = 0.0;
    for (int a = t; a < T; a += 256) a0 += s_r[a];
    ss = block_sum(a0, red) / T;
  } else {
    for (int a = t; a < T; a += 256) s_r[a] = 0.0;
    if (t < 64) s_pcm[t] = 0.0;
  }
  const double rho = rho_all[b];
  const double ps = (pb.p_scale ? pb.p_scale[b] : 1.0) * (lr.w_scale ? lr.w_scale[b] : 1.0);
  const double pd = pb.p_diag ? pb.p_diag[b] : 0.0;
  const double* lb = pb.lb ? pb.lb + (int64_t)b * pb.box_stride : nullptr;
  const double* ub = pb.ub ? pb.ub + (int64_t)b * pb.box_stride : nullptr;
  const double c = s.sigma + pd + (lb ? lr_rho(lb[0], ub[0], rho, s) : 0.0);   // uniform D (host-checked)
  const double a1 = ps / c, a2 = sqrt(fmax(ps, 0.0)) / c;
  if (t < mg) s_sr[t] = sqrt(lr_rho(pb.lg[(int64_t)b * pb.g_stride + t], pb.ug[(int64_t)b * pb.g_stride + t], rho, s));
  __syncthreads();
  double* M = M_all + (int64_t)b * M_stride;
  for (int i = w; i < k_ld; i += 4) {
    const int jend = (i / TB + 1) * TB;
    const bool icg = i >= tmax && i < tmax + mg;
    for (int j = l; j < jend; j += 64) {
      double v = (i == j) ? 1.0 : 0.0;
      const bool jcg = j >= tmax && j < tmax + mg;
      if (i < T && j < T) {
        v += a1 * (Bat(i, j) - s_r[i] - s_r[j] + ss);
      } else if (icg && j < T) {
        const int g = i - tmax;
        v += a2 * s_sr[g] * (pc[(int64_t)s_w[j] * ldpc + g] - s_pcm[g]);
      } else if (i < T && jcg) {   // upper part of a diagonal tile
        const int g = j - tmax;
        v += a2 * s_sr[g] * (pc[(int64_t)s_w[i] * ldpc + g] - s_pcm[g]);
      } else if (icg && jcg) {
        v += s_sr[i - tmax] * s_sr[j - tmax] / c * cc[(i - tmax) * mg + (j - tmax)];
      }
      M[(int64_t)i * k_ld + j] = v;
    }
  }
}

}  // namespace pq

extern "C" int pq_lr_band_gram(const double* panel, int64_t ldp, int32_t n, int32_t r0, int32_t nrows,
                               int32_t W, double* band, int64_t ldo, const double* Cg, int32_t mg,
                               int32_t ld_cg, double* pc, int64_t ldpc, void* stream) {
  PQ_CHECK_ARG(panel && band && nrows > 0 && W > 0 && n > 0 && ldo >= W, "pq_lr_band_gram: bad arguments");
  PQ_CHECK_ARG(mg == 0 || (Cg && pc && ldpc >= mg), "pq_lr_band_gram: general rows need Cg and pc");
  hipStream_t str = (hipStream_t)stream;
  const int nI = (nrows + 63) / 64;
  const int JB = (W + 62) / 64 + 1;
  hipLaunchKernelGGL(pq::k_band_gram, dim3(nI * JB), dim3(256), 0, str, panel, ldp, n, r0, nrows, W, JB, band, ldo);
  PQ_CHECK_LAUNCH("pq_lr_band_gram");
  if (mg > 0) {
    hipLaunchKernelGGL(pq::k_panel_cg, dim3(nrows), dim3(64), 0, str, panel, ldp, n, r0, nrows, Cg, mg, ld_cg,
                       pc, ldpc);
    PQ_CHECK_LAUNCH("pq_lr_band_gram (PC)");
  }
  return 0;
}

extern "C" int pq_lr_capacitance_band(const pq_lowrank* lr, const pq_problem* pb, const pq_state* st,
                                      const int32_t* idx, int32_t nidx, const pq_settings* s, const double* band,
                                      int64_t ldo, int32_t r0, const double* pc, int64_t ldpc, const double* cc,
                                      double* M, int32_t k_ld, int64_t M_stride, void* stream) {
  PQ_CHECK_ARG(lr && pb && st && s && M && band, "pq_lr_capacitance_band: null argument");
  PQ_CHECK_ARG(lr->rows && lr->tlen && lr->tmax > 0 && lr->tmax <= 1024, "pq_lr_capacitance_band: window missing or tmax > 1024");
  PQ_CHECK_ARG(pb->mg >= 0 && pb->mg <= 64 && (pb->mg == 0 || (pb->lg && pb->ug && pc && cc)),
               "pq_lr_capacitance_band: bad general rows");
  PQ_CHECK_ARG(k_ld % 64 == 0 && k_ld >= lr->tmax + pb->mg, "pq_lr_capacitance_band: k_ld too small");
  PQ_CHECK_ARG(st->rho != nullptr, "pq_lr_capacitance_band: rho missing");
  const int grid = idx ? nidx : pb->batch;
  if (grid <= 0) return 0;
  hipLaunchKernelGGL(pq::k_lr_cap_band, dim3(grid), dim3(256), 0, (hipStream_t)stream, *lr, *pb, st->rho, idx, *s,
                     band, ldo, r0, pc, ldpc, cc, M, k_ld, M_stride);
  PQ_CHECK_LAUNCH("pq_lr_capacitance_band");
  return 0;
}

extern "C" int pq_lr_capacitance(const pq_lowrank* lr, const pq_problem* pb, const pq_state* st,
                                 const int32_t* idx, int32_t nidx, const pq_settings* s, double* M,
                                 int32_t k_ld, int64_t M_stride, void* stream) {
  PQ_CHECK_ARG(lr && pb && st && s && M, "pq_lr_capacitance: null argument");
  PQ_CHECK_ARG(lr->panel && lr->rows && lr->tlen && lr->tmax > 0, "pq_lr_capacitance: window missing");
  PQ_CHECK_ARG(pb->mg >= 0 && pb->mg <= 64 && (pb->mg == 0 || (pb->Cg && pb->lg && pb->ug)),
               "pq_lr_capacitance: bad general rows");
  PQ_CHECK_ARG(k_ld % 64 == 0 && k_ld >= lr->tmax + pb->mg, "pq_lr_capacitance: k_ld too small");
  PQ_CHECK_ARG(st->rho != nullptr, "pq_lr_capacitance: rho missing");
  const int grid = idx ? nidx : pb->batch;
  if (grid <= 0) return 0;
  const int nb = k_ld / 64;
  hipLaunchKernelGGL(pq::k_lr_gram, dim3(nb * (nb + 1) / 2, grid), dim3(256), 0, (hipStream_t)stream,
                     *lr, *pb, st->rho, idx, *s, M, k_ld, M_stride);
  PQ_CHECK_LAUNCH("pq_lr_capacitance");
  return 0;
}
