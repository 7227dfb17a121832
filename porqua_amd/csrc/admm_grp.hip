// K3, grouped: the low-rank ADMM of pq_admm_lr_batched for a group of up to 16
// consecutive rebalance dates whose windows slide over one union of panel rows.
//
// A daily backtest's neighbouring windows share T - 1 of their T rows.  One 512-thread
// workgroup owns a group of G <= 16 dates (a slide group of engine.slide_plan, union of
// U = T + sum(shift) <= 320 rows) and runs their ADMM iterations in lock step.  The two
// passes over the window rows of the Woodbury solve become FP64 MFMA GEMMs over the union
// (every union row is read once per iteration for all G dates instead of once per date):
//     pass 1:  W  (U x G) = X_union V          V = D^-1 rhs of every date   (K = n)
//     pass 2:  X~ (n x G) = X_union' Ut        Ut = sqrt(ps) M^-1 w, zero outside a
//                                               date's own window rows      (K = U)
// Between them each wave applies the lower-triangle M_b^-1 of its two dates (the only
// per-date n-independent O(k^2) stream, from HBM).  The O(n) ADMM updates, residuals and
// convergence tests run with one half-wave (32 lanes) per date, so every per-date
// reduction is a half-wave shuffle and no workgroup barrier sits inside them.  Per-date
// vectors (x, z, y, Px and the V / rhs / X~ scratch) stay in global memory (L2), so the
// kernel needs no n-sized LDS and has no n <= 1024 limit.
//
// Replaces qpsolvers.solve_problem (src/qp_problems.py:211-214) for the batched backtest;
// the iterates are those of pq_admm_lr_batched up to summation order.
#include "common.h"
#include "capi_util.h"

namespace pq {

constexpr int GT = 512;      // threads per group workgroup
constexpr int GNW = GT / 64; // waves
constexpr int GMAX = 16;     // dates per group (MFMA N)
constexpr int UMAXG = 320;   // union rows per group
// General constraint rows: the kernel is instantiated with MGG LDS slots per date and
// either MGR > 0 (rows held in register arrays in the fused passes: mg <= MGR) or MGR == 0
// (any mg <= MGG: rows re-read from Cg per element and Cg x~ / Cg V as separate half-wave
// dot products -- group-cap constraints, e.g. 20 sector rows).
constexpr int MGG_SMALL = 8, MGR_SMALL = 4;
constexpr int MGG_BIG = 32;

__device__ __forceinline__ double grho(double l, double u, double rho, const pq_settings& s) {
  if (l == u) return rho * s.eq_scale;
  if (isinf(l) && isinf(u)) return s.rho_min;
  return rho;
}

// reductions over the 32 lanes of a half-wave (xor offsets < 32 stay inside the half)
__device__ __forceinline__ double hsum(double v) {
#pragma unroll
  for (int o = 16; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double hmax(double v) {
#pragma unroll
  for (int o = 16; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
  return v;
}

#ifdef PQ_PROFILE
#define GSTAMP(k)                                                 \
  do {                                                            \
    __syncthreads();                                              \
    if (threadIdx.x == 0) {                                       \
      const long long now_ = wall_clock64();                      \
      pclk[k] += now_ - tclk;                                     \
      tclk = now_;                                                \
    }                                                             \
  } while (0)
#else
#define GSTAMP(k) do { } while (0)
#endif

// FUSE (uniform ADMM diagonal D_g = c_g I and shared Cg, the band-Gram case): V = rhs / c_g
// is never stored (pass 1 multiplies the rhs and scales W by 1 / c_g), and Cg x~ is known
// before the x-update from scalars --
//   Cg x~ = Cg V - (PC' Ut - su Cg mu + Cg Cg' cw) / c_g,   PC[r][g] = x_r . Cg_g,
// so the x-update, residuals and next rhs run as ONE fused pass over each date's vectors
// (pass A's x~ round trip and its Cg x~ reductions disappear).
template <int NQK, int MGG, int MGR, bool FUSE>
__global__ __launch_bounds__(GT) void k_admm_grp(pq_lowrank lr, pq_problem pb, pq_state st,
                                                 const double* Minv_all, int k_ld, int64_t M_stride,
                                                 const int32_t* gdates, const int32_t* urows_all,
                                                 const int32_t* ucnt_all, const int32_t* uoff, int umax,
                                                 pq_settings s, int iters_call, const double* pc,
                                                 int64_t ldpc, int r0, const double* cc,
                                                 const int32_t* cg_nzr, const double* cg_nzv, int nzmax) {
  // pass-1 output W, overwritten in place by the symv with the pass-2 operand Ut (rows outside
  // a date's window zeroed); 2 workgroups fit on a CU
  __shared__ __attribute__((aligned(16))) double WU[(UMAXG + 4) * GMAX];
  double* const W = WU;
  double* const UT = WU;
  __shared__ double g_rho[GMAX], g_sps[GMAX], g_pd[GMAX], g_muv[GMAX], g_su[GMAX];
  __shared__ double g_zg[GMAX * MGG], g_yg[GMAX * MGG], g_rg[GMAX * MGG], g_lg[GMAX * MGG],
      g_ug[GMAX * MGG], g_cgv[GMAX * MGG], g_cgx[GMAX * MGG], g_kug[GMAX * MGG], g_wg[GMAX * MGG],
      g_cw[GMAX * MGG], g_zt[GMAX * MGG], g_rgz[GMAX * MGG];
  __shared__ int g_act[GMAX], g_it[GMAX], g_end[GMAX], g_stat[GMAX], g_off[GMAX], g_T[GMAX];
  __shared__ int s_urow[UMAXG];
  __shared__ double g_dinv[GMAX], g_rb[GMAX], g_cmu[FUSE ? GMAX * MGG : 1];
  __shared__ int s_any;
  __shared__ __attribute__((aligned(16))) double s_part[GNW * NQK * 128];   // symv partial vectors
  __shared__ double s_dot[NQK * 128];                                       // symv dot parts
  __shared__ double s_red[GNW];

  const int grp = xcd_slot(blockIdx.x, gridDim.x);
  const int d0 = gdates[grp];
  const int G = gdates[grp + 1] - d0;
  const int U = ucnt_all[grp];
  const int t = threadIdx.x, w = wave_id(), l = lane_id();
  const int n = pb.n, ld = pb.ld, mg = pb.mg, tmax = lr.tmax;
  const bool has_box = pb.lb != nullptr;
  const double sigma = s.sigma, alpha = s.alpha;
#ifdef PQ_PROFILE
  long long pclk[4] = {0, 0, 0, 0};
  long long tclk = wall_clock64();
#endif

  // ---- setup ---------------------------------------------------------------------------
  for (int u = t; u < UMAXG; u += GT) s_urow[u] = u < U ? urows_all[(int64_t)grp * umax + u] : 0;
  for (int e = t; e < (UMAXG + 4) * GMAX; e += GT) UT[e] = 0.0;
  if (t < GMAX) {
    const int g = t;
    int act = 0;
    if (g < G) {
      const int b = d0 + g;
      const int stt = st.status[b];
      act = (stt == PQ_UNSOLVED || stt == PQ_NEED_REFACTOR);
      g_rho[g] = st.rho[b];
      g_it[g] = st.iters[b];
      g_end[g] = min(s.max_iter, st.iters[b] + iters_call);
      g_stat[g] = stt;
      g_T[g] = lr.tlen[b];
      g_off[g] = uoff[b];
      const double ps = (pb.p_scale ? pb.p_scale[b] : 1.0) * (lr.w_scale ? lr.w_scale[b] : 1.0);
      g_sps[g] = sqrt(fmax(ps, 0.0));
      g_pd[g] = pb.p_diag ? pb.p_diag[b] : 0.0;
      if (FUSE) {   // uniform box rho (host-checked): D = sigma + p_diag + rho_box
        const double rb = has_box ? grho(pb.lb[(int64_t)b * pb.box_stride], pb.ub[(int64_t)b * pb.box_stride],
                                         st.rho[b], s) : 0.0;
        g_rb[g] = rb;
        g_dinv[g] = 1.0 / (sigma + g_pd[g] + rb);
      }
    }
    g_act[g] = act;
  }
  for (int e = t; e < GMAX * MGG; e += GT) {
    const int g = e / MGG, r = e % MGG;
    double zg = 0, yg = 0, lgv = 0, ugv = 0, rg = 0;
    if (g < G && r < mg) {
      const int b = d0 + g;
      zg = st.z[(int64_t)b * st.m_ld + r];
      yg = st.y[(int64_t)b * st.m_ld + r];
      lgv = pb.lg[(int64_t)b * pb.g_stride + r];
      ugv = pb.ug[(int64_t)b * pb.g_stride + r];
      rg = grho(lgv, ugv, st.rho[b], s);
    }
    g_zg[e] = zg;
    g_yg[e] = yg;
    g_lg[e] = lgv;
    g_ug[e] = ugv;
    g_rg[e] = rg;
  }
  __syncthreads();

  // ---- per-date (half-wave) views ---------------------------------------------------------
  const int hg = t >> 5, hl = t & 31;
  const bool hmine = hg < G;
  const int hb = d0 + (hmine ? hg : 0);
  // per-date pointers of the half-wave's date (recomputed where used: keeps them out of the
  // registers that the MFMA phases need)
#define PQ_HPTRS                                                                              \
  const double* __restrict__ q_h = pb.q + (int64_t)hb * pb.q_stride;                          \
  const double* __restrict__ lo_h = has_box ? pb.lb + (int64_t)hb * pb.box_stride : nullptr;  \
  const double* __restrict__ up_h = has_box ? pb.ub + (int64_t)hb * pb.box_stride : nullptr;  \
  const double* __restrict__ Cg_h = mg ? pb.Cg + (int64_t)hb * pb.Cg_stride : nullptr;        \
  const double* __restrict__ mu_h = lr.mu ? lr.mu + (int64_t)hb * lr.mu_stride : nullptr;     \
  double* __restrict__ x_h = st.x + (int64_t)hb * ld;                                         \
  double* __restrict__ Px_h = st.Px + (int64_t)hb * ld;                                       \
  double* __restrict__ zb_h = st.z + (int64_t)hb * st.m_ld + st.mg_pad;                       \
  double* __restrict__ yb_h = st.y + (int64_t)hb * st.m_ld + st.mg_pad;                       \
  double* __restrict__ V_h = st.work + (int64_t)hb * st.work_stride;                          \
  double* __restrict__ R_h = V_h + ld;                                                        \
  double* __restrict__ X_h = V_h + 2 * ld;                                                    \
  (void)q_h; (void)lo_h; (void)up_h; (void)Cg_h; (void)mu_h; (void)x_h; (void)Px_h;           \
  (void)zb_h; (void)yb_h; (void)V_h; (void)R_h; (void)X_h

  // rhs = sigma x - q + rho_box z - y + Cg'(R zg - yg);  V = rhs / D;  mu.V, Cg.V
  auto next_rhs = [&](int g) {
    PQ_HPTRS;
    const double rho = g_rho[g], pd = g_pd[g];
    if (hl < mg) g_wg[g * MGG + hl] = g_rg[g * MGG + hl] * g_zg[g * MGG + hl] - g_yg[g * MGG + hl];
    double muv = 0.0;
    for (int i = hl; i < n; i += 32) {
      const double rb = has_box ? grho(lo_h[i], up_h[i], rho, s) : 0.0;
      double rr = sigma * x_h[i] - q_h[i];
      if (has_box) rr += rb * zb_h[i] - yb_h[i];
      for (int r = 0; r < mg; ++r) rr += Cg_h[(int64_t)r * ld + i] * g_wg[g * MGG + r];
      const double v = rr / (sigma + pd + rb);
      R_h[i] = rr;
      V_h[i] = v;
      if (mu_h) muv = fma(mu_h[i], v, muv);
    }
    for (int i = n + hl; i < ld; i += 32) V_h[i] = 0.0;
    muv = hsum(muv);
    for (int r = 0; r < mg; ++r) {   // Cg . V (each lane re-reads its own V entries)
      double a = 0.0;
      for (int i = hl; i < n; i += 32) a = fma(Cg_h[(int64_t)r * ld + i], V_h[i], a);
      a = hsum(a);
      if (hl == 0) g_cgv[g * MGG + r] = a;
    }
    if (hl == 0) g_muv[g] = muv;
    if (FUSE) {   // Cg . mu of the date (constant over the launch)
      for (int r = 0; r < mg; ++r) {
        double a = 0.0;
        if (mu_h)
          for (int i = hl; i < n; i += 32) a = fma(Cg_h[(int64_t)r * ld + i], mu_h[i], a);
        a = hsum(a);
        if (hl == 0) g_cmu[g * MGG + r] = a;
      }
    }
  };

  // ---- prologue: Cg x and the first rhs -------------------------------------------------
  if (hmine && g_act[hg]) {
    PQ_HPTRS;
    for (int r = 0; r < mg; ++r) {
      double a = 0.0;
      for (int i = hl; i < n; i += 32) a = fma(Cg_h[(int64_t)r * ld + i], x_h[i], a);
      a = hsum(a);
      if (hl == 0) g_cgx[hg * MGG + r] = a;
    }
    next_rhs(hg);
  }
  if (t == 0) {
    int any = 0;
    for (int g = 0; g < G; ++g) any |= g_act[g];
    s_any = any;
  }
  __syncthreads();

  const int ntile = (U + 15) >> 4;
  while (s_any) {
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Wshadow"
    const int t = threadIdx.x + loop_zero();   // re-materialised lane ids (common.h: loop_zero)
    const int w = t >> 6, l = t & 63, hg = t >> 5, hl = t & 31;
#pragma clang diagnostic pop
    (void)hl;
    // ---- pass 1: W = X_union V (MFMA f64 16x16x4; a 16-B load feeds two k-slices) -------
    {
      const int kq = l >> 4, m = l & 15;
      // V of date m (FUSE: its rhs, W scaled by 1 / c_m below)
      const double* Vp = (m < G) ? st.work + (int64_t)(d0 + m) * st.work_stride + (FUSE ? ld : 0) : nullptr;
      const double wsc1 = (FUSE && m < G) ? g_dinv[m] : 1.0;
      f64x4 c[3];
      const double* arow[3];
      bool tv[3], aval[3];
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        c[j] = f64x4{0.0, 0.0, 0.0, 0.0};
        const int u = (w + GNW * j) * 16 + m;
        tv[j] = w + GNW * j < ntile;
        aval[j] = u < U;
        arow[j] = lr.panel + (int64_t)s_urow[u < UMAXG ? u : 0] * lr.ldp;
      }
      // one k-step of 8 columns per buffer, two buffers: loads run a step ahead
      constexpr int HS = 1;
      struct Buf { double2 b[HS]; double2 a[HS][3]; };
      auto load = [&](Buf& f, int k0) {
#pragma unroll
        for (int h = 0; h < HS; ++h) {
          const int kk = k0 + 8 * h + 2 * kq;
          const bool kin = kk + 1 < n;   // n even (host check): kk < n <=> kk + 1 < n
          f.b[h] = (Vp && kin) ? *reinterpret_cast<const double2*>(Vp + kk) : double2{0.0, 0.0};
#pragma unroll
          for (int j = 0; j < 3; ++j)
            f.a[h][j] = (tv[j] && aval[j] && kin) ? *reinterpret_cast<const double2*>(arow[j] + kk)
                                                  : double2{0.0, 0.0};
        }
      };
      auto mma = [&](const Buf& f) {
#pragma unroll
        for (int h = 0; h < HS; ++h)
#pragma unroll
          for (int j = 0; j < 3; ++j)
            if (tv[j]) {
              c[j] = __builtin_amdgcn_mfma_f64_16x16x4f64(f.a[h][j].x, f.b[h].x, c[j], 0, 0, 0);
              c[j] = __builtin_amdgcn_mfma_f64_16x16x4f64(f.a[h][j].y, f.b[h].y, c[j], 0, 0, 0);
            }
      };
      Buf f0, f1;
      load(f0, 0);
      for (int k0 = 0; k0 < n; k0 += 16 * HS) {
        load(f1, k0 + 8 * HS);
        mma(f0);
        load(f0, k0 + 16 * HS);
        mma(f1);
      }
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const int tile = w + GNW * j;
        if (tv[j]) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int u = tile * 16 + kq + 4 * r;
            if (u < UMAXG) W[u * GMAX + m] = wsc1 * c[j][r];
          }
        }
      }
    }
    __syncthreads();
    GSTAMP(0);

    // ---- u = M_b^-1 w, one date at a time with all 8 waves (rows j = w mod 8, lower
    //      triangle: dot part per row + axpy part in registers), then a column-wise combine
    for (int g = 0; g < G; ++g) {
      if (!g_act[g]) continue;   // uniform: LDS flag
      const int b = d0 + g;
      const int T = g_T[g], off = g_off[g];
      const int k = tmax + mg;
      const double sps = g_sps[g], muv = g_muv[g];
      const double* Mi = Minv_all + (int64_t)b * M_stride;
      auto kwv = [&](int j) -> double {
        if (j < T) return sps * (W[(off + j) * GMAX + g] - muv);
        if (j >= tmax && j < k) return sqrt(g_rg[g * MGG + j - tmax]) * g_cgv[g * MGG + j - tmax];
        return 0.0;
      };
      double2 rv[NQK], acc[NQK];
#pragma unroll
      for (int qq = 0; qq < NQK; ++qq) {
        const int c = 128 * qq + 2 * l;
        rv[qq] = double2{kwv(c), kwv(c + 1)};
        acc[qq] = double2{0.0, 0.0};
      }
      constexpr int RU = 4;
      struct RBuf { double2 r[RU][NQK]; };
      auto rload = [&](RBuf& f, int j0) {   // rows j0 + GNW e
#pragma unroll
        for (int e = 0; e < RU; ++e) {
          const int j = j0 + GNW * e;
          const double2* rp = reinterpret_cast<const double2*>(Mi + (int64_t)(j < k ? j : 0) * k_ld) + l;
#pragma unroll
          for (int qq = 0; qq < NQK; ++qq) {
            const int c = 128 * qq + 2 * l;
            f.r[e][qq] = (j < k && c <= j) ? rp[64 * qq] : double2{0.0, 0.0};
          }
        }
      };
      auto rblock = [&](const RBuf& f, int j0) {
        double dd[RU];
#pragma unroll
        for (int e = 0; e < RU; ++e) {
          const int j = j0 + GNW * e;
          const double a = j < k ? kwv(j) : 0.0;
          double sd = 0.0;
#pragma unroll
          for (int qq = 0; qq < NQK; ++qq) {
            const int c = 128 * qq + 2 * l;
            const double yy = (c + 1 <= j) ? f.r[e][qq].y : 0.0;
            sd = fma(f.r[e][qq].x, rv[qq].x, fma(yy, rv[qq].y, sd));
            acc[qq].x = fma(a, (c < j) ? f.r[e][qq].x : 0.0, acc[qq].x);
            acc[qq].y = fma(a, (c + 1 < j) ? yy : 0.0, acc[qq].y);
          }
          dd[e] = sd;
        }
#pragma unroll
        for (int e = 0; e < RU; ++e) dd[e] = wave_sum(dd[e]);
        if (l == 0) {
#pragma unroll
          for (int e = 0; e < RU; ++e) {
            const int j = j0 + GNW * e;
            if (j < k) s_dot[j] = dd[e];
          }
        }
      };
      RBuf b0, b1;
      rload(b0, w);
      for (int j0 = w; j0 < k; j0 += 2 * GNW * RU) {
        rload(b1, j0 + GNW * RU);
        rblock(b0, j0);
        rload(b0, j0 + 2 * GNW * RU);
        rblock(b1, j0 + GNW * RU);
      }
#pragma unroll
      for (int qq = 0; qq < NQK; ++qq)
        reinterpret_cast<double2*>(s_part + w * (NQK * 128))[64 * qq + l] = acc[qq];
      __syncthreads();
      double su = 0.0;
      for (int c = t; c < k; c += GT) {
        if (c < T || c >= tmax) {
          double uu = s_dot[c];
#pragma unroll
          for (int ww = 0; ww < GNW; ++ww) uu += s_part[ww * (NQK * 128) + c];
          if (c < T) {
            UT[(off + c) * GMAX + g] = sps * uu;
            su += sps * uu;
          } else {
            g_kug[g * MGG + (c - tmax)] = uu;
          }
        }
      }
      const int Uk = (U + 3) & ~3;
      for (int u = t; u < Uk; u += GT)
        if (u < off || u >= off + T) UT[u * GMAX + g] = 0.0;
      su = wave_sum(su);
      if (l == 0) s_red[w] = su;
      __syncthreads();
      if (t == 0) {
        double a = 0.0;
        for (int ww = 0; ww < GNW; ++ww) a += s_red[ww];
        g_su[g] = a;
      }
    }
    __syncthreads();
    GSTAMP(1);

    // ---- pass 2: X~raw (n x G) = X_union' Ut; asset pairs of 16-column MFMA tiles (even /
    //      odd columns share each 16-B load), union-row loads run 4-8 steps ahead ---------------
    {
      const int kq = l >> 4, m = l & 15;
      const int Uk = (U + 3) & ~3;
      constexpr int PS = 4;   // k-steps (4 union rows each) per buffer
      for (int p = w; p * 32 < n; p += GNW) {
        const int col = p * 32 + 2 * m;
        const bool cin = col < n;
        f64x4 ce = f64x4{0.0, 0.0, 0.0, 0.0}, co = f64x4{0.0, 0.0, 0.0, 0.0};
        struct ABuf { double2 a[PS]; };
        auto load = [&](ABuf& f, int u0) {
#pragma unroll
          for (int h = 0; h < PS; ++h) {
            const int u = u0 + 4 * h + kq;
            f.a[h] = (u < U && cin)
                ? *reinterpret_cast<const double2*>(lr.panel + (int64_t)s_urow[u] * lr.ldp + col)
                : double2{0.0, 0.0};
          }
        };
        auto mma = [&](const ABuf& f, int u0) {
#pragma unroll
          for (int h = 0; h < PS; ++h) {
            const int u = u0 + 4 * h + kq;
            const double bv = u < Uk ? UT[u * GMAX + m] : 0.0;
            ce = __builtin_amdgcn_mfma_f64_16x16x4f64(f.a[h].x, bv, ce, 0, 0, 0);
            co = __builtin_amdgcn_mfma_f64_16x16x4f64(f.a[h].y, bv, co, 0, 0, 0);
          }
        };
        ABuf f0, f1;
        load(f0, 0);
        for (int u0 = 0; u0 < Uk; u0 += 8 * PS) {
          load(f1, u0 + 4 * PS);
          mma(f0, u0);
          load(f0, u0 + 8 * PS);
          mma(f1, u0 + 4 * PS);
        }
        if (m < G && g_act[m]) {
          double* xr = st.work + (int64_t)(d0 + m) * st.work_stride + 2 * ld;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int i = p * 32 + 2 * (kq + 4 * r);
            if (i < n) xr[i] = ce[r];
            if (i + 1 < n) xr[i + 1] = co[r];
          }
        }
      }
    }
    __syncthreads();
    GSTAMP(2);

    // ---- per-date updates, residuals, convergence, next rhs (half-wave per date): two
    //      fused passes over the date's vectors, 4 elements per lane in flight -------------
    if (hmine && g_act[hg]) {
      PQ_HPTRS;
      const int g = hg;
      const double rho = g_rho[g], pd = g_pd[g], su = g_su[g];
      const double dsig = sigma + pd;
      if (hl < mg) g_cw[g * MGG + hl] = sqrt(g_rg[g * MGG + hl]) * g_kug[g * MGG + hl];
      constexpr int MGRA = MGR > 0 ? MGR : 1;
      if constexpr (!FUSE) {
        // pass A: x~ = v - D^-1 (X~raw - mu su + Cg' cw), and Cg x~
        double ztp[MGRA];
  #pragma unroll
        for (int r = 0; r < MGRA; ++r) ztp[r] = 0.0;
  #pragma unroll 2
        for (int i = hl; i < n; i += 32) {
          double corr = X_h[i] - (mu_h ? su * mu_h[i] : 0.0);
          const double rb = has_box ? grho(lo_h[i], up_h[i], rho, s) : 0.0;
          double cgi[MGRA];
          if constexpr (MGR > 0) {
  #pragma unroll
            for (int r = 0; r < MGR; ++r) {
              cgi[r] = r < mg ? Cg_h[(int64_t)r * ld + i] : 0.0;
              corr = fma(r < mg ? g_cw[g * MGG + r] : 0.0, cgi[r], corr);
            }
          } else {
            for (int r = 0; r < mg; ++r) corr = fma(g_cw[g * MGG + r], Cg_h[(int64_t)r * ld + i], corr);
          }
          const double xt = V_h[i] - corr / (dsig + rb);
          X_h[i] = xt;
          if constexpr (MGR > 0) {
  #pragma unroll
            for (int r = 0; r < MGR; ++r) ztp[r] = fma(cgi[r], xt, ztp[r]);
          }
        }
        if constexpr (MGR > 0) {
  #pragma unroll
          for (int r = 0; r < MGR; ++r) {
            if (r >= mg) break;
            const double a = hsum(ztp[r]);
            if (hl == 0) g_zt[g * MGG + r] = a;
          }
        } else {   // each lane re-reads the x~ entries it wrote
          for (int r = 0; r < mg; ++r) {
            double a = 0.0;
            for (int i = hl; i < n; i += 32) a = fma(Cg_h[(int64_t)r * ld + i], X_h[i], a);
            a = hsum(a);
            if (hl == 0) g_zt[g * MGG + r] = a;
          }
        }
      } else {   // Cg x~ from scalars: Cg V - (PC' Ut - su Cg mu + Cg Cg' cw) / c
        const double dinv = g_dinv[g];
        const int Ug = ucnt_all[grp];
        for (int r = 0; r < mg; ++r) {
          double a = 0.0;
          for (int u = hl; u < Ug; u += 32) a = fma(pc[(int64_t)(s_urow[u] - r0) * ldpc + r], UT[u * GMAX + g], a);
          a = hsum(a);
          double cw = 0.0;
          for (int r2 = 0; r2 < mg; ++r2) cw = fma(cc[r * mg + r2], g_cw[g * MGG + r2], cw);
          if (hl == 0) g_zt[g * MGG + r] = g_cgv[g * MGG + r] - dinv * (a - su * g_cmu[g * MGG + r] + cw);
        }
      }
      double mv[7] = {0, 0, 0, 0, 0, 0, 0};   // |Cx-z| |Cx| |z| |dres| |Px| |C'y| |q|
      if (hl < mg) {   // general row hl: z, y, Cx (lane-owned); R z - y for the next rhs
        const int e = g * MGG + hl;
        const double rg = g_rg[e], zt = g_zt[e];
        const double zh = alpha * zt + (1.0 - alpha) * g_zg[e];
        const double zn = fmin(fmax(zh + g_yg[e] / rg, g_lg[e]), g_ug[e]);
        const double yn = g_yg[e] + rg * (zh - zn);
        const double cx = alpha * zt + (1.0 - alpha) * g_cgx[e];
        mv[0] = fabs(cx - zn);
        mv[1] = fabs(cx);
        mv[2] = fabs(zn);
        g_rgz[e] = rg * zt;
        g_zg[e] = zn;
        g_yg[e] = yn;
        g_cgx[e] = cx;
        g_wg[e] = rg * zn - yn;
      }
      // pass B: x, Px, z, y updates, residual terms, next rhs and V = rhs / D, mu.V, Cg.V
      double muv = 0.0, cvp[MGRA];
#pragma unroll
      for (int r = 0; r < MGRA; ++r) cvp[r] = 0.0;
#pragma unroll 2
      for (int i = hl; i < n; i += 32) {
        const double rb = has_box ? grho(lo_h[i], up_h[i], rho, s) : 0.0;
        const double rr0 = R_h[i];
        double xt, pxt, cgy = 0.0, cgw = 0.0, cgi[MGRA];
        if constexpr (MGR == 0) {   // many rows: each Cg entry of asset i read once for all four sums
          double cwd = 0.0, rgd = 0.0;
          auto row_terms = [&](int r, double c) {
            if (FUSE) cwd = fma(g_cw[g * MGG + r], c, cwd);
            rgd = fma(c, g_rgz[g * MGG + r], rgd);
            cgy = fma(c, g_yg[g * MGG + r], cgy);
            cgw = fma(c, g_wg[g * MGG + r], cgw);
          };
          if (nzmax > 0) {   // sparse columns of the shared rows (e.g. budget + sector memberships)
            for (int e = 0; e < nzmax; ++e) {
              const int r = cg_nzr[(int64_t)i * nzmax + e];
              if (r < 0) break;
              row_terms(r, cg_nzv[(int64_t)i * nzmax + e]);
            }
          } else {
            for (int r = 0; r < mg; ++r) row_terms(r, Cg_h[(int64_t)r * ld + i]);
          }
          // FUSE: x~ = (rhs - X~raw + mu su - Cg' cw) / c, fused with the updates
          xt = FUSE ? (rr0 - (X_h[i] - (mu_h ? su * mu_h[i] : 0.0) + cwd)) * g_dinv[g] : X_h[i];
          pxt = rr0 - sigma * xt - rb * xt - rgd;
          cgi[0] = 0.0;
        } else {
          if constexpr (FUSE) {   // x~ = (rhs - X~raw + mu su - Cg' cw) / c, fused with the updates
            double corr = X_h[i] - (mu_h ? su * mu_h[i] : 0.0);
#pragma unroll
            for (int r = 0; r < MGRA; ++r)
              if (r < mg) corr = fma(g_cw[g * MGG + r], Cg_h[(int64_t)r * ld + i], corr);
            xt = (rr0 - corr) * g_dinv[g];
          } else {
            xt = X_h[i];
          }
          pxt = rr0 - sigma * xt - rb * xt;
#pragma unroll
          for (int r = 0; r < MGR; ++r) {
            cgi[r] = r < mg ? Cg_h[(int64_t)r * ld + i] : 0.0;
            if (r < mg) {
              pxt -= cgi[r] * g_rgz[g * MGG + r];
              cgy = fma(cgi[r], g_yg[g * MGG + r], cgy);
              cgw = fma(cgi[r], g_wg[g * MGG + r], cgw);
            }
          }
        }
        const double xn = alpha * xt + (1.0 - alpha) * x_h[i];
        const double pxn = alpha * pxt + (1.0 - alpha) * Px_h[i];
        const double qi = q_h[i];
        double rr = sigma * xn - qi + cgw;
        double cty = 0.0;
        if (has_box) {
          const double zh = alpha * xt + (1.0 - alpha) * zb_h[i];
          const double zn = fmin(fmax(zh + yb_h[i] / rb, lo_h[i]), up_h[i]);
          const double yn = yb_h[i] + rb * (zh - zn);
          zb_h[i] = zn;
          yb_h[i] = yn;
          cty = yn;
          rr += rb * zn - yn;
          mv[0] = fmax(mv[0], fabs(xn - zn));
          mv[1] = fmax(mv[1], fabs(xn));
          mv[2] = fmax(mv[2], fabs(zn));
        }
        x_h[i] = xn;
        Px_h[i] = pxn;
        mv[4] = fmax(mv[4], fabs(pxn));
        mv[6] = fmax(mv[6], fabs(qi));
        const double cy = cty + cgy;
        mv[3] = fmax(mv[3], fabs((pxn + qi + cty) + (cy - cty)));
        mv[5] = fmax(mv[5], fabs(cy));
        const double v = FUSE ? rr * g_dinv[g] : rr / (dsig + rb);
        R_h[i] = rr;
        if (!FUSE) V_h[i] = v;
        if (mu_h) muv = fma(mu_h[i], v, muv);
        if constexpr (MGR > 0) {
#pragma unroll
          for (int r = 0; r < MGR; ++r) cvp[r] = fma(cgi[r], v, cvp[r]);
        }
      }
#pragma unroll
      for (int e = 0; e < 7; ++e) mv[e] = hmax(mv[e]);
      muv = hsum(muv);
      if constexpr (MGR > 0) {
#pragma unroll
        for (int r = 0; r < MGR; ++r) {
          if (r >= mg) break;
          cvp[r] = hsum(cvp[r]);
        }
      } else {   // Cg V: written straight to the date's slots (read only by the next symv);
                 // four rows per pass over the date's vector (FUSE: V = rhs / c is not stored)
        const double dv = FUSE ? g_dinv[g] : 1.0;
        const double* vsrc = FUSE ? R_h : V_h;
        for (int q0 = 0; q0 < mg; q0 += 4) {
          double a[4] = {0.0, 0.0, 0.0, 0.0};
          for (int i = hl; i < n; i += 32) {
            const double vi = vsrc[i] * dv;
#pragma unroll
            for (int e = 0; e < 4; ++e)
              if (q0 + e < mg) a[e] = fma(Cg_h[(int64_t)(q0 + e) * ld + i], vi, a[e]);
          }
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const double v = hsum(a[e]);
            if (hl == 0 && q0 + e < mg) g_cgv[g * MGG + q0 + e] = v;
          }
        }
      }
      const int it = g_it[g] + 1;
      int stat = PQ_UNSOLVED;
      const double eps_p = s.eps_abs + s.eps_rel * fmax(mv[1], mv[2]);
      const double eps_d = s.eps_abs + s.eps_rel * fmax(mv[4], fmax(mv[5], mv[6]));
      double rnew = rho;
      if (it >= s.min_iter && mv[0] <= eps_p && mv[3] <= eps_d) {
        stat = PQ_SOLVED;
      } else if (s.adapt_interval > 0 && it % s.adapt_interval == 0) {
        const double rp = mv[0] / (fmax(mv[1], mv[2]) + 1e-30);
        const double rd = mv[3] / (fmax(mv[4], fmax(mv[5], mv[6])) + 1e-30);
        double rn = rho * sqrt(rp / (rd + 1e-30));
        rn = fmin(fmax(rn, s.rho_min), s.rho_max);
        if (rn > rho * s.adapt_tol || rn < rho / s.adapt_tol) {
          rnew = rn;
          stat = PQ_NEED_REFACTOR;
        }
      }
      if (stat == PQ_UNSOLVED && it >= s.max_iter) stat = PQ_MAX_ITER;
      const bool cont = (stat == PQ_UNSOLVED) && it < g_end[g];
      if (hl == 0) {
        g_it[g] = it;
        g_rho[g] = rnew;
        g_stat[g] = stat;
        g_act[g] = cont;
        g_muv[g] = muv;
        if constexpr (MGR > 0) {
#pragma unroll
          for (int r = 0; r < MGR; ++r)
            if (r < mg) g_cgv[g * MGG + r] = cvp[r];
        }
      }
    }
    __syncthreads();
    if (t == 0) {
      int any = 0;
      for (int g = 0; g < G; ++g) any |= g_act[g];
      s_any = any;
    }
    __syncthreads();
    GSTAMP(3);
  }

  // ---- write back the per-date scalars and the general rows -------------------------------
  if (t < G) {
    const int b = d0 + t;
    const int stt0 = st.status[b];
    if (stt0 == PQ_UNSOLVED || stt0 == PQ_NEED_REFACTOR) {
      st.iters[b] = g_it[t];
      st.status[b] = g_stat[t];
      st.rho[b] = g_rho[t];
    }
  }
  for (int e = t; e < GMAX * MGG; e += GT) {
    const int g = e / MGG, r = e % MGG;
    if (g < G && r < mg) {
      const int b = d0 + g;
      st.z[(int64_t)b * st.m_ld + r] = g_zg[e];
      st.y[(int64_t)b * st.m_ld + r] = g_yg[e];
    }
  }
#ifdef PQ_PROFILE
  if (t == 0) {   // the timers run on thread 0: share the group's phase times over its dates
    for (int g = 0; g < G; ++g) {
      double* dstp = st.work + (int64_t)(d0 + g) * st.work_stride + PQ_WORK_PROF(ld, st.mg_pad) + 16;
      for (int k2 = 0; k2 < 4; ++k2) dstp[k2] += (double)pclk[k2] / G;
    }
  }
#endif
}

}  // namespace pq

extern "C" int pq_admm_lr_grouped(const pq_lowrank* lr, const pq_problem* pb, pq_state* st,
                                  const double* Minv, int32_t k_ld, int64_t M_stride,
                                  const int32_t* gdates, int32_t ngroups, const int32_t* urows,
                                  const int32_t* ucnt, const int32_t* uoff, int32_t umax,
                                  const pq_settings* s, int32_t iters_this_call, const double* pc,
                                  int64_t ldpc, int32_t r0, const double* cc, const int32_t* cg_nzr,
                                  const double* cg_nzv, int32_t nzmax, void* stream) {
  PQ_CHECK_ARG(lr && pb && st && s && Minv, "pq_admm_lr_grouped: null argument");
  PQ_CHECK_ARG((pc == nullptr) == (cc == nullptr), "pq_admm_lr_grouped: pc and cc go together");
  PQ_CHECK_ARG(nzmax == 0 || (cg_nzr && cg_nzv && nzmax > 0 && nzmax <= pb->mg && pb->Cg_stride == 0),
               "pq_admm_lr_grouped: sparse columns need shared Cg and 0 < nzmax <= mg");
  PQ_CHECK_ARG(pc == nullptr || pb->Cg_stride == 0, "pq_admm_lr_grouped: the fused form needs shared Cg");
  PQ_CHECK_ARG(lr->panel && lr->rows && lr->tlen && lr->tmax > 0, "pq_admm_lr_grouped: window missing");
  PQ_CHECK_ARG(gdates && urows && ucnt && uoff && umax > 0, "pq_admm_lr_grouped: group plan missing");
  PQ_CHECK_ARG(pb->mg >= 0 && pb->mg <= pq::MGG_BIG && (pb->mg == 0 || (pb->Cg && pb->lg && pb->ug)),
               "pq_admm_lr_grouped: needs 0 <= mg <= %d general rows (mg=%d)", pq::MGG_BIG, pb->mg);
  PQ_CHECK_ARG(pb->n % 2 == 0 && lr->ldp % 2 == 0, "pq_admm_lr_grouped: needs even n and panel stride");
  PQ_CHECK_ARG(st->work && st->work_stride >= 3 * (int64_t)pb->ld, "pq_admm_lr_grouped: work buffer too small");
  const int k = lr->tmax + pb->mg;
  PQ_CHECK_ARG(k_ld % 64 == 0 && k_ld >= k && k_ld <= 384, "pq_admm_lr_grouped: need k <= k_ld <= 384 (k=%d)", k);
  if (ngroups <= 0) return 0;
  hipStream_t str = (hipStream_t)stream;
  const int nqk = (k_ld + 127) / 128;
#define PQ_GRP_CASE(NQKV, MGGV, MGRV, FUSEV)                                                              \
  hipLaunchKernelGGL((pq::k_admm_grp<NQKV, MGGV, MGRV, FUSEV>), dim3(ngroups), dim3(pq::GT), 0, str, *lr, *pb,   \
                     *st, Minv, k_ld, M_stride, gdates, urows, ucnt, uoff, umax, *s, iters_this_call, pc, ldpc,  \
                     r0, cc, cg_nzr, cg_nzv, (MGRV) == 0 ? nzmax : 0)
  const bool small = pb->mg <= pq::MGR_SMALL;
  const bool fuse = pc != nullptr && cc != nullptr;
  switch (nqk * 4 + (fuse ? (small ? 2 : 3) : (small ? 0 : 1))) {
    case 4: PQ_GRP_CASE(1, pq::MGG_SMALL, pq::MGR_SMALL, false); break;
    case 5: PQ_GRP_CASE(1, pq::MGG_BIG, 0, false); break;
    case 6: PQ_GRP_CASE(1, pq::MGG_SMALL, pq::MGR_SMALL, true); break;
    case 7: PQ_GRP_CASE(1, pq::MGG_BIG, 0, true); break;
    case 8: PQ_GRP_CASE(2, pq::MGG_SMALL, pq::MGR_SMALL, false); break;
    case 9: PQ_GRP_CASE(2, pq::MGG_BIG, 0, false); break;
    case 10: PQ_GRP_CASE(2, pq::MGG_SMALL, pq::MGR_SMALL, true); break;
    case 11: PQ_GRP_CASE(2, pq::MGG_BIG, 0, true); break;
    case 12: PQ_GRP_CASE(3, pq::MGG_SMALL, pq::MGR_SMALL, false); break;
    case 13: PQ_GRP_CASE(3, pq::MGG_BIG, 0, false); break;
    case 14: PQ_GRP_CASE(3, pq::MGG_SMALL, pq::MGR_SMALL, true); break;
    case 15: PQ_GRP_CASE(3, pq::MGG_BIG, 0, true); break;
    default:
      pq::set_error("pq_admm_lr_grouped: unsupported k_ld=%d", k_ld);
      return -1;
  }
#undef PQ_GRP_CASE
  PQ_CHECK_LAUNCH("pq_admm_lr_grouped");
  return 0;
}
