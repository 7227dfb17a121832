// K2 + K3 with ONE capacitance matrix per slide group ("group capacitance").
//
// The grouped ADMM of admm_grp.hip applies every date's own k x k capacitance inverse
// M_b^-1 (k = T + mg) each iteration: 4749 factorisations per config-3 backtest, and a
// 512 KB per-date stream that dominates the kernel's HBM traffic.  Neighbouring windows
// share all but a few rows, so here the dates of a group (same T, same c = p_scale w_scale,
// same p_diag, one rho) share the capacitance of the UNION of their windows,
//     K_U = d I + W_U' W_U,   W_U = [sqrt(c) X_U ; sqrt(R) Cg]   (raw union rows),
//     M_U = I + W_U W_U' / d   ((U + mg) x (U + mg): one factorisation per group),
// and each date's own system differs from K_U by a low-rank term:
//     K_b = K_U - V_b V_b',   V_b = sqrt(c) [X_Cb' , sqrt(T) mu_b]
// (C_b = the union rows outside the date's window, m = U - T of them; the mean column is
// the centring).  Woodbury on that difference needs only the small SPD matrix
//     H_b = I - V_b' K_U^-1 V_b = [[ (M_U^-1)_CC , -(sqrt(cT)/d) q_C ],
//                                  [ .           , 1 - (cT/d)(mu'mu - a'q/d) ]]
// with a_b = W_U mu_b and q_b = M_U^-1 a_b, so per date the preparation is O(U T + U^2 +
// m^3) (pq_gcap_prepare).  Per ADMM iteration the group does
//     z' = M_U^-1 [sqrt(c) X_U V ; sqrt(R) Cg V]                (one MFMA GEMM, G columns)
//     s_b = [z'_C ; sqrt(cT)(mu_b.V - a_b.z'/d)],  y_b = H_b^-1 s_b
//     Ut_b = sqrt(c) (z' - (M_U^-1)_{:,C} y_C + (sqrt(cT)/d) y_mu q_b)_X,
//     cw_b = sqrt(R) (same)_G,  su_b = sqrt(cT) y_mu,
// after which pass 2 and the fused per-date updates of admm_grp.hip run unchanged
// (x~ = V - D^-1 (X_U' Ut - su mu + Cg' cw)).  Exact algebra: the iterates are those of
// the per-date kernel with the group's rho, to rounding (checked against a dense solve in
// tests).  Adaptive rho is decided per group (geometric mean of the dates' requests), so
// a refactorisation rebuilds one M_U per group.
//
// Replaces qpsolvers.solve_problem (src/qp_problems.py:211-214) for the batched backtest,
// like pq_admm_lr_grouped.
#include "chol_dev.h"   // (common.h; tile_chol_inv64 for the H_b of m + 1 > 32)
#include "capi_util.h"

namespace pq {

constexpr int CT = 256;        // threads per group workgroup (two workgroups per CU: the
constexpr int CNW = CT / 64;   // phases of two groups overlap -- MFMA passes vs memory-bound)
constexpr int CHW = CT / 32;   // half-waves (each serves dates hg, hg + CHW, ...)
constexpr int CTP1 = 5;        // pass-1 row tiles per wave (U <= 320: 20 tiles)
constexpr int CTP2 = 6;        // GEMM row tiles per wave (U + mg <= 324: 21 tiles)
constexpr int CG_MAX = 16;     // dates per group (MFMA N)
constexpr int CU_MAX = 320;    // union rows per group
constexpr int CMG = 4;         // general rows (register-resident, fused form)
constexpr int CMGW = 24;       // general rows, wide form: column-sparse Cg (budget + sector caps)
constexpr int CNZ = 4;         // wide form: nonzeros per Cg column
constexpr int CP1_ROWS = 16 * CNW * CTP1;   // pass-1 MFMA rows: U + mg <= 320
constexpr int CK_MAX = CP1_ROWS + 4;     // capacitance rows (U + mg <= 320)
constexpr int CH_MAX = 64;     // m + 1 = U - T + 1 <= 64

#ifdef PQ_PROFILE
#define CSTAMP(k)                                                 \
  do {                                                            \
    __syncthreads();                                              \
    if (threadIdx.x == 0) {                                       \
      const long long now_ = wall_clock64();                      \
      pclk[k] += now_ - tclk;                                     \
      tclk = now_;                                                \
    }                                                             \
  } while (0)
#else
#define CSTAMP(k) do { } while (0)
#endif

__device__ __forceinline__ double crho(double l, double u, double rho, const pq_settings& s) {
  if (l == u) return rho * s.eq_scale;
  if (isinf(l) && isinf(u)) return s.rho_min;
  return rho;
}
__device__ __forceinline__ double csum32(double v) {
#pragma unroll
  for (int o = 16; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double cmax32(double v) {
#pragma unroll
  for (int o = 16; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
  return v;
}

// uniform ADMM diagonal d and the group constants of date b (rho = the group's)
struct GConst {
  double c, sqc, d, rho;
};
__device__ __forceinline__ GConst gconst(const pq_lowrank& lr, const pq_problem& pb, const pq_settings& s, int b,
                                         double rho) {
  GConst g;
  g.c = (pb.p_scale ? pb.p_scale[b] : 1.0) * (lr.w_scale ? lr.w_scale[b] : 1.0);
  g.sqc = sqrt(fmax(g.c, 0.0));
  const double pd = pb.p_diag ? pb.p_diag[b] : 0.0;
  const double rb = pb.lb ? crho(pb.lb[(int64_t)b * pb.box_stride], pb.ub[(int64_t)b * pb.box_stride], rho, s) : 0.0;
  g.d = s.sigma + pd + rb;
  g.rho = rho;
  return g;
}

// G_U[u][v] = x_u . x_v from the row band (rows relative to r0)
__device__ __forceinline__ double band_at(const double* band, int64_t ldo, int ru, int rv) {
  if (ru < rv) { const int z = ru; ru = rv; rv = z; }
  return band[(int64_t)ru * ldo + (ru - rv)];
}

// ---- assemble M_U (lower 64-tiles, diagonal tiles in full; identity padding) -----------
__global__ __launch_bounds__(256) void k_gcap_assemble(pq_lowrank lr, pq_problem pb, pq_gcap gc, pq_settings s,
                                                       const double* band, int64_t ldo, int r0, const double* pc,
                                                       int64_t ldpc, const double* cc) {
  __shared__ int s_w[CU_MAX];
  __shared__ double s_sr[CMGW];
  const int grp = blockIdx.x;
  const int d0 = gc.gdates[grp];
  const int U = gc.ucnt[grp], mg = pb.mg, k_ld = gc.k_ld;
  const int t = threadIdx.x, w = wave_id(), l = lane_id();
  for (int u = t; u < U; u += 256) s_w[u] = gc.urows[(int64_t)grp * gc.umax + u] - r0;
  const GConst g = gconst(lr, pb, s, d0, gc.grho[grp]);
  if (t < mg) s_sr[t] = sqrt(crho(pb.lg[t], pb.ug[t], g.rho, s));
  __syncthreads();
  const double a1 = g.c / g.d, a2 = g.sqc / g.d;
  double* M = gc.M + (int64_t)grp * gc.M_stride;
  for (int i = w; i < k_ld; i += 4) {
    const int jend = (i / TB + 1) * TB;
    const bool icg = i >= U && i < U + mg;
    for (int j = l; j < jend; j += 64) {
      double v = (i == j) ? 1.0 : 0.0;
      const bool jcg = j >= U && j < U + mg;
      if (i < U && j < U) v += a1 * band_at(band, ldo, s_w[i], s_w[j]);
      else if (icg && j < U) v += a2 * s_sr[i - U] * pc[(int64_t)s_w[j] * ldpc + (i - U)];
      else if (i < U && jcg) v += a2 * s_sr[j - U] * pc[(int64_t)s_w[i] * ldpc + (j - U)];
      else if (icg && jcg) v += s_sr[i - U] * s_sr[j - U] / g.d * cc[(i - U) * mg + (j - U)];
      M[(int64_t)i * k_ld + j] = v;
    }
  }
}

// ---- preparation, one workgroup per GROUP: a_b, q_b = M_U^-1 a_b, H_b^-1 for its dates ------
// The dates of a group share the union rows, so
//   a_b[u] = sqrt(c) (1/T) sum_{t in window b} G_U[u][t]     (G_U: band Gram of the union)
// is one pass over G_U's rows for all of them (masked sums per date), and Q = M_U^-1 A is one
// MFMA GEMM over the group's dates (the ADMM's z' = M_U^-1 B loop) instead of a symv per date.
// Then per date: mu'mu, a'q, H_b (m + 1 x m + 1) assembled in LDS, its Cholesky, and H_b^-1
// column by column (lane t solves for column t, x in LDS).
// ---- H_b^-1 for 16 < m + 1 <= 32 in one wave's registers: 2 x 2 blocks of 16 ----------------
// Matrices in the MFMA C layout (lane (g4 = l >> 4, cc = l & 15), register q holds
// X[g4 + 4q][cc]).  Register s of X is also the A operand slice s of X' and the B operand
// slice s of X, so sum_s mfma(X[s], Y[s]) = X' Y; a transpose goes through the wave's own
// 16 x 17 LDS tile (wave-local ordering, no workgroup barrier).
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
__device__ __forceinline__ void c_transpose(const double (&X)[4], double (&Xt)[4], double* tile) {
  const int l = lane_id(), cc = l & 15, g4 = l >> 4;
#pragma unroll
  for (int q = 0; q < 4; ++q) tile[(g4 + 4 * q) * 17 + cc] = X[q];
  wave_lds_sync();
#pragma unroll
  for (int q = 0; q < 4; ++q) Xt[q] = tile[cc * 17 + g4 + 4 * q];
  wave_lds_sync();   // (the tile is reused by the next transpose)
}
// acc -/+= X' Y
__device__ __forceinline__ f64x4 c_xty(const double (&X)[4], const double (&Y)[4], f64x4 acc) {
#pragma unroll
  for (int q = 0; q < 4; ++q) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(X[q], Y[q], acc, 0, 0, 0);
  return acc;
}
// H (mh x mh, 16 < mh <= 32, identity padding to 32) given element-wise by h(i, j): H^-1 by
// the blocked Cholesky  L = [[L1, 0], [L21, L2]],  L21 = H21 L1^-T,  L2 L2' = H22 - L21 L21',
// L^-1 = [[W1, 0], [X21, W2]] with X21 = -W2 L21 W1, and H^-1 = L^-T L^-1:
//   (H^-1)_11 = W1'W1 + X21'X21,  (H^-1)_21 = W2'X21,  (H^-1)_22 = W2'W2.
// Two 16-step register chains (wave_chol_inv16) and 32 MFMAs instead of mh sweep steps
// through LDS.  Writes the ldh x ldh output (zeros outside mh x mh); returns 1 (uniform) when
// a pivot is not positive (nothing written).
template <typename HF>
__device__ __forceinline__ int wave_inv32(const HF& h, int mh, double* Hi, int ldh, double* tile) {
  const int l = lane_id(), cc = l & 15, g4 = l >> 4;
  double A[4], W1[4], h12[4], S[4], W2[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int r = g4 + 4 * q;
    A[q] = h(r, cc);
    W1[q] = r == cc ? 1.0 : 0.0;
    h12[q] = 16 + cc < mh ? h(r, 16 + cc) : 0.0;                                  // H12 = H21'
    S[q] = (16 + r < mh && 16 + cc < mh) ? h(16 + r, 16 + cc) : (r == cc ? 1.0 : 0.0);   // H22
    W2[q] = r == cc ? 1.0 : 0.0;
  }
  if (wave_chol_inv16(A, W1)) return 1;
  double W1t[4], L21[4], L21t[4];
  c_transpose(W1, W1t, tile);
  f64x4 acc = c_xty(h12, W1t, f64x4{0.0, 0.0, 0.0, 0.0});                            // L21 = H21 W1'
#pragma unroll
  for (int q = 0; q < 4; ++q) L21[q] = acc[q];
  c_transpose(L21, L21t, tile);
  acc = c_xty(L21t, L21t, f64x4{0.0, 0.0, 0.0, 0.0});                                // L21 L21'
#pragma unroll
  for (int q = 0; q < 4; ++q) S[q] -= acc[q];
  if (wave_chol_inv16(S, W2)) return 1;
  double T1[4], W2t[4], X21[4];
  acc = c_xty(L21t, W1, f64x4{0.0, 0.0, 0.0, 0.0});                                  // T1 = L21 W1
#pragma unroll
  for (int q = 0; q < 4; ++q) T1[q] = acc[q];
  c_transpose(W2, W2t, tile);
  acc = c_xty(W2t, T1, f64x4{0.0, 0.0, 0.0, 0.0});                                   // W2 T1
#pragma unroll
  for (int q = 0; q < 4; ++q) X21[q] = -acc[q];
  const f64x4 i11 = c_xty(X21, X21, c_xty(W1, W1, f64x4{0.0, 0.0, 0.0, 0.0}));
  const f64x4 i21 = c_xty(W2, X21, f64x4{0.0, 0.0, 0.0, 0.0});
  const f64x4 i22 = c_xty(W2, W2, f64x4{0.0, 0.0, 0.0, 0.0});
  for (int e = l; e < ldh * ldh; e += 64)   // entries outside the mh x mh block
    if (e / ldh >= mh || e % ldh >= mh) Hi[e] = 0.0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int r = g4 + 4 * q;
    Hi[(int64_t)r * ldh + cc] = i11[q];
    if (16 + r < mh) {
      Hi[(int64_t)(16 + r) * ldh + cc] = i21[q];
      Hi[(int64_t)cc * ldh + 16 + r] = i21[q];
      if (16 + cc < mh) Hi[(int64_t)(16 + r) * ldh + 16 + cc] = i22[q];
    }
  }
  return 0;
}

constexpr int PT_PREP = 512;    // 8 waves: a row of G_U / a GEMM tile / a date per wave; two
                                // workgroups per CU (44 KB of LDS each) for 16-date groups: all
                                // 475 groups of the config-3 batch in one round instead of two
constexpr int PW_PREP = PT_PREP / 64;

template <int NB>
__global__ __launch_bounds__(PT_PREP, 2 / NB) void k_gcap_prep(pq_lowrank lr, pq_problem pb, pq_state st,
                                                   pq_gcap gc, pq_settings s, const int32_t* idx,
                                                   const double* band, int64_t ldo, int r0, const double* pc,
                                                   int64_t ldpc, int skip) {
  constexpr int CG = CG_MAX * NB;   // dates per group
  __shared__ int s_w[CU_MAX];
  // a_b: row u, column (date) g.  q_b = M_U^-1 a_b goes straight to its output rows (gc.aq),
  // and the inversions of H_b (m + 1 > 16) reuse this array once the GEMM is done (at least
  // the two 64 x 65 tiles of an H_b of m + 1 > 32 and its inverse factor: 65 KB of LDS per
  // 16 dates, two workgroups per CU)
  __shared__ __attribute__((aligned(16))) double s_a[(CK_MAX + 16) * CG > 2 * TB * DP ? (CK_MAX + 16) * CG : 2 * TB * DP];
  static_assert(CH_MAX <= TB, "H_b larger than a 64 x 64 tile");
  __shared__ double s_pref[PW_PREP * (CU_MAX + 64 + 1)];   // a wave's prefix sums of one G_U row
  static_assert(PW_PREP * 16 * 17 <= (CK_MAX + 16) * CG, "the waves' transpose tiles do not fit");
  __shared__ double s_mm[CG], s_aq[CG], s_sr[CMGW];
  __shared__ int s_off[CG], s_T[CG];
  const int slot = xcd_slot(blockIdx.x, gridDim.x);
  const int grp = idx ? idx[slot] : slot;
  const int d0 = gc.gdates[grp];
  const int G = gc.gdates[grp + 1] - d0;
  const int U = gc.ucnt[grp], mg = pb.mg, n = pb.n;
  const int kU = U + mg, k_ld = gc.k_ld;
  const int t = threadIdx.x, w = wave_id(), l = lane_id();
  for (int u = t; u < U; u += PT_PREP) s_w[u] = gc.urows[(int64_t)grp * gc.umax + u] - r0;
  if (t < CG) {
    s_off[t] = t < G ? gc.uoff[d0 + t] : 0;
    s_T[t] = t < G ? lr.tlen[d0 + t] : 1;
  }
  const GConst g = gconst(lr, pb, s, d0, gc.grho[grp]);   // c, d, rho uniform in the group
  if (t < mg) s_sr[t] = sqrt(crho(pb.lg[t], pb.ug[t], g.rho, s));
  const int ktile = (kU + 15) >> 4;
  for (int e = t; e < (CK_MAX + 16) * CG; e += PT_PREP) s_a[e] = 0.0;
  __syncthreads();
  // ---- A: a_b for every date (wave per union row; the row of G_U in registers).  Uncentred
  //      windows (lr.mu null, LeastSquares): no mean column, a_b = q_b = 0 and H_b's last
  //      row / column is the unit vector ------------------------------------------------------
  const bool centred = lr.mu != nullptr;
  // a_b[u] over the window [off_b, off_b + T_b) of the union is a difference of two prefix
  // sums of G_U's row u: per row one wave scan of its U entries into the wave's own LDS row,
  // then lane b (a date) reads its two prefixes -- instead of a masked wave reduction per
  // (row, date): 32 of them per row, 75 % of this kernel (330 of 440 us at config 3).  (The
  // prefix before a window sums at most its < 64 outside rows: the rounding is that of the
  // direct sum's order of magnitude)
  double* const Sw = s_pref + w * (CU_MAX + 64 + 1);
  for (int u = w; centred && !(skip & 1) && u < U; u += PW_PREP) {
    double gv[CU_MAX / 64];
#pragma unroll
    for (int j = 0; j < CU_MAX / 64; ++j) {
      const int v = l + 64 * j;
      gv[j] = v < U ? band_at(band, ldo, s_w[u], s_w[v]) : 0.0;
    }
    double run = 0.0;
#pragma unroll
    for (int j = 0; j < CU_MAX / 64; ++j) {   // inclusive scan of each 64-entry block
      double x = gv[j];
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const double y = __shfl_up(x, o, 64);
        if (l >= o) x += y;
      }
      Sw[64 * j + l + 1] = run + x;          // Sw[v] = sum of the entries before v
      run += readlane_f64(x, 63);
    }
    if (l == 0) Sw[0] = 0.0;
    wave_lds_sync();
    if (l < G) {
      const int lo = s_off[l], T = s_T[l];
      s_a[u * CG + l] = g.sqc * (Sw[lo + T] - Sw[lo]) / T;
    }
    wave_lds_sync();   // (the next row overwrites Sw)
  }
  for (int e = w; centred && e < mg * G; e += PW_PREP) {   // general rows: sqrt(R_r) Cg_r mu_b = sqrt(R_r) (1/T) sum PC
    const int r = e / G, gg = e % G;
    double sum = 0.0;
    for (int tt = l; tt < s_T[gg]; tt += 64) sum += pc[(int64_t)s_w[s_off[gg] + tt] * ldpc + r];
    sum = wave_sum(sum);
    if (l == 0) s_a[(U + r) * CG + gg] = s_sr[r] * sum / s_T[gg];
  }
  __syncthreads();
  // ---- B: Q = M_U^-1 A (MFMA; A rows from the full symmetric M_U^-1, B from LDS).  All row
  //      tiles of a wave in one k loop, the next step's A loads in flight during this step's
  //      MFMAs (unconditional loads from clamped addresses: rows / columns >= kU are M_U^-1's
  //      identity padding, multiplied by the zero rows of s_a) ------------------------------------
  const double* Mi = gc.Minv + (int64_t)grp * gc.M_stride;
  {
    constexpr int QT = (CK_MAX / 16 + 1 + PW_PREP - 1) / PW_PREP;   // row tiles per wave (<= 21 tiles)
    const int kq = l >> 4, m = l & 15;
    const int kU4 = (kU + 7) & ~7;
    f64x4 z[QT][NB];
    const double* mrow[QT];
#pragma unroll
    for (int j = 0; j < QT; ++j) {
      const int row = (w + PW_PREP * j) * 16 + m;
      mrow[j] = Mi + (int64_t)(row < k_ld ? row : 0) * k_ld;
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) z[j][nb] = f64x4{0.0, 0.0, 0.0, 0.0};
    }
    auto loadq = [&](double2 (&a)[QT], int k0) {
      const int kk = k0 + 2 * kq;
      const int kc = kk + 1 < k_ld ? kk : 0;
#pragma unroll
      for (int j = 0; j < QT; ++j) a[j] = *reinterpret_cast<const double2*>(mrow[j] + kc);
    };
    auto mmaq = [&](const double2 (&a)[QT], int k0) {
      const int kk = k0 + 2 * kq;
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) {
        const double b0 = s_a[kk * CG + m + 16 * nb];   // rows >= kU of s_a are zero
        const double b1 = s_a[(kk + 1) * CG + m + 16 * nb];
#pragma unroll
        for (int j = 0; j < QT; ++j) {
          z[j][nb] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[j].x, b0, z[j][nb], 0, 0, 0);
          z[j][nb] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[j].y, b1, z[j][nb], 0, 0, 0);
        }
      }
    };
    double2 qa0[QT], qa1[QT];
    loadq(qa0, 0);
    for (int k0 = 0; !(skip & 2) && k0 < kU4; k0 += 16) {
      loadq(qa1, k0 + 8);
      mmaq(qa0, k0);
      loadq(qa0, k0 + 16);
      if (k0 + 8 < kU4) mmaq(qa1, k0 + 8);
    }
#pragma unroll
    for (int j = 0; j < QT; ++j) {
      const int tile = w + PW_PREP * j;
      if (tile * 16 >= kU) continue;
#pragma unroll
      for (int nb = 0; nb < NB; ++nb)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int u = tile * 16 + kq + 4 * r, md = m + 16 * nb;
          if (u < kU && md < G) gc.aq[(int64_t)(d0 + md) * gc.aq_stride + k_ld + u] = z[j][nb][r];   // q_b
        }
    }
  }
  // ---- a out (q_b's padding rows zero); mu'mu and a'q per date (wave per date) ----------------
  for (int e = t; e < G * k_ld; e += PT_PREP) {
    const int gg = e / k_ld, u = e % k_ld;
    double* A = gc.aq + (int64_t)(d0 + gg) * gc.aq_stride;
    A[u] = u < kU ? s_a[u * CG + gg] : 0.0;
    if (u >= kU) A[k_ld + u] = 0.0;
  }
  __syncthreads();   // (q_b rows written above are read back below)
  auto q_at = [&](int gg, int u) -> double { return gc.aq[(int64_t)(d0 + gg) * gc.aq_stride + k_ld + u]; };
  for (int gg = w; gg < G; gg += PW_PREP) {
    double mm = 0.0, aq = 0.0;
    if (centred) {
      const double* mu = lr.mu + (int64_t)(d0 + gg) * lr.mu_stride;
      for (int i = l; i < n; i += 64) mm = fma(mu[i], mu[i], mm);
    }
    for (int u = l; u < kU; u += 64) aq = fma(s_a[u * CG + gg], q_at(gg, u), aq);
    mm = wave_sum(mm);
    aq = wave_sum(aq);
    if (l == 0) {
      s_mm[gg] = mm;
      s_aq[gg] = aq;
    }
  }
  __syncthreads();
  // ---- C: per date H_b (C = union rows outside [off, off + T)), its Cholesky and H_b^-1 ---------
  const double sct_c = g.c / g.d;
  auto h_entry = [&](int gg, int i, int j) -> double {   // H_b[i][j], i, j < m + 1
    const int T = s_T[gg], off = s_off[gg], m = U - T;
    const double sct = sqrt(g.c * T);
    if (i < m && j < m) {
      const int ci = i < off ? i : i + T, cj = j < off ? j : j + T;
      return Mi[(int64_t)ci * k_ld + cj];
    }
    if (i < m) return -(sct / g.d) * q_at(gg, i < off ? i : i + T);
    if (j < m) return -(sct / g.d) * q_at(gg, j < off ? j : j + T);
    return 1.0 - sct_c * T * (s_mm[gg] - s_aq[gg] / g.d);
  };
  // m + 1 <= 16 (the slide groups' usual case): one wave per date, H in registers (MFMA C
  // layout), Cholesky + L^-1 in one shuffle chain (wave_chol_inv16), H^-1 = L^-T L^-1 by four
  // 16x16x4 MFMAs -- no LDS, no barriers.  16 < m + 1 <= 32 (the outer dates of a 32-date
  // group): the same in 2 x 2 blocks of 16 (wave_inv32; its transposes use the wave's own
  // tile of the a_b array, free since the barrier above).  Formerly the symmetric sweep
  // operator through LDS, mh steps of a lane-per-column loop with wave barriers
  double* tile = s_a + w * (16 * 17);
  for (int gg = w; !(skip & 4) && gg < G; gg += PW_PREP) {
    const int mh = U - s_T[gg] + 1;
    const int b = d0 + gg;
    if (mh > 32) continue;
    if (mh > 16) {
      auto hf = [&](int i, int j) -> double { return h_entry(gg, i, j); };
      if (wave_inv32(hf, mh, gc.hinv + (int64_t)b * gc.ldh * gc.ldh, gc.ldh, tile) && l == 0)
        st.status[b] = PQ_NON_CONVEX;   // not SPD to rounding: no group form for it
      continue;
    }
    const int cc = l & 15, g4 = l >> 4;
    double A[4], Bv[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int r = g4 + 4 * q;
      A[q] = (r < mh && cc < mh) ? h_entry(gg, r, cc) : (r == cc ? 1.0 : 0.0);
      Bv[q] = (r == cc) ? 1.0 : 0.0;
    }
    if (wave_chol_inv16(A, Bv)) {
      if (l == 0) st.status[b] = PQ_NON_CONVEX;   // not SPD to rounding: no group form for it
      continue;
    }
    f64x4 hi = f64x4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int q = 0; q < 4; ++q) hi = __builtin_amdgcn_mfma_f64_16x16x4f64(Bv[q], Bv[q], hi, 0, 0, 0);
    double* Hi = gc.hinv + (int64_t)b * gc.ldh * gc.ldh;
    for (int e = l; e < gc.ldh * gc.ldh; e += 64)   // entries outside the mh x mh block
      if (e / gc.ldh >= mh || e % gc.ldh >= mh) Hi[e] = 0.0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int r = g4 + 4 * q;
      if (r < mh && cc < mh) Hi[(int64_t)r * gc.ldh + cc] = hi[q];
    }
  }
  // m + 1 > 32 (monthly or sparser rebalancing: up to 63 union rows outside a window): the
  // whole workgroup per date, H (identity padding to 64) in LDS, factored and inverted by
  // tile_chol_inv64 (16-column register chains + MFMA panel / trailing / inverse tiles, as
  // the factor's diagonal blocks), then H^-1 = L^-T L^-1 as ten 16 x 16 MFMA tiles over the
  // waves.  Formerly the symmetric sweep operator: mh pivots of two barriers each (~110 us
  // per date of a 13-date monthly batch)
  double* const T64 = s_a;               // H, then L (pitch DP)
  double* const X64 = s_a + TB * DP;     // X[c][r] = (L^-1)[r][c] (pitch DP)
  for (int gg = 0; gg < G; ++gg) {
    const int b = d0 + gg;
    const int mh = U - s_T[gg] + 1;
    if (mh <= 32) continue;   // uniform
    __syncthreads();
    for (int e = t; e < TB * TB; e += PT_PREP) {
      const int i = e >> 6, j = e & 63;
      T64[i * DP + j] = (i < mh && j < mh) ? h_entry(gg, i, j) : (i == j ? 1.0 : 0.0);
    }
    if (tile_chol_inv64(T64, X64, mh)) {   // (uniform; all threads, waves 4.. idle)
      if (t == 0) st.status[b] = PQ_NON_CONVEX;
      continue;
    }
    // (H^-1)[i][j] = sum_r (L^-1)[r][i] (L^-1)[r][j] = sum_r X[i][r] X[j][r]: lower 16 x 16 tiles
    double* Hi = gc.hinv + (int64_t)b * gc.ldh * gc.ldh;
    const int ldh = gc.ldh;
    const int cc = l & 15, g4 = l >> 4;
    for (int tt = w; tt < 10; tt += PW_PREP) {
      int I = 0;
      while ((I + 1) * (I + 2) / 2 <= tt) ++I;
      const int J = tt - I * (I + 1) / 2;
      f64x4 acc = f64x4{0.0, 0.0, 0.0, 0.0};
#pragma unroll 4
      for (int k0 = 0; k0 < TB; k0 += 4)
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(X64[(16 * I + cc) * DP + k0 + g4], X64[(16 * J + cc) * DP + k0 + g4],
                                                  acc, 0, 0, 0);
#pragma unroll
      for (int q = 0; q < 4; ++q) {   // element (16 I + g4 + 4q, 16 J + cc) and its mirror
        const int i = 16 * I + g4 + 4 * q, j = 16 * J + cc;
        const bool in = i < mh && j < mh;
        if (i < ldh && j < ldh) Hi[(int64_t)i * ldh + j] = in ? acc[q] : 0.0;
        if (I != J && i < ldh && j < ldh) Hi[(int64_t)j * ldh + i] = in ? acc[q] : 0.0;
      }
    }
  }
}

// ---- the ADMM iterations -------------------------------------------------------------------
#ifndef PQ_GCAP_SKIP1
#define PQ_GCAP_SKIP1 1   // pass 1 skips the MFMAs of row tiles past the union (0: every tile multiplies)
#endif
// MGC: general rows compiled in (0 for box-only problems: no Cg registers in the epilogue;
// CMGW: the wide form, up to 24 shared rows read column-sparse -- cg_nzr / cg_nzv, nzmax <= CNZ
// nonzeros per asset, e.g. the budget plus one 0/1 sector membership -- instead of as
// register-resident columns)
// NB: MFMA column blocks of 16 dates -- NB = 2 takes up to 32 dates per group with one
// 512-thread workgroup per CU (the CU's union rows streamed once per pass for all of them:
// half the union traffic and half the group factorisations of two 16-date groups); NB = 1 is
// the 256-thread, 16-date form (two workgroups per CU).  The wide form runs NB = 2 as well:
// its per-(date, row) LDS (g_part) is indexed by the date within its wave's column block, so
// k_admm_gcap<CMGW, 2> fits the CU's 160 KiB.
template <int MGC, int NB>
__global__ __launch_bounds__(CT * NB) __attribute__((amdgpu_waves_per_eu(2, 2))) void k_admm_gcap(pq_lowrank lr, pq_problem pb, pq_state st, pq_gcap gc,
                                                  pq_settings s, int iters_call, const double* pc, int64_t ldpc,
                                                  int r0, const double* cc, const int32_t* cg_nzr,
                                                  const double* cg_nzv, int nzmax) {
  constexpr bool WIDE = MGC > CMG;
  // (NB = 2 with the wide form fits the CU's 160 KiB of LDS with g_part indexed by the date
  // within its wave's column block: each wave only ever writes its own block's 16 dates)
  constexpr int MGG = WIDE ? CMGW : 8;
  constexpr int CTN = CT * NB, CNWN = CTN / 64, CHWN = CTN / 32;   // threads, waves, half-waves
  constexpr int CG = CG_MAX * NB;                                   // dates per group
  constexpr int CTP1N = (CP1_ROWS / 16 + CNWN - 1) / CNWN;          // pass-1 row tiles per wave
  constexpr int CTP2N = ((CK_MAX + 15) / 16 + CNWN - 1) / CNWN;     // GEMM row tiles per wave
  static_assert(CTP1N * CNWN * 16 >= CP1_ROWS && CTP2N * CNWN * 16 >= CK_MAX, "k_admm_gcap tiling");
  __shared__ __attribute__((aligned(16))) double WU[(CU_MAX + 4) * CG];
  double* const UT = WU;
  __shared__ double g_muv[CG], g_su[CG], g_dinv[CG], g_rn[CG], g_qmax[CG], g_coef[CG];
  __shared__ double g_y[CG * CH_MAX];   // y_b = H_b^-1 s_b of every date
  constexpr int NPART = 5;                    // per wave and date: 4 maxima, mu.V
  __shared__ double g_part[CNWN * CG_MAX * NPART];   // (wave, date of its column block, slot)
  __shared__ double g_gm[CG * 3];
  // per (date, row); the rows' bounds and rho are shared by the group's dates
  __shared__ double g_zg[CG * MGG], g_yg[CG * MGG], g_cgv[CG * MGG], g_cgx[CG * MGG],
      g_wg[CG * MGG], g_cw[CG * MGG], g_rgz[CG * MGG], g_cmu[CG * MGG];
  __shared__ double g_rg[MGG], g_lg[MGG], g_ug[MGG];
  double* const g_zt = g_rgz;   // Cg x~ of (date, row): read, then overwritten by rho z~, by one lane
  __shared__ int g_act[CG], g_it[CG], g_end[CG], g_stat[CG], g_off[CG], g_T[CG];
  __shared__ int s_urow[CU_MAX];
  __shared__ double s_sr[MGG];
  __shared__ double s_rho;
  __shared__ int s_any;

  const int grp = xcd_slot(blockIdx.x, gridDim.x);
  const int d0 = gc.gdates[grp];
  const int G = gc.gdates[grp + 1] - d0;
  const int U = gc.ucnt[grp];
  const int t = threadIdx.x, w = wave_id(), l = lane_id();
  const int n = pb.n, ld = pb.ld, mg = pb.mg, k_ld = gc.k_ld;
  const int kU = U + mg;
  const bool has_box = pb.lb != nullptr;
  const bool centred = lr.mu != nullptr;   // null: uncentred windows (mu = 0 throughout)
  const double sigma = s.sigma, alpha = s.alpha;
  const double* Mi = gc.Minv + (int64_t)grp * gc.M_stride;
#ifdef PQ_PROFILE
  long long pclk[5] = {0, 0, 0, 0, 0};
  long long tclk = wall_clock64();
#endif

  // a group beyond pass 1's rows (U + mg > CP1_ROWS) or the MFMA N cannot be solved here:
  // its dates fail loudly (status NON_CONVEX, found = False) instead of dropping rows
  // (uniform exit, before any barrier; GroupPlan never builds such a group)
  if (kU > CP1_ROWS || U > CU_MAX || G > CG || kU > k_ld) {
    for (int g = t; g < G; g += CTN) st.status[d0 + g] = PQ_NON_CONVEX;
    return;
  }

  // ---- setup -------------------------------------------------------------------------------
  for (int u = t; u < CU_MAX; u += CTN) s_urow[u] = u < U ? gc.urows[(int64_t)grp * gc.umax + u] : 0;
  for (int e = t; e < (CU_MAX + 4) * CG; e += CTN) UT[e] = 0.0;
  if (t == 0) s_rho = gc.grho[grp];
  __syncthreads();
  const double rho = s_rho;
  const GConst gk = gconst(lr, pb, s, d0, rho);
  if (t < mg) s_sr[t] = sqrt(crho(pb.lg[t], pb.ug[t], rho, s));
  if (t < CG) {
    const int g = t;
    int act = 0;
    if (g < G) {
      const int b = d0 + g;
      const int stt = st.status[b];
      act = (stt == PQ_UNSOLVED || stt == PQ_NEED_REFACTOR);
      g_it[g] = st.iters[b];
      g_end[g] = min(s.max_iter, st.iters[b] + iters_call);
      g_stat[g] = stt;
      g_T[g] = lr.tlen[b];
      g_off[g] = gc.uoff[b];
      g_dinv[g] = 1.0 / gk.d;
    }
    g_act[g] = act;
  }
  for (int e = t; e < CG * MGG; e += CTN) {
    const int g = e / MGG, r = e % MGG;
    double zg = 0, yg = 0;
    if (g < G && r < mg) {
      const int b = d0 + g;
      zg = st.z[(int64_t)b * st.m_ld + r];
      yg = st.y[(int64_t)b * st.m_ld + r];
    }
    g_zg[e] = zg;
    g_yg[e] = yg;
  }
  if (t < MGG) {
    const bool ok = t < mg;
    g_lg[t] = ok ? pb.lg[t] : 0.0;
    g_ug[t] = ok ? pb.ug[t] : 0.0;
    g_rg[t] = ok ? crho(pb.lg[t], pb.ug[t], rho, s) : 0.0;
  }
  __syncthreads();

  const int hg = t >> 5, hl = t & 31;
  const int hbase = (hg & 1) * 32;   // first lane of this half-wave within its wave
#define GC_HPTRS                                                                              \
  const double* __restrict__ q_h = pb.q + (int64_t)hb * pb.q_stride;                          \
  const double* __restrict__ lo_h = has_box ? pb.lb + (int64_t)hb * pb.box_stride : nullptr;  \
  const double* __restrict__ up_h = has_box ? pb.ub + (int64_t)hb * pb.box_stride : nullptr;  \
  const double* __restrict__ Cg_h = mg ? pb.Cg : nullptr;                                     \
  const double* __restrict__ mu_h = centred ? lr.mu + (int64_t)hb * lr.mu_stride : nullptr;   \
  double* __restrict__ x_h = st.x + (int64_t)hb * ld;                                         \
  double* __restrict__ Px_h = st.Px + (int64_t)hb * ld;                                       \
  double* __restrict__ zb_h = st.z + (int64_t)hb * st.m_ld + st.mg_pad;                       \
  double* __restrict__ yb_h = st.y + (int64_t)hb * st.m_ld + st.mg_pad;                       \
  double* __restrict__ R_h = st.work + (int64_t)hb * st.work_stride + ld;                     \
  double* __restrict__ X_h = R_h + ld;                                                        \
  (void)q_h; (void)lo_h; (void)up_h; (void)Cg_h; (void)mu_h; (void)x_h; (void)Px_h;           \
  (void)zb_h; (void)yb_h; (void)R_h; (void)X_h

  // ---- prologue: Cg x, the first rhs, mu.V, Cg.V, Cg.mu (admm_grp.hip's next_rhs, fused) --
  for (int g = hg; g < G; g += CHWN) {
    if (!g_act[g]) continue;
    const int hb = d0 + g;
    GC_HPTRS;
    const double dinv = g_dinv[g];
    for (int r = 0; r < mg; ++r) {
      double a = 0.0, am = 0.0;
      for (int i = hl; i < n; i += 32) {
        a = fma(Cg_h[(int64_t)r * ld + i], x_h[i], a);
        if (centred) am = fma(Cg_h[(int64_t)r * ld + i], mu_h[i], am);
      }
      a = csum32(a);
      am = csum32(am);
      if (hl == 0) {
        g_cgx[g * MGG + r] = a;
        g_cmu[g * MGG + r] = am;
      }
    }
    if (hl < mg) g_wg[g * MGG + hl] = g_rg[hl] * g_zg[g * MGG + hl] - g_yg[g * MGG + hl];
    __builtin_amdgcn_wave_barrier();
    double muv = 0.0, cvp[CMG] = {0.0, 0.0, 0.0, 0.0}, qmax = 0.0;
    for (int i = hl; i < n; i += 32) {
      qmax = fmax(qmax, fabs(q_h[i]));
      const double rb = has_box ? crho(lo_h[i], up_h[i], rho, s) : 0.0;
      double rr = sigma * x_h[i] - q_h[i];
      if (has_box) rr += rb * zb_h[i] - yb_h[i];
      if constexpr (WIDE) {   // column-sparse rows (Cg V of the first iteration: pass 1)
        for (int e = 0; e < nzmax; ++e) {
          const int r = cg_nzr[(int64_t)i * nzmax + e];
          if (r >= 0) rr += cg_nzv[(int64_t)i * nzmax + e] * g_wg[g * MGG + r];
        }
      } else {
#pragma unroll
        for (int r = 0; r < CMG; ++r)
          if (r < mg) rr += Cg_h[(int64_t)r * ld + i] * g_wg[g * MGG + r];
      }
      const double v = rr * dinv;
      R_h[i] = rr;
      if (centred) muv = fma(mu_h[i], v, muv);
      if constexpr (!WIDE) {
#pragma unroll
        for (int r = 0; r < CMG; ++r)
          if (r < mg) cvp[r] = fma(Cg_h[(int64_t)r * ld + i], v, cvp[r]);
      }
    }
    muv = csum32(muv);
    qmax = cmax32(qmax);
#pragma unroll
    for (int r = 0; r < CMG; ++r) cvp[r] = csum32(cvp[r]);
    if (hl == 0) {
      g_muv[g] = muv;
      g_qmax[g] = qmax;   // |q| (dual scale) is fixed over the iterations
      if constexpr (!WIDE)
        for (int r = 0; r < mg; ++r) g_cgv[g * MGG + r] = cvp[r];
    }
  }
  if (t == 0) {
    int any = 0;
    for (int g = 0; g < G; ++g) any |= g_act[g];
    s_any = any;
  }
  __syncthreads();

  const int ntile = (U + mg + 15) >> 4;   // pass 1: union rows, then the general rows (Cg V)
  const int ktile = (kU + 15) >> 4;
  while (s_any) {
    // lane ids re-materialised every iteration (loop_zero): the per-lane LDS / global
    // addresses derived from them are then computed where they are used instead of being
    // hoisted above the loop and spilled to scratch for its whole duration
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Wshadow"
    const int t = threadIdx.x + loop_zero();
    const int w = t >> 6, l = t & 63, hg = t >> 5, hl = t & 31;
    const int hbase = (hg & 1) * 32;
#pragma clang diagnostic pop
    (void)hbase;
    // ---- pass 1: W = X_union V (V = rhs / d, W scaled after the MFMAs); each loaded union
    //      row pair feeds the NB column blocks' MFMAs ------------------------------------------
    {
      const int z0 = loop_zero();
      const int kq = l >> 4, m0 = (l & 15) + z0;
      const double* Vp[NB];
      double wsc1[NB];
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) {
        const int m = m0 + 16 * nb;
        Vp[nb] = (m < G) ? st.work + (int64_t)(d0 + m) * st.work_stride + ld : nullptr;
        wsc1[nb] = m < G ? g_dinv[m] : 1.0;
      }
      f64x4 c[CTP1N][NB];
      const double* arow[CTP1N];
      bool tv[CTP1N], aval[CTP1N];
      const int wu = __builtin_amdgcn_readfirstlane(w);   // (tv: wave-uniform, a scalar branch)
#pragma unroll
      for (int j = 0; j < CTP1N; ++j) {
#pragma unroll
        for (int nb = 0; nb < NB; ++nb) c[j][nb] = f64x4{0.0, 0.0, 0.0, 0.0};
        const int u = (w + CNWN * j) * 16 + m0;
        tv[j] = wu + CNWN * j < ntile;
        aval[j] = u < U + mg;
        arow[j] = u < U ? lr.panel + (int64_t)s_urow[u] * lr.ldp : pb.Cg + (int64_t)(u < U + mg ? u - U : 0) * ld;
      }
      struct Buf { double2 b[NB]; double2 a[CTP1N]; double bs[NB]; };
      // unconditional loads from clamped addresses, no select on a loaded register (see pass 2's
      // load): rows past U + mg and tiles past ntile produce output rows nobody reads, and the
      // columns past n meet a zero V (scaled by 0, after the load)
      const double* Vq[NB];
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) Vq[nb] = Vp[nb] ? Vp[nb] : st.work + (int64_t)d0 * st.work_stride + ld;
      auto load = [&](Buf& f, int k0) {
        const int kk = k0 + 2 * kq;
        const bool kin = kk + 1 < n;
        const int kc = kin ? kk : 0;
#pragma unroll
        for (int nb = 0; nb < NB; ++nb) {
          f.b[nb] = *reinterpret_cast<const double2*>(Vq[nb] + kc);
          f.bs[nb] = (Vp[nb] && kin) ? 1.0 : 0.0;
        }
#pragma unroll
        for (int j = 0; j < CTP1N; ++j) f.a[j] = *reinterpret_cast<const double2*>(arow[j] + kc);
      };
      // tiles past ntile (wave-uniform) skip their MFMAs: 18 row tiles of a 284-row union over
      // 8 waves leave two SIMDs 5 tiles and two 4 instead of 6 each (the loads stay
      // unconditional, from clamped addresses)
      auto mma = [&](const Buf& f) {
#pragma unroll
        for (int nb = 0; nb < NB; ++nb) {
          const double bx = f.b[nb].x * f.bs[nb], by = f.b[nb].y * f.bs[nb];
#pragma unroll
          for (int j = 0; j < CTP1N; ++j) {
            if (PQ_GCAP_SKIP1 && !tv[j]) continue;
            c[j][nb] = __builtin_amdgcn_mfma_f64_16x16x4f64(f.a[j].x, bx, c[j][nb], 0, 0, 0);
            c[j][nb] = __builtin_amdgcn_mfma_f64_16x16x4f64(f.a[j].y, by, c[j][nb], 0, 0, 0);
          }
        }
      };
      Buf f0, f1;
      load(f0, 0);
      for (int k0 = 0; k0 < n; k0 += 16) {
        load(f1, k0 + 8);
        mma(f0);
        load(f0, k0 + 16);
        mma(f1);
      }
      // B operand of the group GEMM in place: rows < U = sqrt(c) W, rows U + r = sqrt(R_r) Cg_r V
#pragma unroll
      for (int j = 0; j < CTP1N; ++j) {
        const int tile = w + CNWN * j;
        if (tv[j]) {
#pragma unroll
          for (int nb = 0; nb < NB; ++nb) {
            const int m = m0 + 16 * nb;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int u = tile * 16 + kq + 4 * r;
              if (u < U) {
                WU[u * CG + m] = gk.sqc * wsc1[nb] * c[j][nb][r];
              } else if (u < U + mg) {   // Cg V of date m
                const double cgv = wsc1[nb] * c[j][nb][r];
                if (m < G) g_cgv[m * MGG + (u - U)] = cgv;
                WU[u * CG + m] = s_sr[u - U] * cgv;
              }
            }
          }
        }
      }
    }
    __syncthreads();
    CSTAMP(0);
    // ---- z' = M_U^-1 B (MFMA, B from LDS).  A = M_U^-1 is symmetric: entries left of the row
    //      tile's diagonal block come from its rows (16-byte pairs), the rest from the
    //      transposed position (rows below, 16 consecutive lanes per row), so only the lower
    //      triangle plus the diagonal blocks is streamed -- about half of the matrix ----------
    {
      const int z0 = loop_zero();
      const int kq = l >> 4, m = (l & 15) + z0;
      f64x4 z[CTP2N][NB];
      const double* mrow[CTP2N];
      bool zv[CTP2N], rv[CTP2N];
#pragma unroll
      for (int j = 0; j < CTP2N; ++j) {
#pragma unroll
        for (int nb = 0; nb < NB; ++nb) z[j][nb] = f64x4{0.0, 0.0, 0.0, 0.0};
        const int row = (w + CNWN * j) * 16 + m;
        zv[j] = w + CNWN * j < ktile;
        rv[j] = row < kU;
        mrow[j] = Mi + (int64_t)(rv[j] ? row : 0) * k_ld;
      }
      const int kU4 = (kU + 7) & ~7;
      // double-buffered: the A loads of step k0 + 8 are in flight during step k0's MFMAs
      // unconditional loads from clamped addresses (see pass 2's load): rows / columns >= kU of
      // M^-1 (k_ld padding) are never read, rows past kU and tiles past ktile produce output
      // rows nobody reads, and B is zero past kU
      auto loadA = [&](double2 (&a)[CTP2N], int k0) {
        const int kk = k0 + 2 * kq;
        const int k0c = kk < kU ? kk : 0, k1c = kk + 1 < kU ? kk + 1 : 0;
#pragma unroll
        for (int j = 0; j < CTP2N; ++j) {
          const int ts = zv[j] ? (w + CNWN * j) * 16 : 0;
          const bool left = kk < ts;   // strictly left of the diagonal block: kk + 1 < ts <= row
          const double* mc = Mi + (ts + m);
          a[j].x = *(left ? mrow[j] + kk : mc + (int64_t)k0c * k_ld);
          a[j].y = *(left ? mrow[j] + kk + 1 : mc + (int64_t)k1c * k_ld);
        }
      };
      auto mmaA = [&](const double2 (&a)[CTP2N], int k0) {
        const int kk = k0 + 2 * kq;
#pragma unroll
        for (int nb = 0; nb < NB; ++nb) {
          const double b0 = kk < kU ? WU[kk * CG + m + 16 * nb] : 0.0;
          const double b1 = kk + 1 < kU ? WU[(kk + 1) * CG + m + 16 * nb] : 0.0;
#pragma unroll
          for (int j = 0; j < CTP2N; ++j) {
            if (zv[j]) {
              z[j][nb] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[j].x, b0, z[j][nb], 0, 0, 0);
              z[j][nb] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[j].y, b1, z[j][nb], 0, 0, 0);
            }
          }
        }
      };
      double2 a0[CTP2N], a1[CTP2N];
      loadA(a0, 0);
      for (int k0 = 0; k0 < kU4; k0 += 16) {
        loadA(a1, k0 + 8);
        mmaA(a0, k0);
        loadA(a0, k0 + 16);
        if (k0 + 8 < kU4) mmaA(a1, k0 + 8);
      }
      __syncthreads();   // every wave is done reading B
#pragma unroll
      for (int j = 0; j < CTP2N; ++j) {
        const int tile = w + CNWN * j;
        if (zv[j]) {
#pragma unroll
          for (int nb = 0; nb < NB; ++nb)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int u = tile * 16 + kq + 4 * r;
              if (u < kU) WU[u * CG + m + 16 * nb] = z[j][nb][r];
            }
        }
      }
    }
    __syncthreads();
    CSTAMP(1);
    // ---- per date: s, y = H^-1 s (half-wave per date) -------------------------------------------
    for (int g = hg; g < G; g += CHWN) {
      if (!g_act[g]) continue;
      const int b = d0 + g;
      const int T = g_T[g], off = g_off[g];
      const int m = U - T, mh = m + 1;
      const double d = gk.d, sct = sqrt(gk.c * T);
      const double* A = gc.aq + (int64_t)b * gc.aq_stride;
      const double* Hi = gc.hinv + (int64_t)b * gc.ldh * gc.ldh;
      double az = 0.0;
      for (int u = hl; u < kU; u += 32) az = fma(A[u], WU[u * CG + g], az);
      az = csum32(az);
      // s: lane j < m holds s_j = z'_{C_j}; lane m (or the last) holds s_mu
      double sj[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int j = hl + 32 * h;
        double v = 0.0;
        if (j < m) {
          const int cj = j < off ? j : j + T;
          v = WU[cj * CG + g];
        } else if (j == m) {
          v = sct * (g_muv[g] - az / d);
        }
        sj[h] = v;
      }
      // y = H^-1 s (H^-1 row i . s): lane i computes y_i for i = hl, hl + 32.  Unconditional
      // loads (rows past mh are H^-1's zero padding, row index clamped to ldh): a conditional
      // load in the loop makes the compiler wait for every outstanding load at each j
      double yi[2] = {0.0, 0.0};
      const int ldh = gc.ldh;
      const double* hr0 = Hi + (int64_t)(hl < ldh ? hl : ldh - 1) * ldh;
      const double* hr1 = Hi + (int64_t)(hl + 32 < ldh ? hl + 32 : ldh - 1) * ldh;
      // 8 steps' row loads issued together, then their FMAs: with the monthly windows' mh up
      // to 64 a load-wait per step (~1 us from L2) dominated the iteration
      int j0 = 0;
      for (; j0 + 8 <= mh; j0 += 8) {
        double h0[8], h1[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          h0[u] = hr0[j0 + u];
          h1[u] = hr1[j0 + u];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int j = j0 + u;
          const double sv = __shfl(j < 32 ? sj[0] : sj[1], hbase + (j & 31), 64);
          yi[0] = fma(h0[u], sv, yi[0]);
          yi[1] = fma(h1[u], sv, yi[1]);
        }
      }
      for (int j = j0; j < mh; ++j) {
        const double sv = __shfl(j < 32 ? sj[0] : sj[1], hbase + (j & 31), 64);
        yi[0] = fma(hr0[j], sv, yi[0]);
        yi[1] = fma(hr1[j], sv, yi[1]);
      }
      const double ymu = __shfl(m < 32 ? yi[0] : yi[1], hbase + (m & 31), 64);
#pragma unroll
      for (int h = 0; h < 2; ++h)
        if (hl + 32 * h < m) g_y[g * CH_MAX + hl + 32 * h] = yi[h];
      if (hl == 0) {
        g_coef[g] = sct / d * ymu;
        g_su[g] = sct * ymu;
        g_gm[g * 3] = g_gm[g * 3 + 1] = g_gm[g * 3 + 2] = 0.0;
      }
    }
    __syncthreads();
    // ---- base = z' - M^-1[:, C_g] y_g + coef_g q_g for every date at once (MFMA): C_g are the
    //      union rows outside date g's window, all among the NH head rows [0, NH) and the tail
    //      rows [T, U) (offsets nondecreasing, off_0 = 0), so it is one (kU x NE) x (NE x 16)
    //      product with NE = NH + U - T edge rows; Ut = sqrt(c) base on union rows, cw =
    //      sqrt(R) base on general rows (in place of z' in WU) -------------------------------------
    {
      const int z0 = loop_zero();
      const int kq = l >> 4, gl0 = (l & 15) + z0;
      const int T0 = g_T[0];
      const int NH = g_off[G - 1], NE = NH + (U - T0);
      bool gact[NB];
      int offg[NB];
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) {
        const int gl = gl0 + 16 * nb;
        gact[nb] = gl < G && g_act[gl];
        offg[nb] = gl < G ? g_off[gl] : 0;
      }
      for (int tile = w; tile < ktile; tile += CNWN) {
        const int ua = tile * 16 + gl0;   // A row of this lane
        f64x4 z[NB];
#pragma unroll
        for (int nb = 0; nb < NB; ++nb) z[nb] = f64x4{0.0, 0.0, 0.0, 0.0};
        // unconditional loads (clamped row / column; rows past kU unused, B zero past NE): the
        // epilogue's q_b entries first, then the A entries of EB steps at a time before their
        // MFMAs -- one step ahead left one load in flight, a memory round trip per step (NE is
        // ~62 for daily windows, ~130 monthly), and the q_b loads under the epilogue's
        // conditions were waited for one by one
        double qv[NB][4];
#pragma unroll
        for (int nb = 0; nb < NB; ++nb) {
          const int gl = gl0 + 16 * nb;
          const double* Q = gc.aq + (int64_t)(d0 + (gl < G ? gl : 0)) * gc.aq_stride + k_ld;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int u = tile * 16 + kq + 4 * r;
            qv[nb][r] = Q[u < kU ? u : 0];
          }
        }
        constexpr int EB = 8;
        for (int e00 = 0; e00 < NE; e00 += 4 * EB) {
          double av[EB];
#pragma unroll
          for (int s = 0; s < EB; ++s) {
            const int e = e00 + 4 * s + kq;
            const int cu = e < NH ? e : T0 + (e - NH);
            av[s] = Mi[(int64_t)(e < NE ? cu : 0) * k_ld + (ua < kU ? ua : 0)];
          }
#pragma unroll
          for (int s = 0; s < EB; ++s) {
            const int e0 = e00 + 4 * s;
            if (e0 >= NE) break;   // (uniform)
            const int e = e0 + kq;
            const int cu = e < NH ? e : T0 + (e - NH);   // union row of edge e
#pragma unroll
            for (int nb = 0; nb < NB; ++nb) {
              const int gl = gl0 + 16 * nb;
              double bv = 0.0;
              if (e < NE && gact[nb]) {
                if (e < NH) bv = e < offg[nb] ? g_y[gl * CH_MAX + e] : 0.0;
                else bv = cu >= offg[nb] + T0 ? g_y[gl * CH_MAX + (cu - T0)] : 0.0;
              }
              z[nb] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[s], bv, z[nb], 0, 0, 0);
            }
          }
        }
        // lane holds rows tile * 16 + kq + 4 r of date gl
#pragma unroll
        for (int nb = 0; nb < NB; ++nb) {
          const int gl = gl0 + 16 * nb;
          if (gact[nb]) {
            const double coef = g_coef[gl];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int u = tile * 16 + kq + 4 * r;
              if (u < kU) {
                const double v = WU[u * CG + gl] - z[nb][r] + coef * qv[nb][r];
                if (u < U) UT[u * CG + gl] = gk.sqc * v;
                else g_cw[gl * MGG + (u - U)] = s_sr[u - U] * v;
              }
            }
          }
        }
      }
    }
    if (MGC > 0) {
      __syncthreads();
      // Cg x~ = Cg V - (PC' Ut - su Cg mu + Cg Cg' cw) / d, then the general rows' z / y
      for (int g = hg; g < G; g += CHWN) {
        if (!g_act[g]) continue;
        const double dinv = g_dinv[g], su = g_su[g];
        for (int r = 0; r < mg; ++r) {
          double a = 0.0;
          for (int u = hl; u < U; u += 32) a = fma(pc[(int64_t)(s_urow[u] - r0) * ldpc + r], UT[u * CG + g], a);
          a = csum32(a);
          double cwv = 0.0;
          for (int r2 = 0; r2 < mg; ++r2) cwv = fma(cc[r * mg + r2], g_cw[g * MGG + r2], cwv);
          if (hl == 0) g_zt[g * MGG + r] = g_cgv[g * MGG + r] - dinv * (a - su * g_cmu[g * MGG + r] + cwv);
        }
        __builtin_amdgcn_wave_barrier();
        double gm[3] = {0.0, 0.0, 0.0};   // |Cx - z| |Cx| |z| of the general rows
        if (hl < mg) {
          const int e = g * MGG + hl;
          const double rg = g_rg[hl], zt = g_zt[e];
          const double zh = alpha * zt + (1.0 - alpha) * g_zg[e];
          const double zn = fmin(fmax(zh + g_yg[e] / rg, g_lg[hl]), g_ug[hl]);
          const double yn = g_yg[e] + rg * (zh - zn);
          const double cx = alpha * zt + (1.0 - alpha) * g_cgx[e];
          gm[0] = fabs(cx - zn);
          gm[1] = fabs(cx);
          gm[2] = fabs(zn);
          g_rgz[e] = rg * zt;
          g_zg[e] = zn;
          g_yg[e] = yn;
          g_cgx[e] = cx;
          g_wg[e] = rg * zn - yn;
        }
#pragma unroll
        for (int k = 0; k < 3; ++k) gm[k] = cmax32(gm[k]);
        if (hl == 0)
          for (int k = 0; k < 3; ++k) g_gm[g * 3 + k] = gm[k];
      }
    }
    __syncthreads();
    CSTAMP(2);
    // ---- pass 2 fused with the per-date updates.  The MFMA computes X~raw as (date x asset)
    //      tiles: lane l ends with dates (l>>4) + 4r, r = 0..3, of the asset pair
    //      p * 32 + 2 (l & 15) + {0, 1}, so the epilogue's per-date vectors (x, Px, z, y,
    //      rhs, q, mu) are read and written as 16-byte pairs by 16 consecutive lanes (256
    //      contiguous bytes per date), and the per-asset data (box, Cg columns) once per
    //      lane for all its dates.  Per-date maxima / sums: lane partials, reduced over the
    //      16 lanes of a date, then NP slots per wave in LDS ---------------------------------
    // With NB = 2 the waves split by column block (waves 0-3: dates 0-15, waves 4-7: dates
    // 16-31), wave w + 4 walking the same asset blocks as wave w at the same time, so the union
    // rows it loads come from L1 / L2 right after wave w's: 4 dates per lane as in the 16-date
    // form (8 per lane spilled the epilogue's registers)
    {
      const int z0 = loop_zero();
      const int kq = l >> 4, ia = (l & 15) + z0;
      const int Uk = (U + 3) & ~3;
      const int cb = w / CNW, wb = w - cb * CNW;   // column block of this wave, wave within it
#ifndef PQ_GCAP_PS
#define PQ_GCAP_PS 4
#endif
      constexpr int PS = PQ_GCAP_PS;   // union rows per pass-2 load step (x 4 lanes)
      // the lane's dates: slot r -> date 16 cb + kq + 4 r
      constexpr int NR = 4;
      bool mact[NR];
#pragma unroll
      for (int r = 0; r < NR; ++r) {
        const int m = 16 * cb + kq + 4 * r;
        mact[r] = m < G && g_act[m];
      }
      const bool box_shared = pb.box_stride == 0;
      // per date of the lane: |x-z|, max(|x|, |z|), |dual res|, max(|Px|, |C'y|) (|q|: prologue;
      // Cg V: next pass 1, as extra MFMA rows)
      double mv[NR][4];
      double muv[NR];
#pragma unroll
      for (int r = 0; r < NR; ++r) {
        muv[r] = 0.0;
#pragma unroll
        for (int e = 0; e < 4; ++e) mv[r][e] = 0.0;
      }
      for (int p = wb; p * 32 < n; p += CNW) {
        const int i = p * 32 + 2 * ia;   // this lane's asset pair (n even: i < n => i + 1 < n)
        const bool cin = i < n;
        f64x4 ce = f64x4{0.0, 0.0, 0.0, 0.0}, co = f64x4{0.0, 0.0, 0.0, 0.0};
        struct ABuf { double2 a[PS]; };
        // unconditional loads from clamped addresses and no select on a loaded register: a
        // conditional load becomes an exec-masked block whose else-branch zeroes the load's
        // destination, a write-after-write that makes the compiler wait for EVERY outstanding
        // load (vmcnt(0)) there -- the double buffer would hide nothing.  Rows past U meet a
        // zero Ut instead, and the columns past n are never used
        auto load = [&](ABuf& f, int u0) {
#pragma unroll
          for (int h = 0; h < PS; ++h) {
            const int u = u0 + 4 * h + kq;
            f.a[h] = *reinterpret_cast<const double2*>(lr.panel + (int64_t)s_urow[u < U ? u : 0] * lr.ldp +
                                                       (cin ? i : 0));
          }
        };
        auto mma = [&](const ABuf& f, int u0) {   // (rows past U: Ut zero; columns past n: unused)
#pragma unroll
          for (int h = 0; h < PS; ++h) {
            const int u = u0 + 4 * h + kq;
            const double av = u < U ? UT[u * CG + 16 * cb + ia] : 0.0;   // Ut'[date 16 cb + ia][u]
            ce = __builtin_amdgcn_mfma_f64_16x16x4f64(av, f.a[h].x, ce, 0, 0, 0);
            co = __builtin_amdgcn_mfma_f64_16x16x4f64(av, f.a[h].y, co, 0, 0, 0);
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
        if (!cin) continue;
        // per-asset data, shared by the lane's dates
        // register-resident columns: MGL of them (0 for the box-only and the wide forms; the
        // arrays keep one slot so they are never zero-length, but no loop reads past MGL --
        // an unread slot must not be read: its register is undefined, and 0 * undefined was
        // folded to garbage that stopped every box-only date after one iteration)
        constexpr int MGL = WIDE ? 0 : MGC;
        constexpr int MGR = MGL > 0 ? MGL : 1;
        double2 cg2[MGR];
#pragma unroll
        for (int c = 0; c < MGL; ++c)
          cg2[c] = c < mg ? *reinterpret_cast<const double2*>(pb.Cg + (int64_t)c * ld + i) : double2{0.0, 0.0};
        int nzr2[2][WIDE ? CNZ : 1];   // wide form: the pair's nonzero rows (-1: none) and values
        double nzv2[2][WIDE ? CNZ : 1];
        if constexpr (WIDE) {
#pragma unroll
          for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int e = 0; e < CNZ; ++e) {
              const bool ok = e < nzmax;
              nzr2[h][e] = ok ? cg_nzr[(int64_t)(i + h) * nzmax + e] : -1;
              nzv2[h][e] = ok ? cg_nzv[(int64_t)(i + h) * nzmax + e] : 0.0;
            }
        }
        double2 lo2 = double2{0.0, 0.0}, up2 = double2{0.0, 0.0}, rb2 = double2{0.0, 0.0};
        if (has_box && box_shared) {
          lo2 = *reinterpret_cast<const double2*>(pb.lb + i);
          up2 = *reinterpret_cast<const double2*>(pb.ub + i);
          rb2 = double2{crho(lo2.x, up2.x, rho, s), crho(lo2.y, up2.y, rho, s)};
        }
#pragma unroll
        for (int r = 0; r < NR; ++r) {
          __builtin_amdgcn_sched_barrier(0);   // one date's loads live at a time (VGPR budget)
          if (!mact[r]) continue;
          const int m = 16 * cb + kq + 4 * r;
          const int bm = d0 + m;
          const double su = g_su[m], dinv = g_dinv[m];
          double2 lo = lo2, up = up2, rb = rb2;
          if (has_box && !box_shared) {
            lo = *reinterpret_cast<const double2*>(pb.lb + (int64_t)bm * pb.box_stride + i);
            up = *reinterpret_cast<const double2*>(pb.ub + (int64_t)bm * pb.box_stride + i);
            rb = double2{crho(lo.x, up.x, rho, s), crho(lo.y, up.y, rho, s)};
          }
          double* R_m = st.work + (int64_t)bm * st.work_stride + ld + i;
          double* x_m = st.x + (int64_t)bm * ld + i;
          double* Px_m = st.Px + (int64_t)bm * ld + i;
          double* zb_m = st.z + (int64_t)bm * st.m_ld + st.mg_pad + i;
          double* yb_m = st.y + (int64_t)bm * st.m_ld + st.mg_pad + i;
          const double2 rr2 = *reinterpret_cast<const double2*>(R_m);
          const double2 mu2 = centred ? *reinterpret_cast<const double2*>(lr.mu + (int64_t)bm * lr.mu_stride + i)
                                      : double2{0.0, 0.0};
          const double2 x2 = *reinterpret_cast<const double2*>(x_m);
          const double2 px2 = *reinterpret_cast<const double2*>(Px_m);
          const double2 q2 = *reinterpret_cast<const double2*>(pb.q + (int64_t)bm * pb.q_stride + i);
          double2 z2 = double2{0.0, 0.0}, y2 = double2{0.0, 0.0};
          if (has_box) {
            z2 = *reinterpret_cast<const double2*>(zb_m);
            y2 = *reinterpret_cast<const double2*>(yb_m);
          }
          double cwm[MGR], rgzm[MGR], ygm[MGR], wgm[MGR];
#pragma unroll
          for (int c = 0; c < MGL; ++c) {
            const bool ok = c < mg;
            cwm[c] = ok ? g_cw[m * MGG + c] : 0.0;
            rgzm[c] = ok ? g_rgz[m * MGG + c] : 0.0;
            ygm[c] = ok ? g_yg[m * MGG + c] : 0.0;
            wgm[c] = ok ? g_wg[m * MGG + c] : 0.0;
          }
          double2 xo, pxo, zo, yo, ro;
          auto one = [&](double xr, double rr0, double mui, double xi, double pxi, double qi, double zi, double yi,
                         double loi, double upi, double rbi, int sel, double& xn_o, double& pxn_o, double& zn_o,
                         double& yn_o, double& rr_o) {
            // wide form: the sums over the asset's nonzero rows (Cg' cw, Cg' rho z~, Cg' y, Cg' w)
            double gcw = 0.0, grgz = 0.0, cgy = 0.0, cgw = 0.0;
            if constexpr (WIDE) {
#pragma unroll
              for (int e = 0; e < CNZ; ++e) {
                const int rw = sel ? nzr2[1][e] : nzr2[0][e];
                if (rw >= 0) {
                  const double v = sel ? nzv2[1][e] : nzv2[0][e];
                  const int o = m * MGG + rw;
                  gcw = fma(g_cw[o], v, gcw);
                  grgz = fma(v, g_rgz[o], grgz);
                  cgy = fma(v, g_yg[o], cgy);
                  cgw = fma(v, g_wg[o], cgw);
                }
              }
            }
            double corr = xr - su * mui + gcw;
            double cgi[MGR];
#pragma unroll
            for (int c = 0; c < MGL; ++c) {
              cgi[c] = sel ? cg2[c].y : cg2[c].x;
              corr = fma(cwm[c], cgi[c], corr);
            }
            const double xt = (rr0 - corr) * dinv;
            double pxt = rr0 - sigma * xt - rbi * xt - grgz;
#pragma unroll
            for (int c = 0; c < MGL; ++c) {
              pxt -= cgi[c] * rgzm[c];
              cgy = fma(cgi[c], ygm[c], cgy);
              cgw = fma(cgi[c], wgm[c], cgw);
            }
            const double xn = alpha * xt + (1.0 - alpha) * xi;
            const double pxn = alpha * pxt + (1.0 - alpha) * pxi;
            double rr = sigma * xn - qi + cgw;
            double cty = 0.0;
            zn_o = zi;
            yn_o = yi;
            if (has_box) {
              const double zh = alpha * xt + (1.0 - alpha) * zi;
              const double zn = fmin(fmax(zh + yi / rbi, loi), upi);
              const double yn = yi + rbi * (zh - zn);
              zn_o = zn;
              yn_o = yn;
              cty = yn;
              rr += rbi * zn - yn;
              mv[r][0] = fmax(mv[r][0], fabs(xn - zn));
              mv[r][1] = fmax(mv[r][1], fmax(fabs(xn), fabs(zn)));
            }
            xn_o = xn;
            pxn_o = pxn;
            rr_o = rr;
            const double cy = cty + cgy;
            mv[r][2] = fmax(mv[r][2], fabs((pxn + qi + cty) + (cy - cty)));
            mv[r][3] = fmax(mv[r][3], fmax(fabs(pxn), fabs(cy)));
            muv[r] = fma(mui, rr * dinv, muv[r]);
          };
          one(ce[r], rr2.x, mu2.x, x2.x, px2.x, q2.x, z2.x, y2.x, lo.x, up.x, rb.x, 0, xo.x, pxo.x, zo.x, yo.x, ro.x);
          one(co[r], rr2.y, mu2.y, x2.y, px2.y, q2.y, z2.y, y2.y, lo.y, up.y, rb.y, 1, xo.y, pxo.y, zo.y, yo.y, ro.y);
          *reinterpret_cast<double2*>(x_m) = xo;
          *reinterpret_cast<double2*>(Px_m) = pxo;
          *reinterpret_cast<double2*>(R_m) = ro;
          if (has_box) {
            *reinterpret_cast<double2*>(zb_m) = zo;
            *reinterpret_cast<double2*>(yb_m) = yo;
          }
        }
      }
      // reduce over the 16 lanes of each date (lanes kq * 16 + 0..15), then one slot per wave
#pragma unroll
      for (int r = 0; r < NR; ++r) {
#pragma unroll
        for (int sh = 1; sh < 16; sh <<= 1) {
#pragma unroll
          for (int e = 0; e < 4; ++e) mv[r][e] = fmax(mv[r][e], __shfl_xor(mv[r][e], sh, 64));
          muv[r] += __shfl_xor(muv[r], sh, 64);
        }
        const int m = 16 * cb + kq + 4 * r;
        if (ia == 0) {
          double* pp = g_part + (w * CG_MAX + (m - 16 * cb)) * NPART;
#pragma unroll
          for (int e = 0; e < 4; ++e) pp[e] = mv[r][e];
          pp[4] = muv[r];
        }
      }
    }
    __syncthreads();
    CSTAMP(3);
    // ---- per date: residuals, convergence, rho request (one thread per date) ------------------
    if (t < G && g_act[t]) {
      const int g = t;
      // mv: |Cx-z| max(|Cx|,|z|) - |dres| max(|Px|,|C'y|) - |q| (the 7-slot form of admm_grp)
      double mv[7] = {g_gm[g * 3], fmax(g_gm[g * 3 + 1], g_gm[g * 3 + 2]), 0.0, 0.0, 0.0, 0.0, g_qmax[g]};
      double muv = 0.0;
      for (int ww = (g / 16) * CNW; ww < (g / 16 + 1) * CNW; ++ww) {   // the waves of g's column block
        const double* pp = g_part + (ww * CG_MAX + (g & 15)) * NPART;
        mv[0] = fmax(mv[0], pp[0]);
        mv[1] = fmax(mv[1], pp[1]);
        mv[3] = fmax(mv[3], pp[2]);
        mv[4] = fmax(mv[4], pp[3]);
        muv += pp[4];
      }
      const int it = g_it[g] + 1;
      int stat = PQ_UNSOLVED;
      // the maxima above are fmax reductions, which drop NaN; muv is a sum over every asset of
      // mu_i (rhs_i / d) and carries a NaN iterate even where mu = 0 (0 * NaN = NaN), so a
      // non-finite iterate cannot pass as converged: it fails the date loudly
      const bool finite = isfinite(muv);
      const double eps_p = s.eps_abs + s.eps_rel * fmax(mv[1], mv[2]);
      const double eps_d = s.eps_abs + s.eps_rel * fmax(mv[4], fmax(mv[5], mv[6]));
      double rn = 0.0;   // this date's rho request (0: none)
      if (!finite) {
        stat = PQ_NON_CONVEX;
      } else if (it >= s.min_iter && mv[0] <= eps_p && mv[3] <= eps_d) {
        stat = PQ_SOLVED;
      } else if (s.adapt_interval > 0 && it % s.adapt_interval == 0) {
        const double rp = mv[0] / (fmax(mv[1], mv[2]) + 1e-30);
        const double rd = mv[3] / (fmax(mv[4], fmax(mv[5], mv[6])) + 1e-30);
        rn = fmin(fmax(rho * sqrt(rp / (rd + 1e-30)), s.rho_min), s.rho_max);
      }
      if (stat == PQ_UNSOLVED && it >= s.max_iter) stat = PQ_MAX_ITER;
      g_it[g] = it;
      g_stat[g] = stat;
      g_act[g] = (stat == PQ_UNSOLVED) && it < g_end[g];
      g_rn[g] = rn;
      g_muv[g] = muv;
    }
    __syncthreads();
    if (t == 0) {
      // group rho: the geometric mean of the requests of the dates that are still running;
      // a change beyond adapt_tol stops them all for one refactorisation of M_U
      double lsum = 0.0;
      int nreq = 0;
      for (int g = 0; g < G; ++g)
        if (g_rn[g] > 0.0 && g_stat[g] == PQ_UNSOLVED) { lsum += log(g_rn[g]); ++nreq; }
      int adapt = 0;
      if (nreq) {
        const double rnew = exp(lsum / nreq);
        if (rnew > rho * s.adapt_tol || rnew < rho / s.adapt_tol) {
          adapt = 1;
          s_rho = rnew;
        }
      }
      int any = 0;
      for (int g = 0; g < G; ++g) {
        g_rn[g] = 0.0;
        if (adapt && g_stat[g] == PQ_UNSOLVED) {
          g_stat[g] = PQ_NEED_REFACTOR;
          g_act[g] = 0;
        }
        any |= g_act[g];
      }
      s_any = any;
    }
    __syncthreads();
    CSTAMP(4);
  }

  // ---- write back ---------------------------------------------------------------------------
  if (t < G) {
    const int b = d0 + t;
    const int stt0 = st.status[b];
    if (stt0 == PQ_UNSOLVED || stt0 == PQ_NEED_REFACTOR) {
      st.iters[b] = g_it[t];
      st.status[b] = g_stat[t];
      st.rho[b] = s_rho;
    }
  }
  if (t == 0) gc.grho[grp] = s_rho;
  for (int e = t; e < CG * MGG; e += CTN) {
    const int g = e / MGG, r = e % MGG;
    if (g < G && r < mg) {
      const int b = d0 + g;
      st.z[(int64_t)b * st.m_ld + r] = g_zg[e];
      st.y[(int64_t)b * st.m_ld + r] = g_yg[e];
    }
  }
#ifdef PQ_PROFILE
  if (t == 0) {   // phase times shared over the group's dates (tools/prof_polish.py --gcap)
    for (int g = 0; g < G; ++g) {
      double* dstp = st.work + (int64_t)(d0 + g) * st.work_stride + PQ_WORK_PROF(ld, st.mg_pad) + 16;
      for (int k2 = 0; k2 < 5; ++k2) dstp[k2] += (double)pclk[k2] / G;
    }
  }
#endif
#undef GC_HPTRS
}

}  // namespace pq

static int gcap_check(const pq_lowrank* lr, const pq_problem* pb, const pq_gcap* gc, const char* who) {
  PQ_CHECK_ARG(lr && pb && gc, "%s: null argument", who);
  PQ_CHECK_ARG(gc->gdates && gc->urows && gc->ucnt && gc->uoff && gc->gidx && gc->grho && gc->ngroups > 0,
               "%s: group plan missing", who);
  PQ_CHECK_ARG(gc->umax > 0 && gc->umax <= pq::CU_MAX, "%s: umax must be in (0, %d]", who, pq::CU_MAX);
  PQ_CHECK_ARG(pb->mg >= 0 && pb->mg <= pq::CMGW && pb->Cg_stride == 0 && pb->g_stride == 0,
               "%s: needs shared general rows, mg <= %d", who, pq::CMGW);
  // (a group with ucnt[g] + mg beyond k_ld or pass 1 fails its dates in k_admm_gcap; U <= umax <= 320)
  PQ_CHECK_ARG(gc->k_ld % 64 == 0 && gc->k_ld >= 64 && gc->k_ld <= 384,
               "%s: need 64 <= k_ld <= 384, a multiple of 64 (k_ld=%d)", who, gc->k_ld);
  PQ_CHECK_ARG(gc->gmax >= 0 && gc->gmax <= pq::CG_MAX * 2, "%s: gmax must be in [0, %d] (gmax=%d)", who,
               pq::CG_MAX * 2, gc->gmax);
  return 0;
}

// column blocks of the group kernels: 2 (32-date groups, one 512-thread workgroup per CU) when
// the plan has groups of more than 16 dates
static int gcap_nb(const pq_gcap* gc) { return gc->gmax > pq::CG_MAX ? 2 : 1; }

extern "C" int pq_gcap_assemble(const pq_lowrank* lr, const pq_problem* pb, const pq_gcap* gc,
                                const pq_settings* s, const double* band, int64_t ldo, int32_t r0,
                                const double* pc, int64_t ldpc, const double* cc, void* stream) {
  if (gcap_check(lr, pb, gc, "pq_gcap_assemble")) return -1;
  PQ_CHECK_ARG(s && band && gc->M, "pq_gcap_assemble: null argument");
  PQ_CHECK_ARG(pb->mg == 0 || (pc && cc), "pq_gcap_assemble: general rows need pc and cc");
  hipLaunchKernelGGL(pq::k_gcap_assemble, dim3(gc->ngroups), dim3(256), 0, (hipStream_t)stream, *lr, *pb, *gc, *s,
                     band, ldo, r0, pc, ldpc, cc);
  PQ_CHECK_LAUNCH("pq_gcap_assemble");
  return 0;
}

extern "C" int pq_gcap_prepare(const pq_lowrank* lr, const pq_problem* pb, pq_state* st, const pq_gcap* gc,
                               const pq_settings* s, const int32_t* idx, int32_t nidx, const double* band,
                               int64_t ldo, int32_t r0, const double* pc, int64_t ldpc, void* stream) {
  if (gcap_check(lr, pb, gc, "pq_gcap_prepare")) return -1;
  PQ_CHECK_ARG(st && s && band && gc->Minv && gc->aq && gc->hinv, "pq_gcap_prepare: null argument");
  PQ_CHECK_ARG(gc->aq_stride >= 2 * (int64_t)gc->k_ld && gc->ldh > 0 && gc->ldh <= pq::CH_MAX,
               "pq_gcap_prepare: aq needs 2 k_ld per date, ldh <= %d", pq::CH_MAX);
  PQ_CHECK_ARG(pb->mg == 0 || pc, "pq_gcap_prepare: general rows need pc");
  PQ_CHECK_ARG(gc->umax <= pq::CU_MAX && pb->mg <= pq::CMGW, "pq_gcap_prepare: union or general rows too many");
  const int grid = idx ? nidx : gc->ngroups;   // one workgroup per group (idx: group subset)
  if (grid <= 0) return 0;
  // PQ_PREP_SKIP (timing experiments only; wrong results): bit 0 skips a_b, bit 1 the
  // M_U^-1 A GEMM, bit 2 the per-date H_b^-1 of m + 1 <= 32
  static const int skip = [] {
    const char* e = getenv("PQ_PREP_SKIP");
    return e ? atoi(e) : 0;
  }();
  if (gcap_nb(gc) == 2)
    hipLaunchKernelGGL(pq::k_gcap_prep<2>, dim3(grid), dim3(pq::PT_PREP), 0, (hipStream_t)stream, *lr, *pb, *st, *gc,
                       *s, idx, band, ldo, r0, pc, ldpc, skip);
  else
    hipLaunchKernelGGL(pq::k_gcap_prep<1>, dim3(grid), dim3(pq::PT_PREP), 0, (hipStream_t)stream, *lr, *pb, *st, *gc,
                       *s, idx, band, ldo, r0, pc, ldpc, skip);
  PQ_CHECK_LAUNCH("pq_gcap_prepare");
  return 0;
}

extern "C" int pq_admm_lr_gcap(const pq_lowrank* lr, const pq_problem* pb, pq_state* st, const pq_gcap* gc,
                               const pq_settings* s, int32_t iters_this_call, const double* pc, int64_t ldpc,
                               int32_t r0, const double* cc, const int32_t* cg_nzr, const double* cg_nzv,
                               int32_t nzmax, void* stream) {
  if (gcap_check(lr, pb, gc, "pq_admm_lr_gcap")) return -1;
  PQ_CHECK_ARG(st && s && gc->Minv && gc->aq && gc->hinv, "pq_admm_lr_gcap: null argument");
  PQ_CHECK_ARG(pb->mg == 0 || (pc && cc), "pq_admm_lr_gcap: general rows need pc and cc");
  PQ_CHECK_ARG(pb->n % 2 == 0 && lr->ldp % 2 == 0, "pq_admm_lr_gcap: needs even n and panel stride");
  PQ_CHECK_ARG(st->work && st->work_stride >= 3 * (int64_t)pb->ld, "pq_admm_lr_gcap: work buffer too small");
  // 16-byte pair access of the per-date vectors
  PQ_CHECK_ARG(pb->ld % 2 == 0 && st->work_stride % 2 == 0 && st->m_ld % 2 == 0 && st->mg_pad % 2 == 0 &&
                   pb->q_stride % 2 == 0 && pb->box_stride % 2 == 0 && lr->mu_stride % 2 == 0,
               "pq_admm_lr_gcap: strides must be even");
  PQ_CHECK_ARG(pb->mg <= pq::CMG || (cg_nzr && cg_nzv && nzmax > 0 && nzmax <= pq::CNZ),
               "pq_admm_lr_gcap: more than %d general rows need their column-sparse form (nzmax <= %d)", pq::CMG,
               pq::CNZ);
  const dim3 grid(gc->ngroups);
  const hipStream_t str = (hipStream_t)stream;
  if (gcap_nb(gc) == 2) {   // 32-date groups (one 512-thread workgroup per group)
    const dim3 blk(pq::CT * 2);
    if (pb->mg == 0)
      hipLaunchKernelGGL((pq::k_admm_gcap<0, 2>), grid, blk, 0, str, *lr, *pb, *st, *gc, *s, iters_this_call, pc, ldpc,
                         r0, cc, nullptr, nullptr, 0);
    else if (pb->mg == 1)
      hipLaunchKernelGGL((pq::k_admm_gcap<1, 2>), grid, blk, 0, str, *lr, *pb, *st, *gc, *s, iters_this_call, pc, ldpc,
                         r0, cc, nullptr, nullptr, 0);
    else if (pb->mg <= pq::CMG)
      hipLaunchKernelGGL((pq::k_admm_gcap<pq::CMG, 2>), grid, blk, 0, str, *lr, *pb, *st, *gc, *s, iters_this_call, pc,
                         ldpc, r0, cc, nullptr, nullptr, 0);
    else   // budget + sector caps, column-sparse (config 4): the union streamed once for 32 dates
      hipLaunchKernelGGL((pq::k_admm_gcap<pq::CMGW, 2>), grid, blk, 0, str, *lr, *pb, *st, *gc, *s, iters_this_call, pc,
                         ldpc, r0, cc, cg_nzr, cg_nzv, nzmax);
  } else {
    const dim3 blk(pq::CT);
    if (pb->mg == 0)
      hipLaunchKernelGGL((pq::k_admm_gcap<0, 1>), grid, blk, 0, str, *lr, *pb, *st, *gc, *s, iters_this_call, pc, ldpc,
                         r0, cc, nullptr, nullptr, 0);
    else if (pb->mg == 1)   // the budget row alone (the usual case): one general row in registers
      hipLaunchKernelGGL((pq::k_admm_gcap<1, 1>), grid, blk, 0, str, *lr, *pb, *st, *gc, *s, iters_this_call, pc, ldpc,
                         r0, cc, nullptr, nullptr, 0);
    else if (pb->mg <= pq::CMG)
      hipLaunchKernelGGL((pq::k_admm_gcap<pq::CMG, 1>), grid, blk, 0, str, *lr, *pb, *st, *gc, *s, iters_this_call, pc,
                         ldpc, r0, cc, nullptr, nullptr, 0);
    else   // budget + sector caps: column-sparse rows
      hipLaunchKernelGGL((pq::k_admm_gcap<pq::CMGW, 1>), grid, blk, 0, str, *lr, *pb, *st, *gc, *s, iters_this_call, pc,
                         ldpc, r0, cc, cg_nzr, cg_nzv, nzmax);
  }
  PQ_CHECK_LAUNCH("pq_admm_lr_gcap");
  return 0;
}
