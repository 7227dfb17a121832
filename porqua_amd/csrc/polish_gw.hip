// K4, wide rounds of the grouped polish: dates whose free set is too large for the LDS
// Cholesky of polish_g.hip (tracking least squares at n = 3000: every variable free, P of
// rank T) solve the round's regularised KKT system in n-space,
//     [K  B'] [dx  ]   [r ]      K = P + d I,  r = -q - P x - B' lam,
//     [B -dI] [dlam] = [rl],     rl = rhs_B - B x,
// with B the bordered rows -- the active general rows and the variables held at a bound
// (unit rows) -- and d = p_diag + grho[g] one value per slide group.  K_b differs between
// the dates of a group only by the union rows outside each window, so K_b^-1 is the group
// capacitance of admm_gcap.hip (M_U^-1 of the union plus a per-date Woodbury correction
// H_b^-1) built once per polish call for the polish diagonal, and every window product of
// the refinement is an FP64 MFMA pass over the group's union rows for all 16 dates at once:
//     a) exact residual:  X_U x (pass 1, with the general rows C x), masked / centred,
//                          X_U' w (pass 2) -> P x, r, and the convergence test;
//     b) correction:      t = K^-1 r (pass 1 of r, M_U^-1 GEMM, Woodbury correction),
//                          S dlam = B t - rl with S = B K^-1 B' + delta I (per date, from
//                          the bordered rows' own K^-1 images computed once per round),
//                          dx = K^-1 (r - B' dlam) (pass 2), x += dx, lam += dlam.
// That is polish_w.hip's Woodbury mode (same regularised system, same refinement, same
// tolerances) with the window passes shared by the group's dates instead of repeated per
// date.  The exact P x / checks / scoring of the round follow in polish_g.hip's passes.
//
// Replaces, with polish_g.hip, the accuracy of qpsolvers' interior-point answer
// (src/qp_problems.py:211-214).
#include "common.h"
#include "capi_util.h"
#include "pg_record.h"

namespace pq {

constexpr int YT = 256;          // threads per group workgroup
constexpr int YNW = YT / 64;
constexpr int YHW = YT / 32;     // half-waves
constexpr int YG = 16;           // dates per group (MFMA N)
constexpr int YP1 = 5;           // pass-1 row tiles per wave: union + general rows <= 320
constexpr int YU = 16 * YNW * YP1;
constexpr int YP2 = 6;           // GEMM row tiles per wave: k_ld <= 384
constexpr int YMB = PG_WMB;      // bordered rows per date
constexpr int YMG = PG_WG_MAX;   // general rows
constexpr int YCH = 64;          // Woodbury correction rank U - T + 1
constexpr int YNP = 3;           // per-date partials of a pass-2 epilogue

__device__ __forceinline__ double ysum32(double v) {
#pragma unroll
  for (int o = 16; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__global__ __launch_bounds__(YT) __attribute__((amdgpu_waves_per_eu(2, 2))) void k_pgw(
    pq_lowrank lr, pq_problem pb, pq_state st, pq_gcap gc, double* rec, pq_settings s, const double* pc,
    int64_t ldpc, int r0, const double* cc, const int32_t* nzr, const double* nzv, int nzmax, double* wscr,
    int64_t wstride, int nref) {
  __shared__ __attribute__((aligned(16))) double WU[(YU + 4) * YG];
  __shared__ int s_urow[YU];
  __shared__ double g_y[YG * YCH];
  __shared__ double g_S[YG * YMB * YMB];
  __shared__ double g_lam[YG * YMB], g_dlam[YG * YMB], g_rl[YG * YMB], g_dB[YG * YMB], g_bmu[YG * YMB],
      g_sub[YG * YMB];
  __shared__ int g_bid[YG * YMB];   // bordered row: general row r >= 0, or -1 - i for variable i
  __shared__ double g_cx[YG * YMG], g_lamd[YG * YMG], g_dlamd[YG * YMG];
  __shared__ double g_part[YNW * YG * YNP];
  __shared__ double g_mux[YG], g_mur[YG], g_sw[YG], g_su[YG], g_coef[YG], g_sc[YG], g_muv[YG];
  __shared__ int g_on[YG], g_T[YG], g_off[YG], g_mb[YG], g_ma[YG], g_run[YG];
  __shared__ int c_date[YG], c_j[YG];
  __shared__ int s_any, s_ncol;

  const int grp = xcd_slot(blockIdx.x, gridDim.x);
  const int d0 = gc.gdates[grp];
  const int G = gc.gdates[grp + 1] - d0;
  const int U = gc.ucnt[grp];
  const int t = threadIdx.x, w = wave_id(), l = lane_id();
  const int n = pb.n, ld = pb.ld, mg = pb.mg, k_ld = gc.k_ld;
  const bool centred = lr.mu != nullptr;
  const double c = (pb.p_scale ? pb.p_scale[d0] : 1.0) * (lr.w_scale ? lr.w_scale[d0] : 1.0);
  const double sqc = sqrt(fmax(c, 0.0));
  const double pd = pb.p_diag ? pb.p_diag[d0] : 0.0;
  const double d = pd + gc.grho[grp], dinv = 1.0 / d;
  const double* Mi = gc.Minv + (int64_t)grp * gc.M_stride;
  const int hg = t >> 5, hl = t & 31;
  const int hbase = (hg & 1) * 32;

  // a group whose union + general rows exceed pass 1's YU rows (or whose dates exceed YG)
  // cannot be solved here: its pending dates go to the per-date kernel (uniform exit, before
  // any barrier)
  if (U + mg > YU || G > YG) {
    for (int j = t; j < G; j += YT) {
      double* R = rec + (int64_t)(d0 + j) * PGR;
      if (R[R_STATE] == PQ_PG_PENDING) R[R_STATE] = PQ_PG_FALLBACK;
    }
    return;
  }

  // ---- setup ---------------------------------------------------------------------------
  for (int u = t; u < YU; u += YT) s_urow[u] = u < U ? gc.urows[(int64_t)grp * gc.umax + u] : 0;
  for (int e = t; e < (YU + 4) * YG; e += YT) WU[e] = 0.0;
  if (t < YG) {
    int on = 0;
    if (t < G) {
      const double* R = rec + (int64_t)(d0 + t) * PGR;
      on = R[R_STATE] == PQ_PG_PENDING && R[R_W] == 1.0;
      g_T[t] = lr.tlen[d0 + t];
      g_off[t] = gc.uoff[d0 + t];
      g_ma[t] = on ? (int)R[R_MA] : 0;
      g_mb[t] = on ? (int)R[R_MA] + (int)R[R_NFX] : 0;
      g_sc[t] = R[R_SC];
    } else {
      g_T[t] = 1;
      g_off[t] = 0;
      g_ma[t] = g_mb[t] = 0;
      g_sc[t] = 1.0;
    }
    g_on[t] = on;
    g_run[t] = on;
  }
  __syncthreads();
  if (t == 0) {
    int any = 0, nc = 0;
    for (int g = 0; g < G; ++g) {
      any |= g_on[g];
      nc += g_mb[g];
    }
    s_any = any;
    s_ncol = nc;
  }
  for (int e = t; e < YG * YMG; e += YT) g_lamd[e] = g_dlamd[e] = 0.0;
  __syncthreads();
  if (!s_any) return;
  for (int e = t; e < YG * YMB; e += YT) {
    const int g = e / YMB, j = e % YMB;
    int bid = 0;
    double dB = 0.0, lam = 0.0;
    if (g_on[g] && j < g_mb[g]) {
      const double* R = rec + (int64_t)(d0 + g) * PGR;
      if (j < g_ma[g]) {
        bid = (int)R[R_AL + j];
        dB = R[R_DA + j];
        lam = R[R_SOL + j];
        g_lamd[g * YMG + bid] = lam;
      } else {
        const int jf = j - g_ma[g];
        bid = -1 - (int)R[R_FIX + jf];
        dB = R[R_FIXV + jf];
        lam = R[R_FXL + jf];
      }
    }
    g_bid[e] = bid;
    g_dB[e] = dB;
    g_lam[e] = lam;
  }
  __syncthreads();
  // beta_j . mu (half-wave per (date, bordered row)) and mu . x (half-wave per date)
  for (int e = hg; e < YG * YMB; e += YHW) {
    const int g = e / YMB, j = e % YMB;
    if (!g_on[g] || j >= g_mb[g]) continue;
    const double* mu = centred ? lr.mu + (int64_t)(d0 + g) * lr.mu_stride : nullptr;
    const int bid = g_bid[e];
    double v = 0.0;
    if (mu) {
      if (bid >= 0) {
        const double* cr = pb.Cg + (int64_t)bid * ld;
        for (int i = hl; i < n; i += 32) v = fma(cr[i], mu[i], v);
        v = ysum32(v);
      } else {
        v = mu[-1 - bid];
      }
    }
    if (hl == 0) g_bmu[e] = v;
  }
  for (int g = hg; g < YG; g += YHW) {
    double v = 0.0;
    if (g_on[g] && centred) {
      const double* mu = lr.mu + (int64_t)(d0 + g) * lr.mu_stride;
      const double* x = st.work + (int64_t)(d0 + g) * st.work_stride;   // PGWork xs
      for (int i = hl; i < n; i += 32) v = fma(mu[i], x[i], v);
      v = ysum32(v);
    }
    if (hl == 0) g_mux[g] = v;
  }
  __syncthreads();

  // ---- building blocks -------------------------------------------------------------------
  // pass 1: WU[u][m] = vscale(m) (X_U V_m)[u] for the union rows, g_cx[m][r] = Cg_r . V_m
  // for the general rows (rows U .. U + mgp of the same MFMA image)
  auto pass1 = [&](auto vptr, auto vscale, int mgp) {
    const int z0 = loop_zero();
    const int kq = l >> 4, m = (l & 15) + z0;
    const double* Vp = vptr(m);
    const double wsc = Vp ? vscale(m) : 0.0;
    const int ntile = (U + mgp + 15) >> 4;
    f64x4 cacc[YP1];
    const double* arow[YP1];
    bool tv[YP1], aval[YP1];
#pragma unroll
    for (int j = 0; j < YP1; ++j) {
      cacc[j] = f64x4{0.0, 0.0, 0.0, 0.0};
      const int uu = (w + YNW * j) * 16 + m;
      tv[j] = w + YNW * j < ntile;
      aval[j] = uu < U + mgp;
      arow[j] = uu < U ? lr.panel + (int64_t)s_urow[uu] * lr.ldp : pb.Cg + (int64_t)(uu < U + mgp ? uu - U : 0) * ld;
    }
    // unconditional loads from clamped addresses, V scaled to zero past n / for empty columns
    // (a conditional load makes the compiler wait for every outstanding load at each step);
    // rows past U + mgp give unused outputs
    const double* Vq = Vp ? Vp : lr.panel;
    for (int k0 = 0; k0 < n; k0 += 8) {
      const int kk = k0 + 2 * kq;
      const bool kin = kk + 1 < n;
      const int kc = kin ? kk : 0;
      const double2 bl = *reinterpret_cast<const double2*>(Vq + kc);
      double2 av[YP1];
#pragma unroll
      for (int j = 0; j < YP1; ++j) av[j] = *reinterpret_cast<const double2*>(arow[j] + kc);
      const double sb = (Vp && kin) ? 1.0 : 0.0;
      const double bx = bl.x * sb, by = bl.y * sb;
#pragma unroll
      for (int j = 0; j < YP1; ++j) {
        cacc[j] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[j].x, bx, cacc[j], 0, 0, 0);
        cacc[j] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[j].y, by, cacc[j], 0, 0, 0);
      }
    }
    __syncthreads();   // the previous contents of WU are no longer read
#pragma unroll
    for (int j = 0; j < YP1; ++j) {
      const int tile = w + YNW * j;
      if (tv[j]) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int u = tile * 16 + kq + 4 * r;
          if (u < U) WU[u * YG + m] = wsc * cacc[j][r];
          else if (u < U + mgp) g_cx[m * YMG + (u - U)] = cacc[j][r];
        }
      }
    }
    __syncthreads();
  };
  // z' = M_U^-1 WU in place (the lower triangle of the symmetric M_U^-1 streamed, as in
  // admm_gcap.hip)
  auto gemm = [&]() {
    const int z0 = loop_zero();
    const int kq = l >> 4, m = (l & 15) + z0;
    const int ktile = (U + 15) >> 4;
    f64x4 z[YP2];
    const double* mrow[YP2];
    bool zv[YP2], rv[YP2];
#pragma unroll
    for (int j = 0; j < YP2; ++j) {
      z[j] = f64x4{0.0, 0.0, 0.0, 0.0};
      const int row = (w + YNW * j) * 16 + m;
      zv[j] = w + YNW * j < ktile;
      rv[j] = row < U;
      mrow[j] = Mi + (int64_t)(rv[j] ? row : 0) * k_ld;
    }
    const int kU4 = (U + 7) & ~7;
    for (int k0 = 0; k0 < kU4; k0 += 8) {
      const int kk = k0 + 2 * kq;
      const bool kin = kk < U, kin1 = kk + 1 < U;
      const double b0 = kin ? WU[kk * YG + m] : 0.0;
      const double b1 = kin1 ? WU[(kk + 1) * YG + m] : 0.0;
      // unconditional loads from clamped addresses (B is zero past U; rows past U and tiles
      // past ktile give unused outputs), as admm_gcap.hip's GEMM
      const int k0c = kin ? kk : 0, k1c = kin1 ? kk + 1 : 0;
#pragma unroll
      for (int j = 0; j < YP2; ++j) {
        const int ts = zv[j] ? (w + YNW * j) * 16 : 0;
        const bool left = kk < ts;
        const double* mc = Mi + (ts + m);
        double2 a;
        a.x = *(left ? mrow[j] + kk : mc + (int64_t)k0c * k_ld);
        a.y = *(left ? mrow[j] + kk + 1 : mc + (int64_t)k1c * k_ld);
        if (!zv[j]) continue;
        z[j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a.x, b0, z[j], 0, 0, 0);
        z[j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a.y, b1, z[j], 0, 0, 0);
      }
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < YP2; ++j) {
      const int tile = w + YNW * j;
      if (zv[j]) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int u = tile * 16 + kq + 4 * r;
          if (u < U) WU[u * YG + m] = z[j][r];
        }
      }
    }
    __syncthreads();
  };
  // Woodbury correction of the 16 columns (column m belongs to date cdate(m), -1: none; its
  // mu . V is cmuv(m)): WU <- Ut = sqrt(c) (z' - M^-1[:, C] y_C + coef q_b) on the union rows,
  // g_su[m] = sqrt(cT) y_mu
  auto correct = [&](auto cdate, auto cmuv) {
    for (int m = hg; m < YG; m += YHW) {
      const int gd = cdate(m);
      if (gd < 0) continue;
      const int b = d0 + gd;
      const int T = g_T[gd], off = g_off[gd];
      const int mm = U - T, mh = mm + 1;
      const double sct = sqrt(c * T);
      const double* A = gc.aq + (int64_t)b * gc.aq_stride;
      const double* Hi = gc.hinv + (int64_t)b * gc.ldh * gc.ldh;
      double az = 0.0;
      if (centred)
        for (int u = hl; u < U; u += 32) az = fma(A[u], WU[u * YG + m], az);
      az = ysum32(az);
      double sj[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int j = hl + 32 * h;
        double v = 0.0;
        if (j < mm) v = WU[(j < off ? j : j + T) * YG + m];
        else if (j == mm) v = sct * (cmuv(m) - az * dinv);
        sj[h] = v;
      }
      double yi[2] = {0.0, 0.0};
      for (int j = 0; j < mh; ++j) {
        const double sv = __shfl(j < 32 ? sj[0] : sj[1], hbase + (j & 31), 64);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int i = hl + 32 * h;
          if (i < mh) yi[h] = fma(Hi[(int64_t)i * gc.ldh + j], sv, yi[h]);
        }
      }
      const double ymu = __shfl(mm < 32 ? yi[0] : yi[1], hbase + (mm & 31), 64);
#pragma unroll
      for (int h = 0; h < 2; ++h)
        if (hl + 32 * h < mm) g_y[m * YCH + hl + 32 * h] = yi[h];
      if (hl == 0) {
        g_coef[m] = sct * dinv * ymu;
        g_su[m] = sct * ymu;
      }
    }
    __syncthreads();
    {
      const int z0 = loop_zero();
      const int kq = l >> 4, gl = (l & 15) + z0;
      const int T0 = g_T[0];
      const int NH = g_off[G - 1], NE = NH + (U - T0);
      const int gd = cdate(gl);
      const bool gact = gd >= 0;
      const int offg = gact ? g_off[gd] : 0;
      const double coef = gact ? g_coef[gl] : 0.0;
      const double* Q = gact ? gc.aq + (int64_t)(d0 + gd) * gc.aq_stride + k_ld : nullptr;
      const int ktile = (U + 15) >> 4;
      for (int tile = w; tile < ktile; tile += YNW) {
        const int ua = tile * 16 + gl;
        f64x4 z = f64x4{0.0, 0.0, 0.0, 0.0};
        for (int e0 = 0; e0 < NE; e0 += 4) {
          const int e = e0 + kq;
          const int cu = e < NH ? e : T0 + (e - NH);
          // unconditional load (clamped row / column; rows past U unused, B zero past NE)
          const double av = Mi[(int64_t)(e < NE ? cu : 0) * k_ld + (ua < U ? ua : 0)];
          double bv = 0.0;
          if (e < NE && gact) {
            if (e < NH) bv = e < offg ? g_y[gl * YCH + e] : 0.0;
            else bv = cu >= offg + T0 ? g_y[gl * YCH + (cu - T0)] : 0.0;
          }
          z = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, z, 0, 0, 0);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int u = tile * 16 + kq + 4 * r;
          if (u < U) {
            const double v = gact ? WU[u * YG + gl] - z[r] + (centred ? coef * Q[u] : 0.0) : 0.0;
            WU[u * YG + gl] = sqc * v;
          }
        }
      }
    }
    __syncthreads();
  };
  // pass 2: X_U' WU for every column, epilogue ep(m, i, v_i, v_i+1, part) per date m of the
  // lane and asset pair (i, i + 1); part[YNP]: the lane's per-date partials (summed over the
  // lanes of the date into g_part, max for slot 0)
  auto pass2 = [&](auto ep) {
    const int z0 = loop_zero();
    const int kq = l >> 4, ia = (l & 15) + z0;
    const int Uk = (U + 3) & ~3;
    double part[4][YNP];
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int e = 0; e < YNP; ++e) part[r][e] = 0.0;
    for (int p = w; p * 32 < n; p += YNW) {
      const int i = p * 32 + 2 * ia;
      const bool cin = i < n;
      f64x4 ce = f64x4{0.0, 0.0, 0.0, 0.0}, co = f64x4{0.0, 0.0, 0.0, 0.0};
      // unconditional loads (rows past U meet zero in WU's padding rows, columns past n are
      // unused), four union-row steps' loads issued before their MFMAs
      const int ic = cin ? i : 0;
      for (int u0 = 0; u0 < Uk; u0 += 16) {
        double2 a[4];
#pragma unroll
        for (int h = 0; h < 4; ++h) {
          const int u = u0 + 4 * h + kq;
          a[h] = *reinterpret_cast<const double2*>(lr.panel + (int64_t)s_urow[u < U ? u : 0] * lr.ldp + ic);
        }
#pragma unroll
        for (int h = 0; h < 4; ++h) {
          const int u = u0 + 4 * h + kq;
          const double av = u < U ? WU[u * YG + ia] : 0.0;
          ce = __builtin_amdgcn_mfma_f64_16x16x4f64(av, a[h].x, ce, 0, 0, 0);
          co = __builtin_amdgcn_mfma_f64_16x16x4f64(av, a[h].y, co, 0, 0, 0);
        }
      }
      if (!cin) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = kq + 4 * r;
        if (m < G && g_run[m]) ep(m, i, ce[r], co[r], part[r]);
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
#pragma unroll
      for (int sh = 1; sh < 16; sh <<= 1) {
        part[r][0] = fmax(part[r][0], __shfl_xor(part[r][0], sh, 64));
#pragma unroll
        for (int e = 1; e < YNP; ++e) part[r][e] += __shfl_xor(part[r][e], sh, 64);
      }
      const int m = kq + 4 * r;
      if (ia == 0)
#pragma unroll
        for (int e = 0; e < YNP; ++e) g_part[(w * YG + m) * YNP + e] = part[r][e];
    }
    __syncthreads();
  };
  // sum_r C_ri v_r over the general rows (dense rows, or their column-sparse form)
  auto crow = [&](int i, const double* v) -> double {
    double sum = 0.0;
    if (nzmax > 0) {
      for (int e = 0; e < nzmax; ++e) {
        const int r = nzr[(int64_t)i * nzmax + e];
        if (r >= 0) sum = fma(nzv[(int64_t)i * nzmax + e], v[r], sum);
      }
    } else {
      for (int r = 0; r < mg; ++r) sum = fma(pb.Cg[(int64_t)r * ld + i], v[r], sum);
    }
    return sum;
  };

  // ---- the bordered rows' images: Ut_j, su_j (K^-1 beta_j' in union form) and X_U beta_j' ----
  for (int c0 = 0; c0 < s_ncol; c0 += YG) {
    if (t == 0) {   // columns c0 .. c0 + 15 of the (date, row) enumeration
      int cidx = 0;
      for (int g = 0; g < G; ++g)
        for (int j = 0; j < g_mb[g]; ++j, ++cidx)
          if (cidx >= c0 && cidx < c0 + YG) {
            c_date[cidx - c0] = g;
            c_j[cidx - c0] = j;
          }
      for (int m = (s_ncol - c0 < YG ? s_ncol - c0 : YG); m < YG; ++m) c_date[m] = -1;
    }
    __syncthreads();
    for (int e = t; e < U * YG; e += YT) {   // B operand sqrt(c) X_U beta / d and the raw X_U beta
      const int u = e / YG, m = e % YG;
      double v = 0.0;
      if (c_date[m] >= 0) {
        const int gd = c_date[m], j = c_j[m];
        const int bid = g_bid[gd * YMB + j];
        v = bid >= 0 ? pc[(int64_t)(s_urow[u] - r0) * ldpc + bid] : lr.panel[(int64_t)s_urow[u] * lr.ldp + (-1 - bid)];
        wscr[(int64_t)(d0 + gd) * wstride + (int64_t)(YMB + j) * k_ld + u] = v;
      }
      WU[u * YG + m] = sqc * dinv * v;
    }
    __syncthreads();
    gemm();
    correct([&](int m) { return c_date[m]; },
            [&](int m) { return c_date[m] >= 0 ? g_bmu[c_date[m] * YMB + c_j[m]] * dinv : 0.0; });
    for (int e = t; e < U * YG; e += YT) {
      const int u = e / YG, m = e % YG;
      if (c_date[m] >= 0) wscr[(int64_t)(d0 + c_date[m]) * wstride + (int64_t)c_j[m] * k_ld + u] = WU[u * YG + m];
    }
    if (t < YG && c_date[t] >= 0) g_sub[c_date[t] * YMB + c_j[t]] = g_su[t];
    __syncthreads();
  }
  // S = B K^-1 B' + delta I (lower), per date:  beta_j . K^-1 beta_k' =
  //   beta_j . beta_k / d - ((X_U beta_j) . Ut_k - su_k beta_j . mu) / d
  for (int e = hg; e < YG * YMB * YMB; e += YHW) {
    const int g = e / (YMB * YMB), j = (e / YMB) % YMB, k = e % YMB;
    if (!g_on[g] || j >= g_mb[g] || k > j) continue;
    const double* ws = wscr + (int64_t)(d0 + g) * wstride;
    double v = 0.0;
    for (int u = hl; u < U; u += 32) v = fma(ws[(int64_t)(YMB + j) * k_ld + u], ws[(int64_t)k * k_ld + u], v);
    v = ysum32(v);
    if (hl == 0) {
      const int bj = g_bid[g * YMB + j], bk = g_bid[g * YMB + k];
      double bb;
      if (bj >= 0 && bk >= 0) bb = cc[bj * mg + bk];
      else if (bj >= 0) bb = pb.Cg[(int64_t)bj * ld + (-1 - bk)];
      else if (bk >= 0) bb = pb.Cg[(int64_t)bk * ld + (-1 - bj)];
      else bb = bj == bk ? 1.0 : 0.0;
      const double delta = s.delta * g_sc[g];
      g_S[g * YMB * YMB + j * YMB + k] =
          bb * dinv - dinv * (v - g_sub[g * YMB + k] * g_bmu[g * YMB + j]) + (j == k ? delta : 0.0);
    }
  }
  __syncthreads();
  if (t < G && g_on[t]) {   // Cholesky of S (lower, in place), one thread per date
    double* S = g_S + t * YMB * YMB;
    const int mb = g_mb[t];
    int bad = 0;
    for (int cI = 0; cI < mb && !bad; ++cI) {
      double dd = S[cI * YMB + cI];
      for (int k = 0; k < cI; ++k) dd -= S[cI * YMB + k] * S[cI * YMB + k];
      if (!(dd > 0.0) || !isfinite(dd)) { bad = 1; break; }
      dd = sqrt(dd);
      S[cI * YMB + cI] = dd;
      for (int r = cI + 1; r < mb; ++r) {
        double v = S[r * YMB + cI];
        for (int k = 0; k < cI; ++k) v -= S[r * YMB + k] * S[cI * YMB + k];
        S[r * YMB + cI] = v / dd;
      }
    }
    if (bad) {   // left for the per-date kernel
      rec[(int64_t)(d0 + t) * PGR + R_STATE] = PQ_PG_FALLBACK;
      g_on[t] = g_run[t] = 0;
    }
  }
  __syncthreads();

  // ---- proximal iterative refinement ---------------------------------------------------------
  for (int it = 0; it <= nref; ++it) {
    // a) residual of the current point: X_U x (+ C x), window mask and centring, X_U' w
    pass1([&](int m) -> const double* { return (m < G && g_run[m]) ? st.work + (int64_t)(d0 + m) * st.work_stride : nullptr; },
          [&](int) { return 1.0; }, mg);
    for (int e = t; e < U * YG; e += YT) {
      const int u = e / YG, m = e % YG;
      const bool inw = m < G && g_run[m] && u >= g_off[m] && u < g_off[m] + g_T[m];
      WU[e] = inw ? WU[e] - g_mux[m] : 0.0;
    }
    __syncthreads();
    for (int m = hg; m < YG; m += YHW) {
      double v = 0.0;
      if (g_run[m])
        for (int u = hl; u < U; u += 32) v += WU[u * YG + m];
      v = ysum32(v);
      if (hl == 0) g_sw[m] = v;
    }
    __syncthreads();
    pass2([&](int m, int i, double v0, double v1, double* part) {
      const int b = d0 + m;
      double* W = st.work + (int64_t)b * st.work_stride;
      PGWork wk(st, b, ld);
      const double* q = pb.q + (int64_t)b * pb.q_stride;
      const double* mu = centred ? lr.mu + (int64_t)b * lr.mu_stride : nullptr;
      const double* lamd = g_lamd + m * YMG;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int ii = i + h;
        const double mui = mu ? mu[ii] : 0.0;
        const double xi = W[ii];
        const double pxi = c * ((h ? v1 : v0) - mui * g_sw[m]) + pd * xi;
        const double ri = -q[ii] - pxi - (mg ? crow(ii, lamd) : 0.0);
        wk.g[ii] = ri;
        if (wk.fl[ii] == 0) part[0] = fmax(part[0], fabs(ri));   // fixed rows: completed below
        part[1] = fma(mui, ri, part[1]);
      }
    });
    if (t < G && g_run[t]) {   // per date: max |r|, mu . r, the bordered residuals, convergence
      const int m = t, b = d0 + m;
      PGWork wk(st, b, ld);
      const double* mu = centred ? lr.mu + (int64_t)b * lr.mu_stride : nullptr;
      double rm = 0.0, mur = 0.0;
      for (int ww = 0; ww < YNW; ++ww) {
        rm = fmax(rm, g_part[(ww * YG + m) * YNP]);
        mur += g_part[(ww * YG + m) * YNP + 1];
      }
      for (int j = 0; j < g_mb[m]; ++j) {
        const int bid = g_bid[m * YMB + j];
        double bx;
        if (bid >= 0) {
          bx = g_cx[m * YMG + bid];
        } else {   // unit row: r_i gets -lam_j, rl_j = bound - x_i
          const int i = -1 - bid;
          const double lamj = g_lam[m * YMB + j];
          const double ri = wk.g[i] - lamj;
          wk.g[i] = ri;
          rm = fmax(rm, fabs(ri));
          if (mu) mur -= mu[i] * lamj;
          bx = wk.xs[i];
        }
        const double dBj = g_dB[m * YMB + j];
        const double v = dBj - bx;
        const double rl = fabs(v) <= 1e-14 * (1.0 + fabs(dBj) + fabs(bx)) ? 0.0 : v;
        g_rl[m * YMB + j] = rl;
        rm = fmax(rm, fabs(rl));
      }
      g_mur[m] = mur;
      if (rm <= 1e-13 * g_sc[m] || it == nref) g_run[m] = 0;   // converged (or out of steps)
    }
    __syncthreads();
    if (t == 0) {
      int any = 0;
      for (int g = 0; g < G; ++g) any |= g_run[g];
      s_any = any;
    }
    __syncthreads();
    if (!s_any) break;
    // b) t = K^-1 r, Schur step for dlam, dx = K^-1 (r - B' dlam)
    pass1([&](int m) -> const double* {
            return (m < G && g_run[m]) ? st.work + (int64_t)(d0 + m) * st.work_stride + 2 * (int64_t)ld : nullptr;
          },
          [&](int) { return sqc * dinv; }, mg);   // PGWork g = r; rows U.. give C r
    gemm();
    correct([&](int m) { return (m < G && g_run[m]) ? m : -1; }, [&](int m) { return g_mur[m] * dinv; });
    // Schur (one thread per date): B t - rl, dlam = S^-1 (B t - rl)
    for (int e = hg; e < YG * YMB; e += YHW) {   // (X_U beta_j) . Ut_r per (date, row)
      const int m = e / YMB, j = e % YMB;
      if (!g_run[m] || j >= g_mb[m]) continue;
      const double* xb = wscr + (int64_t)(d0 + m) * wstride + (int64_t)(YMB + j) * k_ld;
      double v = 0.0;
      for (int u = hl; u < U; u += 32) v = fma(xb[u], WU[u * YG + m], v);
      v = ysum32(v);
      if (hl == 0) g_dlam[e] = v;
    }
    __syncthreads();
    if (t < G && g_run[t]) {
      const int m = t, b = d0 + m;
      PGWork wk(st, b, ld);
      const int mb = g_mb[m];
      double wl[YMB];
#pragma unroll
      for (int j = 0; j < YMB; ++j) {
        if (j >= mb) { wl[j] = 0.0; continue; }
        const int bid = g_bid[m * YMB + j];
        const double br = bid >= 0 ? g_cx[m * YMG + bid] : wk.g[-1 - bid];
        const double tj = br * dinv - dinv * (g_dlam[m * YMB + j] - g_su[m] * g_bmu[m * YMB + j]);
        wl[j] = tj - g_rl[m * YMB + j];
      }
      const double* S = g_S + m * YMB * YMB;
      for (int i = 0; i < mb; ++i) {
        double v = wl[i];
        for (int j = 0; j < i; ++j) v -= S[i * YMB + j] * wl[j];
        wl[i] = v / S[i * YMB + i];
      }
      for (int i = mb - 1; i >= 0; --i) {
        double v = wl[i];
        for (int j = i + 1; j < mb; ++j) v -= S[j * YMB + i] * wl[j];
        wl[i] = v / S[i * YMB + i];
      }
      double suf = g_su[m];
      for (int j = 0; j < YMB; ++j) {
        if (j >= mb) break;
        g_dlam[m * YMB + j] = wl[j];
        suf -= wl[j] * g_sub[m * YMB + j];
        const int bid = g_bid[m * YMB + j];
        if (bid >= 0) g_dlamd[m * YMG + bid] = wl[j];
      }
      g_su[m] = suf;
    }
    __syncthreads();
    // Ut_f = Ut_r - sum_j dlam_j Ut_j
    for (int e = t; e < U * YG; e += YT) {
      const int u = e / YG, m = e % YG;
      if (!g_run[m]) continue;
      const double* ws = wscr + (int64_t)(d0 + m) * wstride;
      double v = WU[e];
      for (int j = 0; j < g_mb[m]; ++j) v -= g_dlam[m * YMB + j] * ws[(int64_t)j * k_ld + u];
      WU[e] = v;
    }
    __syncthreads();
    pass2([&](int m, int i, double v0, double v1, double* part) {
      const int b = d0 + m;
      PGWork wk(st, b, ld);
      const double* mu = centred ? lr.mu + (int64_t)b * lr.mu_stride : nullptr;
      const double* dl = g_dlamd + m * YMG;
      const double su = g_su[m];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int ii = i + h;
        const double mui = mu ? mu[ii] : 0.0;
        const double ri = wk.g[ii] - (mg ? crow(ii, dl) : 0.0);
        const double dx = (ri - ((h ? v1 : v0) - su * mui)) * dinv;
        const double xn = wk.xs[ii] + dx;
        wk.xs[ii] = xn;
        part[1] = fma(mui, xn, part[1]);
      }
    });
    if (t < G && g_run[t]) {   // unit rows: dx_i gets -dlam_j / d; lam += dlam; mu . x
      const int m = t, b = d0 + m;
      PGWork wk(st, b, ld);
      const double* mu = centred ? lr.mu + (int64_t)b * lr.mu_stride : nullptr;
      double mux = 0.0;
      for (int ww = 0; ww < YNW; ++ww) mux += g_part[(ww * YG + m) * YNP + 1];
      for (int j = 0; j < g_mb[m]; ++j) {
        const double dlj = g_dlam[m * YMB + j];
        const int bid = g_bid[m * YMB + j];
        if (bid < 0) {
          const int i = -1 - bid;
          wk.xs[i] -= dlj * dinv;
          if (mu) mux -= mu[i] * dlj * dinv;
        } else {
          g_lamd[m * YMG + bid] += dlj;
          g_dlamd[m * YMG + bid] = 0.0;
        }
        g_lam[m * YMB + j] += dlj;
      }
      g_mux[m] = mux;
    }
    __syncthreads();
  }

  // ---- write back: x (fixed variables exactly at their bound), multipliers ----------------------
  for (int e = t; e < YG * YMB; e += YT) {
    const int m = e / YMB, j = e % YMB;
    if (!g_on[m] || j >= g_mb[m]) continue;
    double* R = rec + (int64_t)(d0 + m) * PGR;
    const int bid = g_bid[e];
    if (bid < 0) {
      st.work[(int64_t)(d0 + m) * st.work_stride + (-1 - bid)] = g_dB[e];
      R[R_FXL + (j - g_ma[m])] = g_lam[e];
    } else {
      R[R_SOL + j] = g_lam[e];
    }
  }
  for (int e = t; e < YG * 64; e += YT) {
    const int m = e / 64, r = e % 64;
    if (g_on[m]) rec[(int64_t)(d0 + m) * PGR + R_LAM + r] = r < mg ? g_lamd[m * YMG + r] : 0.0;
  }
}

}  // namespace pq

// launched by pq_polish_grouped_round (polish_g.hip) after the LDS solves of the round
int pq_pg_wide_launch(const pq_lowrank* lr, const pq_problem* pb, pq_state* st, double* rec, const pq_settings* s,
                      const pq_pg_wide* wd, hipStream_t stream) {
  const pq_gcap* gc = wd->gc;
  PQ_CHECK_ARG(gc && gc->Minv && gc->aq && gc->hinv && gc->grho && gc->ngroups > 0,
               "pq_polish_grouped_round: wide mode needs the polish group capacitance");
  // (a group with ucnt[g] + mg > YU rows hands its pending dates to the per-date kernel in k_pgw)
  PQ_CHECK_ARG(gc->umax > 0 && gc->umax <= pq::YU && gc->k_ld % 64 == 0 && gc->k_ld <= 384 && gc->ldh > 0 &&
                   gc->ldh <= pq::YCH,
               "pq_polish_grouped_round: wide mode needs umax <= %d, k_ld <= 384, ldh <= %d", pq::YU, pq::YCH);
  PQ_CHECK_ARG(pb->mg <= pq::YMG && pb->Cg_stride == 0 && pb->g_stride == 0 && (pb->mg == 0 || (wd->pc && wd->cc)),
               "pq_polish_grouped_round: wide mode needs shared general rows (mg <= %d) with pc / cc", pq::YMG);
  PQ_CHECK_ARG(pb->mg <= 4 || (wd->nzr && wd->nzv && wd->nzmax > 0),
               "pq_polish_grouped_round: wide mode with mg > 4 needs the column-sparse rows");
  PQ_CHECK_ARG(wd->wscr && wd->wscr_stride >= PQ_PG_WSCR(gc->k_ld), "pq_polish_grouped_round: wide scratch too small");
  PQ_CHECK_ARG(pb->n % 2 == 0 && lr->ldp % 2 == 0 && pb->q_stride % 2 == 0, "pq_polish_grouped_round: even strides");
  const int nref = wd->refine_steps > 1 ? wd->refine_steps : 1;
  hipLaunchKernelGGL(pq::k_pgw, dim3(gc->ngroups), dim3(pq::YT), 0, stream, *lr, *pb, *st, *gc, rec, *s, wd->pc,
                     wd->ldpc, wd->r0, wd->cc, wd->nzr, wd->nzv, pb->mg > 4 ? wd->nzmax : 0, wd->wscr,
                     wd->wscr_stride, nref);
  PQ_CHECK_LAUNCH("pq_polish_grouped_round (wide)");
  return 0;
}
