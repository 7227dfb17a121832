// K4, grouped pipeline: the per-date solve of a polish round (k_pg_solve's arithmetic) with
// P_FF + delta I factored in the REGISTERS of one wave, for free sets of at most 96.
//
// Why: k_pg_solve holds the packed triangle in LDS (26-37 KB at |F| = 80..96) and spreads a
// date over 2-4 waves that meet at two barriers per 16-column block, so a CU holds only 4-5
// dates and each date's time is a chain of LDS round trips and barriers.  Here one 64-lane
// wave owns a date: the lower 16 x 16 tiles of the matrix live in its VGPRs (15 tiles = 120
// VGPRs at |F| <= 80), the block columns are factored with the register pivot chain
// (wave_chol_inv16) and the panel / trailing updates are FP64 MFMAs whose operands come
// straight from the tile registers, no barriers between waves and ~10 KB of LDS per date.
//
// Tile layout ("stored" form S(X) of a 16 x 16 tile X): lane l, register q holds
// X[l & 15][(l >> 4) + 4 q] -- the MFMA C/D layout of X^T.  With the gfx950 f64 lane maps
// (common.h) register s of S(X) is at once the A operand (k-chunk s) of X and the B operand
// of X^T, so
//     mfma(S(X)[s], S(Y)[s]) over s = 0..3  ->  D = X Y^T in C layout = S(Y X^T),
// which is exactly the trailing update A_IJ' -= L_IJ L_J'J^T in stored form (S(A_IJ') -=
// S(L_IJ L_J'J^T) = C-layout(L_J'J L_IJ^T)), and the panel L_IJ^T = Linv_JJ A_IJ^T.
// Diagonal tiles keep the inverse of their Cholesky block (stored form), as in k_pg_solve.
//
// The single refinement step's residual needs P_FF x at the warm start, which is known
// before the factorisation: it is accumulated from the tile values while they are loaded
// (row sums of every lower tile, column sums of the off-diagonal ones), so the solve reads
// the K scratch once per factorisation.  Everything else -- the active rows' Schur block,
// the acceptance of the refinement, the inner primal step and the outputs -- is
// k_pg_solve's (polish_g.hip), so the pipeline's other kernels see the same record.
// Replaces, with the rest of the grouped polish, the accuracy of qpsolvers' answer
// (src/qp_problems.py:211-214).
#include <cstdlib>

#include "polish_dev.h"
#include "pg_record.h"

namespace pq {
namespace {

constexpr int RT_WMA = 8;   // active general rows of the solve (more: fallback), as k_pg_solve

__device__ constexpr int ti(int I, int J) { return I * (I + 1) / 2 + J; }

__device__ __forceinline__ double sum16r(double v) {   // over the 16 lanes of a row group
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double sum_g(double v) {    // over the 4 row groups (lanes l ^ 16, l ^ 32)
  v += __shfl_xor(v, 16, 64);
  v += __shfl_xor(v, 32, 64);
  return v;
}

// Tiles of P_FF + delta I (identity beyond k) from the K scratch (both triangles stored:
// element (r, c) is read as K[map c][map r], so a load instruction touches four 16-double
// row segments), and px = P_FF x (no delta) from the same values.  Every tile's load is issued
// before any is used (straight into the tile registers: one memory round trip, not one per
// block column).
template <int NB>
PQ_DEVFN void rt_load(f64x4 (&S)[NB * (NB + 1) / 2], const double* K, int ldk, const int* s_map, int k,
                      double delta, const double* xF, double* px) {
  const int l = (threadIdx.x + loop_zero()) & 63, c16 = l & 15, g = l >> 4;
  const int nbk = (k + 15) >> 4;
  // 1. raw values, clamped addresses, no use yet
#pragma unroll
  for (int I = 0; I < NB; ++I) {
    if (I < nbk) {
      const int r = 16 * I + c16;
      const int mr = s_map[r < k ? r : 0];
#pragma unroll
      for (int J = 0; J <= I; ++J)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int c = 16 * J + g + 4 * q;
          S[ti(I, J)][q] = K[s_map[c < k ? c : 0] * ldk + mr];   // (32-bit offsets: ldk <= 256)
        }
    }
  }
  // 2. px: row sums of every lower tile, column sums of the off-diagonal ones (masked beyond
  // k); then delta on the diagonal, identity beyond k
  double pr[NB];
#pragma unroll
  for (int I = 0; I < NB; ++I) pr[I] = 0.0;
#pragma unroll
  for (int J = 0; J < NB; ++J) {
    double pc[4] = {0.0, 0.0, 0.0, 0.0};
    if (J < nbk) {
#pragma unroll
      for (int I = J; I < NB; ++I) {
        if (I < nbk) {
          const int r = 16 * I + c16;
          const bool rv = r < k;
          const double xr = rv ? xF[r] : 0.0;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int c = 16 * J + g + 4 * q;
            const bool cv = c < k;
            const double v = (rv && cv) ? S[ti(I, J)][q] : 0.0;
            pr[I] = fma(v, cv ? xF[c] : 0.0, pr[I]);
            if (I > J) pc[q] = fma(v, xr, pc[q]);
            S[ti(I, J)][q] = (r == c) ? (rv ? v + delta : 1.0) : v;
          }
        } else {
#pragma unroll
          for (int q = 0; q < 4; ++q) S[ti(I, J)][q] = 0.0;
        }
      }
    } else {
#pragma unroll
      for (int I = J; I < NB; ++I)
#pragma unroll
        for (int q = 0; q < 4; ++q) S[ti(I, J)][q] = (I == J && c16 == g + 4 * q) ? 1.0 : 0.0;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) pc[q] = sum16r(pc[q]);   // (A_IJ' x_I)[16J + g + 4q], I > J
    if (c16 == 0) {
#pragma unroll
      for (int q = 0; q < 4; ++q) px[16 * J + g + 4 * q] = pc[q];
    }
  }
  __syncthreads();
#pragma unroll
  for (int I = 0; I < NB; ++I) {
    const double v = sum_g(pr[I]);
    if (g == 0) px[16 * I + c16] += v;
  }
  __syncthreads();
}

// In-register blocked Cholesky of the stored tiles: diagonal tiles end as the stored form of
// their block's L^-1, the others as L.  Returns 0, or the failing block column + 1 (uniform).
template <int NB>
PQ_DEVFN int rt_potrf(f64x4 (&S)[NB * (NB + 1) / 2], int k, double* tsc) {
  const int nbk = (k + 15) >> 4;
#pragma unroll
  for (int J = 0; J < NB; ++J) {
    if (J < nbk) {
      // lane ids from an opaque zero per block column: the chain's per-lane masks stay local
      const int l = (threadIdx.x + loop_zero()) & 63, c16 = l & 15, g = l >> 4;
      double A[4], Bv[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        A[q] = S[ti(J, J)][q];                 // symmetric: stored form = C layout
        Bv[q] = (g + 4 * q == c16) ? 1.0 : 0.0;
      }
      if (wave_chol_inv16(A, Bv, l)) return J + 1;
      // Bv = L_JJ^-1 in C layout (lane l: [g + 4q][c16]) -> stored form ([c16][g + 4q])
#pragma unroll
      for (int q = 0; q < 4; ++q) tsc[(g + 4 * q) * 17 + c16] = Bv[q];
      __syncthreads();
#pragma unroll
      for (int q = 0; q < 4; ++q) S[ti(J, J)][q] = tsc[c16 * 17 + g + 4 * q];
      __syncthreads();
      // panel: S(L_IJ) = C layout of L_JJ^-1 A_IJ^T
#pragma unroll
      for (int I = J + 1; I < NB; ++I) {
        if (I < nbk) {
          f64x4 acc = f64x4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
          for (int s4 = 0; s4 < 4; ++s4)
            acc = __builtin_amdgcn_mfma_f64_16x16x4f64(S[ti(J, J)][s4], S[ti(I, J)][s4], acc, 0, 0, 0);
          S[ti(I, J)] = acc;
        }
      }
      // trailing: A_IJ' -= L_IJ L_J'J^T  (S(A_IJ') += mfma(-S(L_J'J), S(L_IJ)))
#pragma unroll
      for (int Jp = J + 1; Jp < NB; ++Jp) {
#pragma unroll
        for (int I = Jp; I < NB; ++I) {
          if (I < nbk) {
            f64x4 acc = S[ti(I, Jp)];
#pragma unroll
            for (int s4 = 0; s4 < 4; ++s4)
              acc = __builtin_amdgcn_mfma_f64_16x16x4f64(-S[ti(Jp, J)][s4], S[ti(I, J)][s4], acc, 0, 0, 0);
            S[ti(I, Jp)] = acc;
          }
        }
      }
    }
  }
  return 0;
}

// y = L^-1 b (b, y: LDS vectors of length >= 16 nbk, zero-padded beyond k; y may not alias b)
template <int NB>
PQ_DEVFN void rt_fwd(const f64x4 (&S)[NB * (NB + 1) / 2], int k, const double* b, double* y) {
  const int l = (threadIdx.x + loop_zero()) & 63, c16 = l & 15, g = l >> 4;
  const int nbk = (k + 15) >> 4;
#pragma unroll
  for (int J = 0; J < NB; ++J) {
    if (J < nbk) {
      double part = 0.0;
#pragma unroll
      for (int K = 0; K < J; ++K)
#pragma unroll
        for (int q = 0; q < 4; ++q) part = fma(S[ti(J, K)][q], y[16 * K + g + 4 * q], part);
      part = sum_g(part);
      const double rj = b[16 * J + c16] - part;          // row c16 of the block, every row group
      double p2 = 0.0;
#pragma unroll
      for (int q = 0; q < 4; ++q) p2 = fma(S[ti(J, J)][q], __shfl(rj, g + 4 * q, 64), p2);
      p2 = sum_g(p2);
      if (g == 0) y[16 * J + c16] = p2;
      __syncthreads();
    }
  }
}

// x = L^-T y (LDS vectors as rt_fwd; x may not alias y)
template <int NB>
PQ_DEVFN void rt_bwd(const f64x4 (&S)[NB * (NB + 1) / 2], int k, const double* y, double* x, double* tv) {
  const int l = (threadIdx.x + loop_zero()) & 63, c16 = l & 15, g = l >> 4;
  const int nbk = (k + 15) >> 4;
#pragma unroll
  for (int J = NB - 1; J >= 0; --J) {
    if (J < nbk) {
      double a[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int I = J + 1; I < NB; ++I) {
        if (I < nbk) {
          const double xi = x[16 * I + c16];
#pragma unroll
          for (int q = 0; q < 4; ++q) a[q] = fma(S[ti(I, J)][q], xi, a[q]);
        }
      }
      if (J + 1 < nbk) {
#pragma unroll
        for (int q = 0; q < 4; ++q) a[q] = sum16r(a[q]);   // (sum_I L_IJ' x_I)[g + 4q]
      }
      if (c16 == 0) {
#pragma unroll
        for (int q = 0; q < 4; ++q) tv[g + 4 * q] = y[16 * J + g + 4 * q] - a[q];
      }
      __syncthreads();
      const double rr = tv[c16];
#pragma unroll
      for (int q = 0; q < 4; ++q) a[q] = sum16r(S[ti(J, J)][q] * rr);   // (L_JJ^-T r)[g + 4q]
      if (c16 == 0) {
#pragma unroll
        for (int q = 0; q < 4; ++q) x[16 * J + g + 4 * q] = a[q];
      }
      __syncthreads();
    }
  }
}

}  // namespace

// the LDS of one date's solve, sized for the largest register bucket (|F| <= 96)
constexpr int RT_KS = 96;
struct RtLds {
  double *xF, *rx, *t1, *t2, *px, *vv, *tsc, *Sm, *lamv, *wl, *rl, *dAv;
  int *s_map, *s_m2, *s_f2, *s_vp, *s_vi, *s_al, *s_flag;
};

template <int NB>
__device__ __forceinline__ void rt_solve_date(int b, const pq_problem& pb, const pq_state& st, double* rec,
                                              const pq_settings& s, int ldk, int klo, int inner, const RtLds& L_) {
  constexpr int KS = 16 * NB;
  constexpr int NT = NB * (NB + 1) / 2;
  static_assert(KS <= RT_KS, "rt_solve_date: bucket beyond the LDS sizing");
  double *xF = L_.xF, *rx = L_.rx, *t1 = L_.t1, *t2 = L_.t2, *px = L_.px, *vv = L_.vv, *tsc = L_.tsc;
  double *Sm = L_.Sm, *lamv = L_.lamv, *wl = L_.wl, *rl = L_.rl, *dAv = L_.dAv;
  int *s_map = L_.s_map, *s_m2 = L_.s_m2, *s_f2 = L_.s_f2, *s_vp = L_.s_vp, *s_vi = L_.s_vi, *s_al = L_.s_al;
  int& s_flag = *L_.s_flag;
  double* R = rec + (int64_t)b * PGR;
  if (R[R_STATE] != PQ_PG_PENDING || R[R_W] != 0.0) return;
  const int kb = (int)R[R_KB];   // the bucket key (R_K may already be lowered by this kernel)
  if (kb <= klo || kb > KS) return;
  int k = kb;
  const int ma = (int)R[R_MA];
  const int t = threadIdx.x;
  if (ma > RT_WMA) {
    if (t == 0) R[R_STATE] = PQ_PG_FALLBACK;
    return;
  }
  const int n = pb.n, ld = pb.ld;
  const double* Cg = pb.Cg ? pb.Cg + (int64_t)b * pb.Cg_stride : nullptr;
  PGWork wk(st, b, ld);
  const double sc = R[R_SC];
  const double delta = s.delta * sc;
  const double* K = st.K + (int64_t)b * st.K_stride;   // P_FF (both triangles)
  const bool reuse = R[R_REUSE] != 0.0;
  for (int p = t; p < KS; p += 64) {
    s_map[p] = p < k ? (reuse ? wk.posF[wk.Fl[p]] : p) : 0;
    xF[p] = p < k ? wk.solx[p] : 0.0;
  }
  if (t < ma) {
    s_al[t] = (int)R[R_AL + t];
    lamv[t] = R[R_SOL + t];
    dAv[t] = R[R_DA + t];
  }
  const bool has_box = pb.lb != nullptr;
  const double* lb = has_box ? pb.lb + (int64_t)b * pb.box_stride : nullptr;
  const double* ub = has_box ? pb.ub + (int64_t)b * pb.box_stride : nullptr;
  __syncthreads();
#ifdef PQ_PROFILE
  long long t_last_ = wall_clock64();
#define RSTAMP(k_)                                                         \
  do {                                                                     \
    __syncthreads();                                                       \
    if (t == 0) { const long long n_ = wall_clock64(); R[8 + (k_)] += (double)(n_ - t_last_); t_last_ = n_; } \
  } while (0)
#else
#define RSTAMP(k_) do { } while (0)
#endif
  f64x4 S[NT];
  for (int it_in = 0;; ++it_in) {
    const int l = threadIdx.x + loop_zero();
    rt_load<NB>(S, K, ldk, s_map, k, delta, xF, px);
    RSTAMP(0);
    if (rt_potrf<NB>(S, k, tsc)) {
      if (l == 0) R[R_STATE] = PQ_PG_FALLBACK;
      return;
    }
    RSTAMP(1);
    // U = L^-1 C_aF' (rows a of the U scratch), S = U'U + delta I
    for (int a = 0; a < ma; ++a) {
      const double* cr = Cg + (int64_t)s_al[a] * ld;
      for (int p = l; p < KS; p += 64) t1[p] = p < k ? cr[wk.Fl[p]] : 0.0;
      __syncthreads();
      rt_fwd<NB>(S, k, t1, t2);
      for (int p = l; p < k; p += 64) wk.U[(int64_t)a * ld + p] = t2[p];
      __syncthreads();
    }
    for (int e = 0; e < ma * ma; ++e) {
      const int ii = e / ma, jj = e % ma;
      if (jj > ii) continue;
      const double* ui = wk.U + (int64_t)ii * ld;
      const double* uj = wk.U + (int64_t)jj * ld;
      double sum = 0.0;
      for (int p = l; p < k; p += 64) sum += ui[p] * uj[p];
      sum = wave_sum(sum);
      if (l == 0) Sm[ii * RT_WMA + jj] = sum + (ii == jj ? delta : 0.0);
    }
    __syncthreads();
    if (l == 0) {   // tiny Cholesky of S (ma <= 8), one lane
      int sbad = 0;
      for (int c = 0; c < ma && !sbad; ++c) {
        double d = Sm[c * RT_WMA + c];
        for (int m = 0; m < c; ++m) d -= Sm[c * RT_WMA + m] * Sm[c * RT_WMA + m];
        if (!(d > 0.0) || !isfinite(d)) { sbad = 1; break; }
        d = sqrt(d);
        Sm[c * RT_WMA + c] = d;
        for (int r = c + 1; r < ma; ++r) {
          double v = Sm[r * RT_WMA + c];
          for (int m = 0; m < c; ++m) v -= Sm[r * RT_WMA + m] * Sm[c * RT_WMA + m];
          Sm[r * RT_WMA + c] = v / d;
        }
      }
      s_flag = sbad;
    }
    __syncthreads();
    if (s_flag) {
      if (l == 0) R[R_STATE] = PQ_PG_FALLBACK;
      return;
    }
    RSTAMP(2);
    // ---- proximal iterative refinement (k_pg_solve's) -------------------------------------
    for (int itr = 0; itr < s.refine_iters; ++itr) {
      if (itr > 0) {   // later steps: P_FF x from the K scratch (the first has it from the load)
        for (int p = l; p < k; p += 64) {
          double sum = 0.0;
#pragma unroll 8
          for (int qq = 0; qq < k; ++qq) sum = fma(K[(int64_t)s_map[qq] * ldk + s_map[p]], xF[qq], sum);
          px[p] = sum;
        }
      }
      for (int a = 0; a < ma; ++a) {
        const double* cr = Cg + (int64_t)s_al[a] * ld;
        double sum = 0.0;
        for (int p = l; p < k; p += 64) sum += cr[wk.Fl[p]] * xF[p];
        sum = wave_sum(sum);
        if (l == 0) {
          const double v = dAv[a] - sum;
          rl[a] = fabs(v) <= 1e-14 * (1.0 + fabs(dAv[a]) + fabs(sum)) ? 0.0 : v;
        }
      }
      __syncthreads();
      double rm = 0.0;
      for (int p = l; p < KS; p += 64) {
        double v = 0.0;
        if (p < k) {
          v = wk.rF[p] - px[p];
          const int fp = wk.Fl[p];
          for (int a = 0; a < ma; ++a) v -= Cg[(int64_t)s_al[a] * ld + fp] * lamv[a];
        }
        rx[p] = v;
        rm = fmax(rm, fabs(v));
      }
      if (l < ma) rm = fmax(rm, fabs(rl[l]));
      __syncthreads();
      RSTAMP(3);
      if (wave_max(rm) <= 1e-13 * sc) break;   // uniform
      rt_fwd<NB>(S, k, rx, t2);   // t2 = L^-1 rx
      for (int a = 0; a < ma; ++a) {   // wl = U' t2 - rl
        const double* ua = wk.U + (int64_t)a * ld;
        double sum = 0.0;
        for (int p = l; p < k; p += 64) sum += ua[p] * t2[p];
        sum = wave_sum(sum);
        if (l == 0) wl[a] = sum - rl[a];
      }
      __syncthreads();
      if (l == 0) {   // dlam = S^-1 wl
        for (int ii = 0; ii < ma; ++ii) {
          double v = wl[ii];
          for (int jj = 0; jj < ii; ++jj) v -= Sm[ii * RT_WMA + jj] * wl[jj];
          wl[ii] = v / Sm[ii * RT_WMA + ii];
        }
        for (int ii = ma - 1; ii >= 0; --ii) {
          double v = wl[ii];
          for (int jj = ii + 1; jj < ma; ++jj) v -= Sm[jj * RT_WMA + ii] * wl[jj];
          wl[ii] = v / Sm[ii * RT_WMA + ii];
        }
      }
      __syncthreads();
      for (int p = l; p < KS; p += 64) {
        double v = p < k ? t2[p] : 0.0;
        for (int a = 0; a < ma; ++a) v -= (p < k ? wk.U[(int64_t)a * ld + p] : 0.0) * wl[a];
        t1[p] = v;
      }
      __syncthreads();
      rt_bwd<NB>(S, k, t1, t2, rx);   // t2 = L^-T (t2 - U dlam)   (rx: scratch)
      for (int p = l; p < k; p += 64) xF[p] += t2[p];
      if (l < ma) lamv[l] += wl[l];
      __syncthreads();
      RSTAMP(4);
    }
    // ---- inner primal step (k_pg_solve's): free variables outside their box fixed at the
    // bound they cross, the others compacted in order, the reduced rhs updated -----------------
    if (it_in >= inner || !has_box) break;   // uniform
    {
      int nk = 0, nv = 0;
      for (int p0 = 0; p0 < k; p0 += 64) {
        const int p = p0 + l;
        int f = 0, i = 0;
        double v = 0.0;
        if (p < k) {
          i = wk.Fl[p];
          const double xi = xF[p];
          if (!isinf(lb[i]) && xi < lb[i] - 1e-12 * (1.0 + fabs(lb[i]))) { f = 1; v = lb[i]; }
          else if (!isinf(ub[i]) && xi > ub[i] + 1e-12 * (1.0 + fabs(ub[i]))) { f = 2; v = ub[i]; }
        }
        const unsigned long long mv = __ballot(p < k && f != 0);
        const unsigned long long mk = __ballot(p < k && f == 0);
        const unsigned long long below = (1ull << l) - 1ull;
        if (p < k && f != 0) {
          const int j = nv + __popcll(mv & below);
          s_vp[j] = s_map[p];
          s_vi[j] = 4 * i + f;
          vv[j] = v;
        } else if (p < k) {
          const int j = nk + __popcll(mk & below);
          s_m2[j] = s_map[p];
          s_f2[j] = i;
          t1[j] = xF[p];
          t2[j] = wk.rF[p];
        }
        nv += __popcll(mv);
        nk += __popcll(mk);
      }
      __syncthreads();
#ifdef PQ_PROFILE
      if (t == 0) {   // inner-step counters: solves, steps taken, violators, (unused), k at the check
        R[20] += 1.0;
        R[21] += (nv > 0 && nv < k) ? 1.0 : 0.0;
        R[22] += (nv < k) ? (double)nv : 0.0;
        R[24] += (double)k;
      }
#endif
      if (nv == 0 || nv == k) break;   // uniform: feasible, or nothing left free (the rounds decide)
      const int k2 = k - nv;
      for (int p = l; p < KS; p += 64) {
        if (p < k2) {
          const int mp = s_m2[p];
          double r = t2[p];
          for (int j = 0; j < nv; ++j)
            if (vv[j] != 0.0) r = fma(-K[(int64_t)mp * ldk + s_vp[j]], vv[j], r);
          wk.rF[p] = r;
          wk.Fl[p] = s_f2[p];
          s_map[p] = mp;
          xF[p] = t1[p];
        } else {
          s_map[p] = 0;
          xF[p] = 0.0;
        }
      }
      for (int j = l; j < nv; j += 64) {
        const int i = s_vi[j] >> 2;
        wk.fl[i] = s_vi[j] & 3;
        wk.xb[i] = vv[j];
      }
      for (int a = 0; a < ma; ++a) {
        const double* cr = Cg + (int64_t)s_al[a] * ld;
        double sum = 0.0;
        for (int j = l; j < nv; j += 64) sum += cr[s_vi[j] >> 2] * vv[j];
        sum = wave_sum(sum);
        if (l == 0) dAv[a] -= sum;
      }
      if (l == 0) R[R_K] = k2;
      k = k2;
      __syncthreads();
    }
  }
  // ---- expand: xs = x_B off F, x_F on F; general multipliers by row ------------------------
  for (int ii = t; ii < n; ii += 64) wk.xs[ii] = wk.xb[ii];
  __syncthreads();
  for (int p = t; p < k; p += 64) {
    wk.xs[wk.Fl[p]] = xF[p];
    wk.solx[p] = xF[p];
  }
  R[R_LAM + t] = 0.0;   // the 64 row slots
  __syncthreads();
  if (t < ma) {
    R[R_LAM + s_al[t]] = lamv[t];
    R[R_SOL + t] = lamv[t];
  }
  RSTAMP(5);
#undef RSTAMP
}

// One launch for the four register buckets (one wave per date): workgroups [0, B) take the
// dates of the |F| <= 96 bucket's list, [B, 2B) those of <= 80, then <= 64 and <= 48 -- the
// largest free sets (the longest solves) are dispatched first, and no bucket waits for
// another's launch on a shared hardware queue (with separate launches on side streams, one
// of them started only after another bucket's kernel had ended).  Registers: the <= 96 path
// sets the budget (2 waves per SIMD, as the <= 80 path alone needs).
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2, 2)))
void k_pg_solve_rt(pq_problem pb, pq_state st, double* rec, pq_settings s, int ldk, int inner, int nbmax) {
  __shared__ double xF[RT_KS], rx[RT_KS], t1[RT_KS], t2[RT_KS], px[RT_KS], vv[RT_KS];
  __shared__ double tsc[16 * 17];
  __shared__ double Sm[RT_WMA * RT_WMA], lamv[RT_WMA], wl[RT_WMA], rl[RT_WMA], dAv[RT_WMA];
  __shared__ int s_map[RT_KS], s_m2[RT_KS], s_f2[RT_KS], s_vp[RT_KS], s_vi[RT_KS];
  __shared__ int s_al[RT_WMA];
  __shared__ int s_flag;
  const RtLds L_{xF, rx, t1, t2, px, vv, tsc, Sm, lamv, wl, rl, dAv, s_map, s_m2, s_f2, s_vp, s_vi, s_al, &s_flag};
  const int B = pb.batch;
  const int sel = blockIdx.x / B, i = blockIdx.x - sel * B;
  const int nb = nbmax - sel;   // 6, 5, 4, 3
  const int bk = pg_bucket(16 * nb);
  if ((unsigned long long)i >= reinterpret_cast<const unsigned long long*>(rec + R_CNT)[bk]) return;
  const int b = (int)rec[(int64_t)i * PGR + R_LIST + bk];
  switch (nb) {
    case 6: rt_solve_date<6>(b, pb, st, rec, s, ldk, 80, inner, L_); break;
    case 5: rt_solve_date<5>(b, pb, st, rec, s, ldk, 64, inner, L_); break;
    case 4: rt_solve_date<4>(b, pb, st, rec, s, ldk, 48, inner, L_); break;
    default: rt_solve_date<3>(b, pb, st, rec, s, ldk, 0, inner, L_); break;
  }
}

}  // namespace pq

// the register buckets |F| <= 16 nbmax (nbmax in 3..6: 48 .. 96), one launch
int pq_pg_solve_rt_launch(int nbmax, int B, hipStream_t str, const pq_problem* pb, pq_state* st, double* rec,
                          const pq_settings* s, int ldk) {
  if (nbmax < 3 || nbmax > 6) return -1;
  const int inner = s->polish_inner > 0 ? s->polish_inner : 0;
  hipLaunchKernelGGL(pq::k_pg_solve_rt, dim3((nbmax - 2) * B), dim3(64), 0, str, *pb, *st, rec, *s, ldk, inner,
                     nbmax);
  return 0;
}
