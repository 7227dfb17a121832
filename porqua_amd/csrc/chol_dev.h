// Workgroup-level blocked Cholesky on FP64 MFMA (header-only, shared by K2 and K4).
// See chol.hip for the algorithm description.
#pragma once
#include "common.h"

namespace pq {

constexpr int DP = 65;  // pitch of the row-major diagonal work tile

// Unblocked Cholesky of the 64x64 row-major tile T (pitch DP, lower used).  Returns the
// 1-based local column of the first non-positive pivot, 0 on success (uniform).  Rows and
// columns >= nvalid must already hold the identity (the zero-padded tail of a matrix whose
// padding is the identity): their pivot steps are skipped.
//
// One wave does the whole tile with lane i holding row i in registers (fully unrolled, so
// every register index is static); the pivot column of each step is exchanged through the
// tile's padding column T[j][64] (LDS broadcast reads: a wave's LDS operations complete in
// order, so no barrier is needed inside the wave).  All threads must call.
__device__ int tile_potrf(double* T, int nvalid) {
  const int kend = nvalid < TB ? (nvalid > 0 ? nvalid : 0) : TB;
  __syncthreads();   // the tile was written by every wave
  if (wave_id() == 0) {
    const int i = lane_id();
    double r[TB];
#pragma unroll
    for (int j = 0; j < TB; ++j) r[j] = T[i * DP + j];
    int bad = 0;
#pragma unroll
    for (int k = 0; k < TB; ++k) {
      if (k < kend && !bad) {
        T[i * DP + TB] = r[k];
        const double d = T[k * DP + TB];
        if (!(d > 0.0) || !isfinite(d)) {
          bad = k + 1;
        } else {
          const double s = sqrt(d);
          const double lik = (i > k) ? r[k] / s : (i == k ? s : 0.0);
          r[k] = lik;
          T[i * DP + TB] = lik;
#pragma unroll
          for (int j = k + 1; j < TB; ++j) r[j] = fma(-lik, T[j * DP + TB], r[j]);
        }
      }
    }
#pragma unroll
    for (int j = 0; j < TB; ++j)
      if (j <= i) T[i * DP + j] = r[j];
    if (i == 0) T[TB] = (double)bad;   // padding slot of row 0 carries the result
  }
  __syncthreads();
  const int bad = (int)T[TB];
  __syncthreads();
  return bad;
}

// The same factorisation with the whole workgroup and LDS only (few registers): for the
// small Schur-complement tile of the polish, whose valid size is the number of active rows.
PQ_DEVFN int tile_potrf_lds(double* T, int nvalid) {
  const int t = threadIdx.x;
  const int kend = nvalid < TB ? (nvalid > 0 ? nvalid : 0) : TB;
  for (int k = 0; k < kend; ++k) {
    __syncthreads();
    const double d = T[k * DP + k];
    if (!(d > 0.0) || !isfinite(d)) return k + 1;
    const double s = sqrt(d);
    __syncthreads();
    if (t < TB) {
      if (t == k) T[k * DP + k] = s;
      else if (t > k) T[t * DP + k] /= s;
    }
    __syncthreads();
    const int rem = kend - 1 - k;
    for (int e = t; e < rem * rem; e += blockDim.x) {
      const int i = k + 1 + e / rem, j = k + 1 + e % rem;
      if (j <= i) T[i * DP + j] -= T[i * DP + k] * T[j * DP + k];
    }
  }
  __syncthreads();
  return 0;
}

// Inverse of the lower-triangular tile T (pitch DP) into X (row c = column c of T^-1,
// pitch DP).  One wave: lane c builds column c in registers by forward substitution over
// the broadcast rows of T.  Rows / columns >= nvalid are the identity.  All threads call.
__device__ void tile_trinv(const double* T, double* X, int nvalid) {
  __syncthreads();
  if (wave_id() == 0) {
    const int c = lane_id();
    double x[TB];
#pragma unroll
    for (int r = 0; r < TB; ++r) {
      // four partial sums: a 4x shorter dependent FMA chain per row
      double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
      if (r < nvalid) {
#pragma unroll
        for (int k = 0; k + 3 < r; k += 4) {
          a0 = fma(T[r * DP + k], x[k], a0);
          a1 = fma(T[r * DP + k + 1], x[k + 1], a1);
          a2 = fma(T[r * DP + k + 2], x[k + 2], a2);
          a3 = fma(T[r * DP + k + 3], x[k + 3], a3);
        }
#pragma unroll
        for (int k = r & ~3; k < r; ++k) a0 = fma(T[r * DP + k], x[k], a0);
      }
      const double acc = (a0 + a1) + (a2 + a3);
      const double dg = T[r * DP + r];
      x[r] = (r < c) ? 0.0 : (r == c ? 1.0 / dg : -acc / dg);
    }
#pragma unroll
    for (int r = 0; r < TB; ++r) X[c * DP + r] = x[r];
  }
  __syncthreads();
}


// Cholesky AND inverse of the 64x64 tile T (pitch DP, lower used, rows / columns >= nvalid
// the identity) by the whole 256-thread workgroup in 16-column blocks: wave 0 factors and
// inverts each 16x16 diagonal block in registers (wave_chol_inv16: cross-lane shuffles, no
// LDS round trip per pivot), the panel L_ip = A_ip L_pp^-T and the trailing update
// A_ij -= L_ip L_jp' are 16x16x4 MFMA tiles spread over the four waves, and the off-diagonal
// blocks of L^-1 follow by blocked forward substitution (one wave per block column).  On
// exit T's lower triangle holds L and X (pitch DP) holds X[c][r] = (L^-1)[r][c] (the layout
// of tile_trinv).  Returns 0, or 1 + the first column of the 16-block whose pivot failed
// (uniform).  Replaces tile_potrf + tile_trinv, whose 64-step single-wave pivot chains
// through LDS dominated the blocked factorisations (k_factor, pq_polish_w_batched).
PQ_DEVFN int tile_chol_inv64(double* T, double* X, int nvalid) {
  const int t = threadIdx.x, w = wave_id(), l = lane_id();
  const int cc = l & 15, gg = l >> 4;
  const int nv = nvalid < 0 ? 0 : (nvalid > TB ? TB : nvalid);
  for (int e = t; e < TB * DP; e += blockDim.x) X[e] = 0.0;
  __syncthreads();   // T written by every wave; X cleared
  for (int p = 0; p < 4; ++p) {
    const int p0 = 16 * p;
    if (w == 0) {   // diagonal block: L_pp (lower, into T) and L_pp^-1 (into X, transposed)
      double A[4], Bv[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int r = gg + 4 * q;
        const bool in = p0 + r < nv && p0 + cc < nv;
        A[q] = in ? (cc <= r ? T[(p0 + r) * DP + p0 + cc] : T[(p0 + cc) * DP + p0 + r]) : (r == cc ? 1.0 : 0.0);
        Bv[q] = (r == cc) ? 1.0 : 0.0;
      }
      const int bad = wave_chol_inv16(A, Bv);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int r = gg + 4 * q;
        if (cc <= r) {
          T[(p0 + r) * DP + p0 + cc] = A[q];
          X[(p0 + cc) * DP + p0 + r] = Bv[q];
        }
      }
      if (l == 0) T[TB] = bad ? (double)(p0 + 1) : 0.0;   // row 0's padding slot carries the result
    }
    __syncthreads();
    if (T[TB] != 0.0) {
      const int bad = (int)T[TB];
      __syncthreads();
      return bad;
    }
    // panel: L_ip = A_ip L_pp^-T, i = p + 1 + w (MFMA: A[m][k] = A_ip[m][k], B[k][n] = Linv_pp[n][k])
    const int i_p = p + 1 + w;
    if (i_p < 4) {
      const int i0 = 16 * i_p;
      f64x4 acc = f64x4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) {
        const int k = 4 * s4 + gg;
        const double av = T[(i0 + cc) * DP + p0 + k];
        const double bv = X[(p0 + k) * DP + p0 + cc];   // Linv_pp[cc][k] (0 for k > cc)
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc, 0, 0, 0);
      }
      __builtin_amdgcn_wave_barrier();   // every lane's reads of A_ip precede the writes
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) T[(i0 + gg + 4 * rr) * DP + p0 + cc] = acc[rr];
    }
    __syncthreads();
    // trailing update A_ij -= L_ip L_jp' for p < j <= i (lower 16x16 tiles, round-robin over waves)
    const int m = 3 - p, ntr = m * (m + 1) / 2;
    for (int tt = w; w < 4 && tt < ntr; tt += 4) {   // (waves 4.. of k_factor_sk: no tiles)
      int ii = 0;
      while ((ii + 1) * (ii + 2) / 2 <= tt) ++ii;
      const int jj = tt - ii * (ii + 1) / 2;
      const int i0 = 16 * (p + 1 + ii), j0 = 16 * (p + 1 + jj);
      f64x4 acc = f64x4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) {
        const int k = 4 * s4 + gg;
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(T[(i0 + cc) * DP + p0 + k], T[(j0 + cc) * DP + p0 + k], acc, 0, 0, 0);
      }
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) T[(i0 + gg + 4 * rr) * DP + j0 + cc] -= acc[rr];
    }
    __syncthreads();
  }
  // L^-1 below the diagonal blocks, block column p = w:  Linv_ip = -Linv_ii sum_{k=p}^{i-1} L_ik Linv_kp
  if (w < 3) {
    const int p = w, p0 = 16 * p;
    for (int i = p + 1; i < 4; ++i) {
      const int i0 = 16 * i;
      f64x4 S = f64x4{0.0, 0.0, 0.0, 0.0};
      for (int k = p; k < i; ++k) {
        const int k0 = 16 * k;
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) {
          const int tk = 4 * s4 + gg;
          S = __builtin_amdgcn_mfma_f64_16x16x4f64(T[(i0 + cc) * DP + k0 + tk], X[(p0 + cc) * DP + k0 + tk], S, 0, 0, 0);
        }
      }
      // S in the C layout is the B operand of the next product: lane l holds S[gg + 4 s4][cc]
      f64x4 o = f64x4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) {
        const int tk = 4 * s4 + gg;
        o = __builtin_amdgcn_mfma_f64_16x16x4f64(X[(i0 + tk) * DP + i0 + cc], S[s4], o, 0, 0, 0);
      }
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) X[(p0 + cc) * DP + i0 + gg + 4 * rr] = -o[rr];
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
  }
  __syncthreads();
  return 0;
}

// KKT matrix K = ps P + pd I + sigma I + Cg' R Cg + R_box, element by element (K2 / K2L)
struct FormCtx {
  const double* P;
  int64_t ld;
  int n, mg;
  double ps, pd, sigma;
  const double* Cg;
  const double* lg;   // general-row bounds (rho of each row derived on the fly)
  const double* ug;
  const double* lb;
  const double* ub;
  double rho, rho_min, eq_scale;
};

__device__ __forceinline__ double rho_for(double l, double u, double rho, double rho_min,
                                          double eq_scale) {
  if (l == u) return rho * eq_scale;
  if (isinf(l) && isinf(u)) return rho_min;
  return rho;
}

__device__ __forceinline__ double form_elem(const FormCtx& f, int gi, int gj) {
  if (gi >= f.n || gj >= f.n) return gi == gj ? 1.0 : 0.0;
  double v = f.ps * f.P[(int64_t)gi * f.ld + gj];
  for (int r = 0; r < f.mg; ++r)
    v += rho_for(f.lg[r], f.ug[r], f.rho, f.rho_min, f.eq_scale) * f.Cg[(int64_t)r * f.ld + gi] *
         f.Cg[(int64_t)r * f.ld + gj];
  if (gi == gj) {
    v += f.pd + f.sigma;
    if (f.lb != nullptr) v += rho_for(f.lb[gi], f.ub[gi], f.rho, f.rho_min, f.eq_scale);
  }
  return v;
}

struct FormOp {
  const FormCtx* f;
  __device__ __forceinline__ double operator()(int gi, int gj) const { return form_elem(*f, gi, gj); }
};

// LDS needed by wg_cholesky: 4*STAGE (stream buffers / W image / diag tile) + TB*LDW.
constexpr int CHOL_LDS = 4 * STAGE + TB * LDW;

// Factor the nb*64 x nb*64 matrix whose lower-triangle elements are produced by
// `form(gi, gj)` (read exactly once each) into L stored in K (ld), with the transposed
// inverses of the diagonal blocks in Dt.  Returns info (0 = success, else first failing
// column + 1).  All threads of the (256-thread) workgroup must call it.
// kStoreDiag = false leaves K's diagonal 64x64 blocks untouched (nothing downstream of the
// polish reads them: the solves use Dt), so they can keep the matrix being factored.
template <bool kStoreDiag = true, typename Form>
PQ_DEVFN int wg_cholesky(const Form& f, double* K, int64_t ld, int nb, int nv, double* Dt, double* smem) {
  double* stg = smem;
  double* sD = smem + 4 * STAGE;
  for (int J = 0; J < nb; ++J) {
    Acc acc;
    acc.zero();
    gemm_stream<MODE_IK, MODE_IK>(acc, stg, K, ld, J * TB, 0, K, ld, J * TB, 0, J * TB);
    __syncthreads();
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int nn = 0; nn < 2; ++nn)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int i = acc_row(m, r), j = acc_col(nn);
          stg[i * DP + j] = f(J * TB + i, J * TB + j) - acc.c[m][nn][r];
        }
    double* X = sD;  // inverse computed with pitch DP inside the sD region
    const int bad = tile_chol_inv64(stg, X, nv - J * TB);
    if (bad) return J * TB + bad;
    double xr[TB * TB / 256];
#pragma unroll
    for (int q = 0; q < TB * TB / 256; ++q) {
      const int e = threadIdx.x + q * 256;
      const int i = e >> 6, j = e & 63;
      if (kStoreDiag) K[(int64_t)(J * TB + i) * ld + J * TB + j] = (j <= i) ? stg[i * DP + j] : 0.0;
      xr[q] = X[i * DP + j];                             // (T^-1)[j][i]
      Dt[(int64_t)J * TB * TB + i * TB + j] = xr[q];     // Dt[c][r] = Dinv[r][c]
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < TB * TB / 256; ++q) {
      const int e = threadIdx.x + q * 256;
      sD[(e >> 6) * LDW + (e & 63)] = xr[q];             // image SB[k][j] = Dinv[j][k]
    }
    __syncthreads();
    for (int I = J + 1; I < nb; ++I) {
      acc.zero();
      gemm_stream<MODE_IK, MODE_IK>(acc, stg, K, ld, I * TB, 0, K, ld, J * TB, 0, J * TB);
      __syncthreads();
#pragma unroll
      for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int nn = 0; nn < 2; ++nn)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int i = acc_row(m, r), k = acc_col(nn);
            stg[k * LDW + i] = f(I * TB + i, J * TB + k) - acc.c[m][nn][r];
          }
      __syncthreads();
      Acc o;
      o.zero();
      mma_lds(o, stg, sD, TB);
      acc_store(o, K, ld, I * TB, J * TB);
    }
  }
  __syncthreads();
  return 0;
}

}  // namespace pq
