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
__device__ int tile_potrf(double* T, int nvalid) {
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
// pitch DP).  Thread c < 64 owns column c.  Rows / columns >= nvalid are the identity.
__device__ void tile_trinv(const double* T, double* X, int nvalid) {
  const int c = threadIdx.x;
  if (c < TB) {
    for (int r = 0; r < c; ++r) X[c * DP + r] = 0.0;
    X[c * DP + c] = 1.0 / T[c * DP + c];
    for (int r = c + 1; r < TB; ++r) {
      double acc = 0.0;
      if (r < nvalid)
        for (int k = c; k < r; ++k) acc += T[r * DP + k] * X[c * DP + k];
      X[c * DP + r] = -acc / T[r * DP + r];
    }
  }
  __syncthreads();
}


// LDS needed by wg_cholesky: 4*STAGE (stream buffers / W image / diag tile) + TB*LDW.
constexpr int CHOL_LDS = 4 * STAGE + TB * LDW;

// Factor the nb*64 x nb*64 matrix whose lower-triangle elements are produced by
// `form(gi, gj)` (read exactly once each) into L stored in K (ld), with the transposed
// inverses of the diagonal blocks in Dt.  Returns info (0 = success, else first failing
// column + 1).  All threads of the (256-thread) workgroup must call it.
template <typename Form>
__device__ int wg_cholesky(const Form& f, double* K, int64_t ld, int nb, int nv, double* Dt, double* smem) {
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
    const int bad = tile_potrf(stg, nv - J * TB);
    if (bad) return J * TB + bad;
    double* X = sD;  // inverse computed with pitch DP inside the sD region
    tile_trinv(stg, X, nv - J * TB);
    double xr[TB * TB / 256];
#pragma unroll
    for (int q = 0; q < TB * TB / 256; ++q) {
      const int e = threadIdx.x + q * 256;
      const int i = e >> 6, j = e & 63;
      K[(int64_t)(J * TB + i) * ld + J * TB + j] = (j <= i) ? stg[i * DP + j] : 0.0;
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
