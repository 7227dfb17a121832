// Batched matrix-vector products with the window matrices of the interior-point methods
// (porqua_amd/ipm_l1.py: U = [sqrt(w) Xc; A; G] per date, (T + mc) x n):
//   trans = 0:  y[b] = U[b] x[b]     (m outputs, one wave per row, lanes over the n columns)
//   trans = 1:  y[b] = U[b]' x[b]    (n outputs, one thread per column pair, rows streamed)
// One product reads U once (8 m n bytes per date) and is HBM-bound; rocBLAS's batched GEMM
// with one right-hand side (64 x 128 macro tiles for an N of 1) ran these at ~1 TB/s and was
// 58 % of the turnover + leverage IPM's time.  16-byte loads when rows are 16-byte aligned.
#include "capi_util.h"

namespace {

constexpr int kWG = 256;
constexpr int kRowsN = 16;    // trans = 0: rows per workgroup (4 per wave)
constexpr int kColsT = 512;   // trans = 1: columns per workgroup (2 per thread)

template <bool VEC>
__global__ __launch_bounds__(kWG) void k_gemv_n(const double* __restrict__ U, int64_t ldu, int64_t su, int m,
                                                int n, const double* __restrict__ x, int64_t sx,
                                                double* __restrict__ y, int64_t sy) {
  const int b = blockIdx.y;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const double* Ub = U + (int64_t)b * su;
  const double* xb = x + (int64_t)b * sx;
  for (int rr = 0; rr < kRowsN / 4; ++rr) {
    const int r = blockIdx.x * kRowsN + wave * (kRowsN / 4) + rr;
    if (r >= m) break;   // uniform per wave
    const double* row = Ub + (int64_t)r * ldu;
    double acc = 0.0;
    if (VEC) {
      for (int c = 2 * lane; c < n; c += 128) {
        const double2 u = *reinterpret_cast<const double2*>(row + c);
        const double2 v = *reinterpret_cast<const double2*>(xb + c);
        acc = fma(u.y, v.y, fma(u.x, v.x, acc));
      }
    } else {
      for (int c = lane; c < n; c += 64) acc = fma(row[c], xb[c], acc);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
    if (lane == 0) y[(int64_t)b * sy + r] = acc;
  }
}

template <bool VEC>
__global__ __launch_bounds__(kWG) void k_gemv_t(const double* __restrict__ U, int64_t ldu, int64_t su, int m,
                                                int n, const double* __restrict__ x, int64_t sx,
                                                double* __restrict__ y, int64_t sy) {
  extern __shared__ double w[];   // x[b] (m doubles)
  const int b = blockIdx.y;
  const double* Ub = U + (int64_t)b * su;
  for (int r = threadIdx.x; r < m; r += kWG) w[r] = x[(int64_t)b * sx + r];
  __syncthreads();
  const int c = blockIdx.x * kColsT + 2 * threadIdx.x;
  if (c >= n) return;
  double a0 = 0.0, a1 = 0.0;
  if (VEC && c + 1 < n) {
    const double* p = Ub + c;
    int r = 0;
    for (; r + 4 <= m; r += 4) {   // four rows in flight per thread
      const double2 u0 = *reinterpret_cast<const double2*>(p + (int64_t)r * ldu);
      const double2 u1 = *reinterpret_cast<const double2*>(p + (int64_t)(r + 1) * ldu);
      const double2 u2 = *reinterpret_cast<const double2*>(p + (int64_t)(r + 2) * ldu);
      const double2 u3 = *reinterpret_cast<const double2*>(p + (int64_t)(r + 3) * ldu);
      a0 = fma(u3.x, w[r + 3], fma(u2.x, w[r + 2], fma(u1.x, w[r + 1], fma(u0.x, w[r], a0))));
      a1 = fma(u3.y, w[r + 3], fma(u2.y, w[r + 2], fma(u1.y, w[r + 1], fma(u0.y, w[r], a1))));
    }
    for (; r < m; ++r) {
      const double2 u = *reinterpret_cast<const double2*>(p + (int64_t)r * ldu);
      a0 = fma(u.x, w[r], a0);
      a1 = fma(u.y, w[r], a1);
    }
    y[(int64_t)b * sy + c] = a0;
    y[(int64_t)b * sy + c + 1] = a1;
  } else {
    for (int r = 0; r < m; ++r) {
      a0 = fma(Ub[(int64_t)r * ldu + c], w[r], a0);
      if (c + 1 < n) a1 = fma(Ub[(int64_t)r * ldu + c + 1], w[r], a1);
    }
    y[(int64_t)b * sy + c] = a0;
    if (c + 1 < n) y[(int64_t)b * sy + c + 1] = a1;
  }
}

}  // namespace

extern "C" int pq_gemv_batched(const double* U, int64_t ldu, int64_t su, int32_t m, int32_t n, int32_t batch,
                               int32_t trans, const double* x, int64_t sx, double* y, int64_t sy, void* stream) {
  PQ_CHECK_ARG(U && x && y && m >= 0 && n >= 0 && batch >= 0 && ldu >= n, "pq_gemv_batched: bad arguments");
  PQ_CHECK_ARG(trans == 0 || m <= 8192, "pq_gemv_batched: trans needs m <= 8192 (x staged in LDS)");
  if (m == 0 || n == 0 || batch == 0) return 0;
  hipStream_t str = (hipStream_t)stream;
  const bool vec = (n % 2 == 0) && (ldu % 2 == 0) && (su % 2 == 0) && ((reinterpret_cast<uintptr_t>(U) & 15) == 0) &&
                   (trans == 1 || ((sx % 2 == 0) && (reinterpret_cast<uintptr_t>(x) & 15) == 0));
  if (trans == 0) {
    dim3 grid((m + kRowsN - 1) / kRowsN, batch);
    if (vec) hipLaunchKernelGGL(k_gemv_n<true>, grid, dim3(kWG), 0, str, U, ldu, su, m, n, x, sx, y, sy);
    else hipLaunchKernelGGL(k_gemv_n<false>, grid, dim3(kWG), 0, str, U, ldu, su, m, n, x, sx, y, sy);
  } else {
    dim3 grid((n + kColsT - 1) / kColsT, batch);
    const size_t lds = (size_t)m * sizeof(double);
    if (vec) hipLaunchKernelGGL(k_gemv_t<true>, grid, dim3(kWG), lds, str, U, ldu, su, m, n, x, sx, y, sy);
    else hipLaunchKernelGGL(k_gemv_t<false>, grid, dim3(kWG), lds, str, U, ldu, su, m, n, x, sx, y, sy);
  }
  PQ_CHECK_LAUNCH("pq_gemv_batched");
  return 0;
}
