// Weighted window Gram for the window-form (Woodbury) interior-point methods
// (porqua_amd/ipm_lr.py: the LAD LP of src/optimization.py:296-345 and the QPs with both
// l1 terms of src/qp_problems.py:40-118).
//
// An IPM normal matrix on a window is H = Lam + U' diag(e) U with Lam, e > 0 diagonal and U
// the k x n window rows (k = T (+ a few dense rows) < n).  Woodbury needs only the k x k
// capacitance
//
//     M_b = diag(d_b) + diag(r_b) U_b diag(w_b) U_b' diag(r_b)      (r = sqrt(e), w = 1/Lam)
//
// which changes every IPM iteration (Lam and e do), so there is no band / slide reuse: it is
// one weighted SYRK per date and iteration, 2 k^2 n flop (T = 252, n = 1000: 1.3e8) instead
// of the 2 T n^2 + n^3 / 3 of forming and factoring H itself.  One 256-thread workgroup
// computes one lower 64 x 64 tile of one M_b as FP64 MFMA (16x16x4) products contracted over
// the n columns in 16-wide chunks, double-buffered through LDS (K-major images, pitch LDW);
// the column weight w_c is applied to the A operand while it is staged.  Rows k..k_ld-1 are
// identity padding so K2 (pq_factor_batched) can factor the k_ld x k_ld matrix as is.
#include "common.h"
#include "capi_util.h"

namespace pq {
namespace {

struct WG {
  const double* U; int64_t ldu, su;     // rows of date b: U + b su + t ldu
  const double* w; int64_t sw;          // column weights (b, n)
  const double* r; int64_t sr;          // row scale (b, k), NULL = 1
  const double* d; int64_t sd;          // diagonal (b, k), NULL = 1
  int k, n, k_ld;
  double* M; int64_t sm;                // lower k_ld x k_ld tiles, row-major, batch stride sm
};

// 4 consecutive columns c0 + (t & 3) * 4 + e of tile row i = t >> 2 (scaled by `rs`, and by
// the column weights in LDS when `wl` != NULL); zero outside the matrix
__device__ __forceinline__ void load_row4(double (&v)[4], const double* row, double rs, int c0, int n,
                                          const double* wl) {
  const int cc = (threadIdx.x & 3) * 4;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int c = c0 + cc + e;
    double x = 0.0;
    if (row && c < n) {
      x = row[c] * rs;
      if (wl) x *= wl[cc + e];
    }
    v[e] = x;
  }
}

__device__ __forceinline__ void store_row4(const double (&v)[4], double* S) {
  const int i = threadIdx.x >> 2, cc = (threadIdx.x & 3) * 4;
#pragma unroll
  for (int e = 0; e < 4; ++e) S[(cc + e) * LDW + i] = v[e];
}

__device__ __forceinline__ int tri_row_w(int t) {
  int I = (int)((sqrt(8.0 * t + 1.0) - 1.0) * 0.5);
  while ((I + 1) * (I + 2) / 2 <= t) ++I;
  while (I * (I + 1) / 2 > t) --I;
  return I;
}

__global__ __launch_bounds__(256) void k_wgram(WG g) {
  __shared__ __attribute__((aligned(16))) double smem[4 * STAGE + 2 * KC];
  double* wl = smem + 4 * STAGE;                  // column weights of the current / next chunk
  const int b = blockIdx.y;
  const int I = tri_row_w(blockIdx.x), J = blockIdx.x - I * (I + 1) / 2;
  const int i = threadIdx.x >> 2;
  const int ra_i = I * TB + i, rb_i = J * TB + i;
  const double* Ub = g.U + (int64_t)b * g.su;
  const double* rowa = ra_i < g.k ? Ub + (int64_t)ra_i * g.ldu : nullptr;
  const double* rowb = rb_i < g.k ? Ub + (int64_t)rb_i * g.ldu : nullptr;
  const double sa = (g.r && rowa) ? g.r[(int64_t)b * g.sr + ra_i] : 1.0;
  const double sb = (g.r && rowb) ? g.r[(int64_t)b * g.sr + rb_i] : 1.0;
  const double* wb = g.w + (int64_t)b * g.sw;
  const int n = g.n;
  auto weights = [&](int c0, double* dst) {
    if (threadIdx.x < KC) {
      const int c = c0 + threadIdx.x;
      dst[threadIdx.x] = c < n ? wb[c] : 0.0;
    }
  };
  Acc acc;
  acc.zero();
  double va[4], vb[4];
  weights(0, wl);
  __syncthreads();
  load_row4(va, rowa, sa, 0, n, wl);
  load_row4(vb, rowb, sb, 0, n, nullptr);
  store_row4(va, smem);
  store_row4(vb, smem + STAGE);
  __syncthreads();
  int buf = 0;
  for (int c0 = 0; c0 < n; c0 += KC) {
    const bool more = c0 + KC < n;
    double* wn = wl + ((c0 / KC + 1) & 1) * KC;
    if (more) weights(c0 + KC, wn);
    __syncthreads();
    if (more) {
      load_row4(va, rowa, sa, c0 + KC, n, wn);
      load_row4(vb, rowb, sb, c0 + KC, n, nullptr);
    }
    mma_lds(acc, smem + buf * 2 * STAGE, smem + buf * 2 * STAGE + STAGE, KC);
    if (more) {
      store_row4(va, smem + (buf ^ 1) * 2 * STAGE);
      store_row4(vb, smem + (buf ^ 1) * 2 * STAGE + STAGE);
    }
    __syncthreads();
    buf ^= 1;
  }
  double* M = g.M + (int64_t)b * g.sm;
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int nn = 0; nn < 2; ++nn)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int gi = I * TB + acc_row(m, r), gj = J * TB + acc_col(nn);
        double v = acc.c[m][nn][r];
        if (gi == gj) v += (gi < g.k && g.d) ? g.d[(int64_t)b * g.sd + gi] : 1.0;
        M[(int64_t)gi * g.k_ld + gj] = v;
      }
}

}  // namespace
}  // namespace pq

extern "C" int pq_wgram_batched(const double* U, int64_t ldu, int64_t su, int32_t k, int32_t n, int32_t batch,
                                const double* w, int64_t sw, const double* r, int64_t sr, const double* d,
                                int64_t sd, double* M, int32_t k_ld, int64_t sm, void* stream) {
  PQ_CHECK_ARG(U && w && M, "pq_wgram_batched: NULL U, w or M");
  PQ_CHECK_ARG(k >= 1 && n >= 1 && batch >= 0, "pq_wgram_batched: bad sizes k=%d n=%d batch=%d", k, n, batch);
  PQ_CHECK_ARG(k_ld % 64 == 0 && k_ld >= k, "pq_wgram_batched: k_ld=%d must be a multiple of 64 and >= k=%d",
               k_ld, k);
  PQ_CHECK_ARG(ldu >= n && sw >= n && sm >= (int64_t)k_ld * k_ld, "pq_wgram_batched: bad strides");
  PQ_CHECK_ARG(!r || sr >= k, "pq_wgram_batched: row-scale stride < k");
  PQ_CHECK_ARG(!d || sd >= k, "pq_wgram_batched: diagonal stride < k");
  PQ_CHECK_ARG(batch <= 65535, "pq_wgram_batched: batch %d > 65535 (launch in chunks)", batch);
  if (batch == 0) return 0;
  pq::WG g{U, ldu, su, w, sw, r, sr, d, sd, k, n, k_ld, M, sm};
  const int nt = k_ld / 64;
  hipLaunchKernelGGL(pq::k_wgram, dim3(nt * (nt + 1) / 2, batch), dim3(256), 0, (hipStream_t)stream, g);
  PQ_CHECK_LAUNCH("pq_wgram_batched");
  return 0;
}
