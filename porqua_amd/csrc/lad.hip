// Batched multi-vector products for the LAD interior-point method (porqua_amd/lad.py):
// out[b] = M[b] V[b]  or  out[b] = S[b] - M[b] V[b],  M n x n (row stride ldm), V / S / out
// n x k row-major (k <= 4).  Each LAD iteration applies H^-1 (from K2) and H to a handful of
// right-hand sides; the product is HBM-bound on M (8 n^2 bytes per date), so one wave
// streams whole rows of M with coalesced (16-B when aligned) loads while V sits in LDS, and the k dot products
// of a row share every load of M.  Beyond 1024 columns (the large-n IPM of
// porqua_amd/ipm.py behind the per-QP drop-in) V is read from global memory instead of LDS:
// it is n k doubles, a few hundred KB at most, and stays in L2 across the row blocks.
#include "capi_util.h"

namespace {

constexpr int kWG = 256;          // 4 waves
constexpr int kRowsPerWG = 16;    // 4 rows per wave
constexpr int kMaxN = 1024;       // V staged in LDS up to here
constexpr int kMaxK = 4;

template <int K, bool VEC, bool LDSV>
__global__ __launch_bounds__(kWG) void k_lad_mv(const double* __restrict__ M, int64_t ldm, int64_t sm,
                                                int n, const double* __restrict__ V, int64_t sv,
                                                const double* __restrict__ S, int64_t ss,
                                                double* __restrict__ out, int64_t so) {
  __shared__ double vl[LDSV ? kMaxN * K : 1];
  const int b = blockIdx.y;
  const double* Vb = V + (int64_t)b * sv;
  if (LDSV) {
    for (int i = threadIdx.x; i < n * K; i += kWG) vl[i] = Vb[i];
    __syncthreads();
  }
  const double* v = LDSV ? vl : Vb;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const double* Mb = M + (int64_t)b * sm;
  for (int rr = 0; rr < kRowsPerWG / 4; ++rr) {
    const int r = blockIdx.x * kRowsPerWG + wave * (kRowsPerWG / 4) + rr;
    if (r >= n) break;                       // uniform per wave
    const double* row = Mb + (int64_t)r * ldm;
    double acc[K];
#pragma unroll
    for (int j = 0; j < K; ++j) acc[j] = 0.0;
    if (VEC) {                               // 16-B loads: rows 16-B aligned, n even
      for (int c = 2 * lane; c < n; c += 128) {
        const double2 m = *reinterpret_cast<const double2*>(row + c);
#pragma unroll
        for (int j = 0; j < K; ++j) acc[j] = fma(m.y, v[(c + 1) * K + j], fma(m.x, v[c * K + j], acc[j]));
      }
    } else {
      for (int c = lane; c < n; c += 64) {
        const double m = row[c];
#pragma unroll
        for (int j = 0; j < K; ++j) acc[j] = fma(m, v[c * K + j], acc[j]);
      }
    }
#pragma unroll
    for (int j = 0; j < K; ++j) {
      double a = acc[j];
      for (int off = 32; off > 0; off >>= 1) a += __shfl_xor(a, off, 64);
      acc[j] = a;
    }
    if (lane < K) {
      double a = acc[0];
#pragma unroll
      for (int j = 1; j < K; ++j)
        if (lane == j) a = acc[j];
      const int64_t o = (int64_t)r * K + lane;
      out[(int64_t)b * so + o] = S ? S[(int64_t)b * ss + o] - a : a;
    }
  }
}

template <int K>
void launch(const double* M, int64_t ldm, int64_t sm, int n, int batch, const double* V, int64_t sv,
            const double* S, int64_t ss, double* out, int64_t so, hipStream_t st) {
  dim3 grid((n + kRowsPerWG - 1) / kRowsPerWG, batch);
  const bool vec = (n % 2 == 0) && (ldm % 2 == 0) && (sm % 2 == 0) && ((uintptr_t)M % 16 == 0);
  if (n <= kMaxN) {
    if (vec)
      hipLaunchKernelGGL((k_lad_mv<K, true, true>), grid, dim3(kWG), 0, st, M, ldm, sm, n, V, sv, S, ss, out, so);
    else
      hipLaunchKernelGGL((k_lad_mv<K, false, true>), grid, dim3(kWG), 0, st, M, ldm, sm, n, V, sv, S, ss, out, so);
  } else {
    if (vec)
      hipLaunchKernelGGL((k_lad_mv<K, true, false>), grid, dim3(kWG), 0, st, M, ldm, sm, n, V, sv, S, ss, out, so);
    else
      hipLaunchKernelGGL((k_lad_mv<K, false, false>), grid, dim3(kWG), 0, st, M, ldm, sm, n, V, sv, S, ss, out, so);
  }
}

}  // namespace

extern "C" int pq_lad_mv_batched(const double* M, int64_t ldm, int64_t sm, int32_t n, int32_t batch,
                                 const double* V, int64_t sv, int32_t k, const double* S, int64_t ss,
                                 double* out, int64_t so, void* stream) {
  PQ_CHECK_ARG(M && V && out, "pq_lad_mv_batched: null pointer");
  PQ_CHECK_ARG(n > 0 && ldm >= n && batch >= 0 && batch <= 65535, "pq_lad_mv_batched: bad n / ldm / batch (n=%d)", n);
  PQ_CHECK_ARG(k >= 1 && k <= kMaxK, "pq_lad_mv_batched: k must be in [1, 4] (k=%d)", k);
  PQ_CHECK_ARG(sv >= (int64_t)n * k && so >= (int64_t)n * k && (!S || ss >= (int64_t)n * k),
               "pq_lad_mv_batched: bad vector strides");
  if (batch == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  switch (k) {
    case 1: launch<1>(M, ldm, sm, n, batch, V, sv, S, ss, out, so, st); break;
    case 2: launch<2>(M, ldm, sm, n, batch, V, sv, S, ss, out, so, st); break;
    case 3: launch<3>(M, ldm, sm, n, batch, V, sv, S, ss, out, so, st); break;
    default: launch<4>(M, ldm, sm, n, batch, V, sv, S, ss, out, so, st); break;
  }
  PQ_CHECK_LAUNCH("pq_lad_mv_batched");
  return 0;
}
