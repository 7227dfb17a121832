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

}  // namespace pq

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
