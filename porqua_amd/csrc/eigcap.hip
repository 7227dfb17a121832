// K2, eigen form: capacitance inverses of many problems that share one window (the
// risk-aversion x date sweep, BASELINE configs[4]) from ONE symmetric eigendecomposition
// per date instead of one Cholesky factorisation per problem.
//
// Problem b (date d = pdate[b]) has the Woodbury capacitance (lowrank.hip)
//     M_b = I + U_b D_b^-1 U_b',   U_b = [sqrt(ps_b) Xc_d ; sqrt(rho_r) Cg_r],  D_b = c_b I
// (uniform box rho, host-checked).  With the centred window Gram Xc_d Xc_d' = V diag(ev) V'
// (the caller's eigendecomposition, one per date) and W = Xc_d Cg', What = V' W:
//     A = I + (ps/c) Xc Xc'  = V diag(a) V',        a_k = 1 + (ps/c) ev_k >= 1
//     B = (sqrt(ps)/c) W R^1/2,  C = I + R^1/2 (Cg Cg') R^1/2 / c,  R = diag(rho_r)
//     S = C - B' A^-1 B   (mg x mg Schur complement),  Q = A^-1 B = V Z,
//     Z = diag(1/a) What R^1/2 sqrt(ps)/c
//     M_b^-1 = [ V diag(1/a) V' + Q S^-1 Q'   -Q S^-1 ]
//              [ -S^-1 Q'                      S^-1   ]
// Nothing of this depends on a factorisation of M_b, so a change of rho (the adaptive-rho
// NEED_REFACTOR rounds) re-forms M_b^-1 from the same eigenvectors, and every problem keeps
// its own rho.  k_eig_border: one workgroup per problem builds a, Z, S^-1, Q, Q S^-1 and the
// border rows; k_eig_tiles: the lower 64 x 64 tiles of V diag(1/a) V' on FP64 MFMA (the
// eigenvector tiles of a date are shared by its problems through L2), plus Q (Q S^-1)' in
// the epilogue, mirrored to the upper triangle.  The output is what pq_factor_batched's
// inverse mode leaves for the ADMM kernels (full symmetric M_b^-1, identity padding).
//
// Replaces the per-(date, lambda) factorisation behind qpsolvers.solve_problem
// (src/qp_problems.py:211-214) for MeanVariance objectives P = 2 lambda Sigma_d
// (src/optimization.py:168-174) swept over lambda.
#include "common.h"
#include "capi_util.h"

namespace pq {

constexpr int EMG = 4;        // general rows supported (budget + up to 3 more)
constexpr int EKMAX = 512;    // k_ld limit (lowrank_shape_ok)

__device__ __forceinline__ double eig_rho(double l, double u, double rho, const pq_settings& s) {
  if (l == u) return rho * s.eq_scale;
  if (isinf(l) && isinf(u)) return s.rho_min;
  return rho;
}

struct EigScal {
  double ps, c;
};

__device__ __forceinline__ EigScal eig_scal(const pq_lowrank& lr, const pq_problem& pb, const double* rho_all,
                                            const pq_settings& s, int b) {
  const double rho = rho_all[b];
  const double ps = (pb.p_scale ? pb.p_scale[b] : 1.0) * (lr.w_scale ? lr.w_scale[b] : 1.0);
  const double pd = pb.p_diag ? pb.p_diag[b] : 0.0;
  const double* lb = pb.lb ? pb.lb + (int64_t)b * pb.box_stride : nullptr;
  const double* ub = pb.ub ? pb.ub + (int64_t)b * pb.box_stride : nullptr;
  return EigScal{ps, s.sigma + pd + (lb ? eig_rho(lb[0], ub[0], rho, s) : 0.0)};
}

// ---- per problem: Schur complement, Q, Q S^-1, border rows, padding ---------------------
__global__ __launch_bounds__(256) void k_eig_border(pq_lowrank lr, pq_problem pb, const double* rho_all,
                                                    pq_settings s, const int32_t* pdate, const double* V,
                                                    const double* evals, const double* What, const double* cc,
                                                    int k_ld, const int32_t* idx, double* Minv_all,
                                                    int64_t M_stride, double* scratch) {
  __shared__ double s_ainv[EKMAX];
  __shared__ double s_z[EKMAX * EMG];
  __shared__ double s_sr[EMG], s_S[EMG * EMG], s_Si[EMG * EMG];
  __shared__ double red[16];
  const int b = idx ? idx[blockIdx.x] : blockIdx.x;
  const int d = pdate[b];
  const int t = threadIdx.x, w = wave_id(), l = lane_id();
  const int T = lr.tmax, mg = pb.mg, k = T + mg;
  const EigScal sc = eig_scal(lr, pb, rho_all, s, b);
  const double a1 = sc.ps / sc.c;
  if (t < mg)
    s_sr[t] = sqrt(eig_rho(pb.lg[(int64_t)b * pb.g_stride + t], pb.ug[(int64_t)b * pb.g_stride + t],
                           rho_all[b], s));
  const double* ev = evals + (int64_t)d * k_ld;
  const double* Wh = What + (int64_t)d * k_ld * EMG;
  __syncthreads();
  const double zs = sqrt(fmax(sc.ps, 0.0)) / sc.c;
  for (int j = t; j < k_ld; j += 256) {
    const double ai = j < T ? 1.0 / fma(a1, ev[j], 1.0) : 0.0;
    s_ainv[j] = ai;
#pragma unroll
    for (int r = 0; r < EMG; ++r) s_z[j * EMG + r] = r < mg ? zs * s_sr[r] * Wh[j * EMG + r] * ai : 0.0;
  }
  // S = C - B' A^-1 B:  S_rs = d_rs + sr_r sr_s cc_rs / c - (ps / c^2) sr_r sr_s sum_k Wh_kr Wh_ks / a_k
  for (int r = 0; r < mg; ++r)
    for (int q = 0; q <= r; ++q) {
      double p = 0.0;
      for (int j = t; j < T; j += 256) p = fma(Wh[j * EMG + r] * Wh[j * EMG + q], s_ainv[j], p);
      p = block_sum(p, red);
      if (t == 0) {
        const double v = (r == q ? 1.0 : 0.0) + s_sr[r] * s_sr[q] * (cc[r * mg + q] / sc.c - a1 / sc.c * p);
        s_S[r * EMG + q] = v;
        s_S[q * EMG + r] = v;
      }
    }
  __syncthreads();
  if (t == 0) {   // S^-1 by Gauss-Jordan (S is SPD: no pivoting), mg <= 4
    double A[EMG][2 * EMG];
    for (int r = 0; r < mg; ++r)
      for (int q = 0; q < 2 * mg; ++q) A[r][q] = q < mg ? s_S[r * EMG + q] : (q - mg == r ? 1.0 : 0.0);
    for (int p = 0; p < mg; ++p) {
      const double inv = 1.0 / A[p][p];
      for (int q = 0; q < 2 * mg; ++q) A[p][q] *= inv;
      for (int r = 0; r < mg; ++r)
        if (r != p) {
          const double f = A[r][p];
          for (int q = 0; q < 2 * mg; ++q) A[r][q] = fma(-f, A[p][q], A[r][q]);
        }
    }
    for (int r = 0; r < EMG; ++r)
      for (int q = 0; q < EMG; ++q) s_Si[r * EMG + q] = (r < mg && q < mg) ? A[r][mg + q] : 0.0;
  }
  __syncthreads();
  double* Mi = Minv_all + (int64_t)b * M_stride;
  double* qq = scratch + (int64_t)b * k_ld * 2 * EMG;   // row i: Q[i][0..4) | (Q S^-1)[i][0..4)
  const double* Vd = V + (int64_t)d * k_ld * k_ld;
  // Q = V Z, one wave per row (lanes over the eigen index: coalesced V rows)
  for (int i = w; i < k_ld; i += 4) {
    double qv[EMG] = {0.0, 0.0, 0.0, 0.0};
    if (i < T && mg > 0) {
      const double* vr = Vd + (int64_t)i * k_ld;
      for (int j = l; j < T; j += 64) {
        const double v = vr[j];
#pragma unroll
        for (int r = 0; r < EMG; ++r) qv[r] = fma(v, s_z[j * EMG + r], qv[r]);
      }
#pragma unroll
      for (int r = 0; r < EMG; ++r) qv[r] = wave_sum(qv[r]);
    }
    double qs[EMG];
#pragma unroll
    for (int r = 0; r < EMG; ++r) {
      double a = 0.0;
#pragma unroll
      for (int q = 0; q < EMG; ++q) a = fma(qv[q], s_Si[q * EMG + r], a);
      qs[r] = a;
    }
    if (l < 2 * EMG) qq[(int64_t)i * 2 * EMG + l] = l < EMG ? qv[l] : qs[l - EMG];
    if (i < T && l < mg) {   // border: M^-1[T + r][i] = M^-1[i][T + r] = -(Q S^-1)[i][r]
      Mi[(int64_t)(T + l) * k_ld + i] = -qs[l];
      Mi[(int64_t)i * k_ld + T + l] = -qs[l];
    }
  }
  // S^-1 block, and identity padding of rows / columns [k, k_ld)
  if (t < mg * mg) Mi[(int64_t)(T + t / mg) * k_ld + T + t % mg] = s_Si[(t / mg) * EMG + t % mg];
  for (int i = k + w; i < k_ld; i += 4)
    for (int j = l; j < k_ld; j += 64) {
      Mi[(int64_t)i * k_ld + j] = i == j ? 1.0 : 0.0;
      Mi[(int64_t)j * k_ld + i] = i == j ? 1.0 : 0.0;
    }
}

// ---- per problem and lower 64 x 64 tile: V diag(1/a) V' + Q (Q S^-1)' ------------------
__global__ __launch_bounds__(256) void k_eig_tiles(pq_lowrank lr, pq_problem pb, const double* rho_all,
                                                   pq_settings s, const int32_t* pdate, const double* V,
                                                   const double* evals, int k_ld, const int32_t* idx,
                                                   double* Minv_all, int64_t M_stride, const double* scratch) {
  __shared__ __attribute__((aligned(16))) double lds[4 * STAGE];
  __shared__ double s_ainv[EKMAX];
  const int b = idx ? idx[blockIdx.y] : blockIdx.y;
  const int d = pdate[b];
  const int t = threadIdx.x;
  const int T = lr.tmax;
  // lower tile (I, J), I >= J, of the T x T block
  int I = 0, rem = blockIdx.x;
  while (rem > I) { rem -= I + 1; ++I; }
  const int J = rem;
  const EigScal sc = eig_scal(lr, pb, rho_all, s, b);
  const double a1 = sc.ps / sc.c;
  const double* ev = evals + (int64_t)d * k_ld;
  for (int j = t; j < k_ld; j += 256) s_ainv[j] = j < T ? 1.0 / fma(a1, ev[j], 1.0) : 0.0;
  const double* Vd = V + (int64_t)d * k_ld * k_ld;
  const int K = (T + KC - 1) / KC * KC;
  Acc acc;
  acc.zero();
  Stage4 ra, rb;
  auto stage = [&](int k0, double* SA, double* SB) {   // SA[k][i] = V[I0+i][k0+k] / a_k, SB[k][j] = V[J0+j][k0+k]
    const int i = t >> 2, kk = (t & 3) * 4;
#pragma unroll
    for (int e = 0; e < 4; ++e) SA[(kk + e) * LDW + i] = ra.v[e] * s_ainv[k0 + kk + e];
    store_ik(rb, SB);
  };
  __syncthreads();
  load_ik(ra, Vd, k_ld, 0, I * TB);
  load_ik(rb, Vd, k_ld, 0, J * TB);
  stage(0, lds, lds + STAGE);
  __syncthreads();
  int buf = 0;
  for (int k0 = 0; k0 < K; k0 += KC) {
    const bool more = (k0 + KC) < K;
    if (more) {
      load_ik(ra, Vd, k_ld, k0 + KC, I * TB);
      load_ik(rb, Vd, k_ld, k0 + KC, J * TB);
    }
    mma_lds(acc, lds + buf * 2 * STAGE, lds + buf * 2 * STAGE + STAGE, KC);
    if (more) stage(k0 + KC, lds + (buf ^ 1) * 2 * STAGE, lds + (buf ^ 1) * 2 * STAGE + STAGE);
    __syncthreads();
    buf ^= 1;
  }
  const double* qq = scratch + (int64_t)b * k_ld * 2 * EMG;
  double* Mi = Minv_all + (int64_t)b * M_stride;
  const int mg = pb.mg;
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int gi = I * TB + acc_row(m, r), gj = J * TB + acc_col(n);
        if (gi < T && gj < T) {
          double v = acc.c[m][n][r];
          for (int g = 0; g < mg; ++g) v = fma(qq[gi * 2 * EMG + g], qq[gj * 2 * EMG + EMG + g], v);
          Mi[(int64_t)gi * k_ld + gj] = v;
          if (I != J) Mi[(int64_t)gj * k_ld + gi] = v;
        }
      }
}

}  // namespace pq

extern "C" int pq_eigcap_form(const pq_lowrank* lr, const pq_problem* pb, const pq_state* st, const pq_settings* s,
                              const int32_t* pdate, const double* V, const double* evals, const double* What,
                              const double* cc, int32_t k_ld, const int32_t* idx, int32_t nidx, double* Minv,
                              int64_t M_stride, double* scratch, void* stream) {
  PQ_CHECK_ARG(lr && pb && st && s && pdate && V && evals && Minv && scratch, "pq_eigcap_form: null argument");
  PQ_CHECK_ARG(lr->tmax > 0 && k_ld % 64 == 0 && k_ld <= pq::EKMAX && k_ld >= lr->tmax + pb->mg,
               "pq_eigcap_form: need tmax + mg <= k_ld <= 512, k_ld % 64 == 0");
  PQ_CHECK_ARG(pb->mg >= 0 && pb->mg <= pq::EMG && (pb->mg == 0 || (What && cc && pb->lg && pb->ug)),
               "pq_eigcap_form: at most 4 general rows (What, cc, lg, ug needed)");
  PQ_CHECK_ARG(st->rho != nullptr && M_stride >= (int64_t)k_ld * k_ld, "pq_eigcap_form: rho missing / M_stride");
  const int grid = idx ? nidx : pb->batch;
  if (grid <= 0) return 0;
  hipStream_t str = (hipStream_t)stream;
  hipLaunchKernelGGL(pq::k_eig_border, dim3(grid), dim3(256), 0, str, *lr, *pb, st->rho, *s, pdate, V, evals, What,
                     cc, k_ld, idx, Minv, M_stride, scratch);
  PQ_CHECK_LAUNCH("pq_eigcap_form (border)");
  const int nb = (lr->tmax + 63) / 64;
  hipLaunchKernelGGL(pq::k_eig_tiles, dim3(nb * (nb + 1) / 2, grid), dim3(256), 0, str, *lr, *pb, st->rho, *s, pdate,
                     V, evals, k_ld, idx, Minv, M_stride, scratch);
  PQ_CHECK_LAUNCH("pq_eigcap_form (tiles)");
  return 0;
}
