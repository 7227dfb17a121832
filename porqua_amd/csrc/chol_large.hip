// K2L: the KKT factorisation of K2 (pq_factor_batched) for LARGE dense problems -- the
// per-QP drop-in at thousands of assets (QuadraticProgram.solve with a dense n x n P,
// src/qp_problems.py:184-216, e.g. the serial Backtest.run of BASELINE configs 4/5 at
// n = 3000 / 5000).  pq_factor_batched runs one workgroup per problem, which is right for
// thousands of rebalance dates but leaves 255 of 256 CUs idle for one 5000 x 5000 matrix;
// here every problem is spread over many workgroups, one 64 x 64 tile each, in launches
// ordered on the stream:
//
//   form      K = ps P + pd I + sigma I + Cg' R Cg + R_box, lower tiles (once)
//   for J:    diag   (1 WG)           L_JJ = chol(K_JJ), Dinv_J = L_JJ^-1 (LDS, one wave)
//             panel  (nb-J-1 WGs)     L_IJ = K_IJ Dinv_J'                 (MFMA)
//             update (m(m+1)/2 WGs)   K_IK -= L_IJ L_KJ'  for J < K <= I  (MFMA, right-looking)
//   invert:   trtri per J, right to left (nb-J WGs): W_IJ = -(sum_{k=J+1..I} W_Ik L_kJ) Dinv_J
//             into the scratch buffer (W = L^-1; column J is written only, later columns
//             only read, so no workgroup races another);
//             lauum (nb(nb+1)/2 WGs): K^-1_IJ = sum_{k>=I} W_kI' W_kJ, over K (whose L is no
//             longer needed), mirrored for invert = 2.
//
// The right-looking order gives the update launches O(nb^2) independent tiles (528 at
// n = 2048) -- the parallelism a single large problem needs.  Total FP64 work n^3/3 (potrf)
// + n^3/3 (trtri) + n^3/3 (lauum) on v_mfma_f64_16x16x4, tiles staged through LDS by the
// shared gemm_stream machinery (common.h).  A problem whose diagonal block fails (not PD)
// records info = first failing column + 1 and status PQ_NON_CONVEX; its later launches
// return at once.
#include "chol_dev.h"
#include "capi_util.h"

namespace pq {

struct LargeCtx {
  pq_problem pb;
  pq_state st;
  const int32_t* idx;
  pq_settings s;
  double* W;           // scratch (trtri output), per launch slot
  int64_t W_stride;
};

__device__ __forceinline__ int lg_problem(const LargeCtx& c) {
  return c.idx ? c.idx[blockIdx.y] : (int)blockIdx.y;
}

// lower-triangle tile t -> (I, J), I >= J (row-major order of the lower triangle)
__device__ __forceinline__ void tri_tile(int t, int& I, int& J) {
  int i = (int)((sqrt(8.0 * t + 1.0) - 1.0) * 0.5);
  while ((i + 1) * (i + 2) / 2 <= t) ++i;
  while (i * (i + 1) / 2 > t) --i;
  I = i;
  J = t - i * (i + 1) / 2;
}

__global__ __launch_bounds__(256) void k_l_form(LargeCtx c) {
  const int b = lg_problem(c);
  const pq_problem& pb = c.pb;
  int I, J;
  tri_tile(blockIdx.x, I, J);
  const int ld = pb.ld;
  FormCtx f;
  f.P = pb.P + (int64_t)b * pb.P_stride;
  f.ld = ld; f.n = pb.n; f.mg = pb.mg;
  f.ps = pb.p_scale ? pb.p_scale[b] : 1.0;
  f.pd = pb.p_diag ? pb.p_diag[b] : 0.0;
  f.sigma = c.s.sigma;
  f.Cg = pb.Cg ? pb.Cg + (int64_t)b * pb.Cg_stride : nullptr;
  f.lb = pb.lb ? pb.lb + (int64_t)b * pb.box_stride : nullptr;
  f.ub = pb.ub ? pb.ub + (int64_t)b * pb.box_stride : nullptr;
  f.rho = c.st.rho[b]; f.rho_min = c.s.rho_min; f.eq_scale = c.s.eq_scale;
  f.lg = pb.mg ? pb.lg + (int64_t)b * pb.g_stride : nullptr;
  f.ug = pb.mg ? pb.ug + (int64_t)b * pb.g_stride : nullptr;
  double* K = c.st.K + (int64_t)b * c.st.K_stride;
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    c.st.info[b] = 0;
  }
  for (int e = threadIdx.x; e < TB * TB; e += blockDim.x) {
    const int i = e >> 6, j = e & 63;
    K[(int64_t)(I * TB + i) * ld + J * TB + j] = form_elem(f, I * TB + i, J * TB + j);
  }
}

// step J, one workgroup per problem: factor + invert the (fully updated) diagonal block
__global__ __launch_bounds__(256) void k_l_diag(LargeCtx c, int J) {
  __shared__ __attribute__((aligned(16))) double T[TB * DP];
  __shared__ __attribute__((aligned(16))) double X[TB * DP];
  const int b = lg_problem(c);
  if (c.st.info[b] != 0) return;
  const int ld = c.pb.ld;
  double* K = c.st.K + (int64_t)b * c.st.K_stride;
  double* Dt = c.st.Dt + (int64_t)b * c.st.Dt_stride;
  for (int e = threadIdx.x; e < TB * TB; e += blockDim.x) {
    const int i = e >> 6, j = e & 63;
    T[i * DP + j] = K[(int64_t)(J * TB + i) * ld + J * TB + j];
  }
  const int nv = c.pb.n - J * TB;
  const int bad = tile_chol_inv64(T, X, nv);
  if (bad) {
    if (threadIdx.x == 0) {
      c.st.info[b] = J * TB + bad;
      c.st.status[b] = PQ_NON_CONVEX;
    }
    return;
  }
  for (int e = threadIdx.x; e < TB * TB; e += blockDim.x) {
    const int i = e >> 6, j = e & 63;
    K[(int64_t)(J * TB + i) * ld + J * TB + j] = (j <= i) ? T[i * DP + j] : 0.0;
    Dt[(int64_t)J * TB * TB + i * TB + j] = X[i * DP + j];     // Dt[i][j] = Dinv[j][i]
  }
}

// image SB[k][j] = Dinv_J[j][k] = Dt[k][j] (for products X Dinv_J')
__device__ __forceinline__ void load_dinv_T(double* sD, const double* Dt, int J) {
  for (int e = threadIdx.x; e < TB * TB; e += blockDim.x) {
    const int k = e >> 6, j = e & 63;
    sD[k * LDW + j] = Dt[(int64_t)J * TB * TB + k * TB + j];
  }
}
// image SB[k][j] = Dinv_J[k][j] = Dt[j][k] (for products X Dinv_J)
__device__ __forceinline__ void load_dinv(double* sD, const double* Dt, int J) {
  for (int e = threadIdx.x; e < TB * TB; e += blockDim.x) {
    const int k = e >> 6, j = e & 63;
    sD[k * LDW + j] = Dt[(int64_t)J * TB * TB + j * TB + k];
  }
}

// step J: L_IJ = K_IJ Dinv_J' for I = J + 1 + blockIdx.x
__global__ __launch_bounds__(256) void k_l_panel(LargeCtx c, int J) {
  __shared__ __attribute__((aligned(16))) double SA[TB * LDW];
  __shared__ __attribute__((aligned(16))) double SB[TB * LDW];
  const int b = lg_problem(c);
  if (c.st.info[b] != 0) return;
  const int I = J + 1 + blockIdx.x;
  const int ld = c.pb.ld;
  double* K = c.st.K + (int64_t)b * c.st.K_stride;
  const double* Dt = c.st.Dt + (int64_t)b * c.st.Dt_stride;
  for (int e = threadIdx.x; e < TB * TB; e += blockDim.x) {
    const int i = e >> 6, k = e & 63;
    SA[k * LDW + i] = K[(int64_t)(I * TB + i) * ld + J * TB + k];
  }
  load_dinv_T(SB, Dt, J);
  __syncthreads();
  Acc o;
  o.zero();
  mma_lds(o, SA, SB, TB);
  acc_store(o, K, ld, I * TB, J * TB);
}

// step J: K_IK -= L_IJ L_KJ' over the trailing lower triangle (tile t of m(m+1)/2)
__global__ __launch_bounds__(256) void k_l_update(LargeCtx c, int J) {
  __shared__ __attribute__((aligned(16))) double stg[4 * STAGE];
  const int b = lg_problem(c);
  if (c.st.info[b] != 0) return;
  int ii, kk;
  tri_tile(blockIdx.x, ii, kk);
  const int I = J + 1 + ii, K2 = J + 1 + kk;
  const int ld = c.pb.ld;
  double* K = c.st.K + (int64_t)b * c.st.K_stride;
  Acc acc;
  acc.zero();
  gemm_stream<MODE_IK, MODE_IK>(acc, stg, K, ld, I * TB, J * TB, K, ld, K2 * TB, J * TB, TB);
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int nn = 0; nn < 2; ++nn)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        double* p = K + (int64_t)(I * TB + acc_row(m, r)) * ld + K2 * TB + acc_col(nn);
        *p -= acc.c[m][nn][r];
      }
}

// trtri step J (right to left): blockIdx.x == 0 writes W_JJ = Dinv_J; blockIdx.x = d >= 1
// computes W_IJ (I = J + d) = -(sum_{k=J+1..I} W_Ik L_kJ) Dinv_J.
__global__ __launch_bounds__(256) void k_l_trtri(LargeCtx c, int J) {
  __shared__ __attribute__((aligned(16))) double stg[4 * STAGE];
  __shared__ __attribute__((aligned(16))) double sD[TB * LDW];
  const int b = lg_problem(c);
  if (c.st.info[b] != 0) return;
  const int ld = c.pb.ld;
  const double* K = c.st.K + (int64_t)b * c.st.K_stride;
  const double* Dt = c.st.Dt + (int64_t)b * c.st.Dt_stride;
  double* W = c.W + (int64_t)blockIdx.y * c.W_stride;
  if (blockIdx.x == 0) {
    for (int e = threadIdx.x; e < TB * TB; e += blockDim.x) {
      const int r = e >> 6, cc = e & 63;
      W[(int64_t)(J * TB + r) * ld + J * TB + cc] = (cc <= r) ? Dt[(int64_t)J * TB * TB + cc * TB + r] : 0.0;
    }
    return;
  }
  const int I = J + blockIdx.x;
  Acc acc;
  acc.zero();
  // A(i, k) = W[64 I + i][k] (IK), B(k, j) = L[k][64 J + j] (KI), k over [64(J+1), 64(I+1))
  gemm_stream<MODE_IK, MODE_KI>(acc, stg, W, ld, I * TB, (J + 1) * TB, K, ld, J * TB, (J + 1) * TB,
                                (I - J) * TB);
  load_dinv(sD, Dt, J);
  __syncthreads();
  acc_to_lds_T(acc, stg, -1.0);
  __syncthreads();
  Acc o;
  o.zero();
  mma_lds(o, stg, sD, TB);
  acc_store(o, W, ld, I * TB, J * TB);
}

// lauum: K^-1_IJ = sum_{k >= I} W_kI' W_kJ (tile t of the lower triangle); invert = 2 mirrors
__global__ __launch_bounds__(256) void k_l_lauum(LargeCtx c, int nb, int invert) {
  __shared__ __attribute__((aligned(16))) double stg[4 * STAGE];
  const int b = lg_problem(c);
  if (c.st.info[b] != 0) return;
  int I, J;
  tri_tile(blockIdx.x, I, J);
  const int ld = c.pb.ld;
  double* K = c.st.K + (int64_t)b * c.st.K_stride;
  const double* W = c.W + (int64_t)blockIdx.y * c.W_stride;
  Acc acc;
  acc.zero();
  gemm_stream<MODE_KI, MODE_KI>(acc, stg, W, ld, I * TB, I * TB, W, ld, J * TB, I * TB, (nb - I) * TB);
  acc_store(acc, K, ld, I * TB, J * TB);
  if (invert == 2 && J < I) acc_store_T(acc, K, ld, J * TB, I * TB);
}

}  // namespace pq

extern "C" int pq_factor_large(const pq_problem* pb, pq_state* st, const int32_t* idx, int32_t nidx,
                               const pq_settings* s, int32_t invert, double* scratch, int64_t scratch_stride,
                               void* stream) {
  PQ_CHECK_ARG(pb && st && s, "pq_factor_large: null argument");
  PQ_CHECK_ARG(pb->n > 0 && pb->ld >= pb->n && pb->ld % 64 == 0,
               "pq_factor_large: need n > 0 and ld a multiple of 64 >= n (n=%d ld=%d)", pb->n, pb->ld);
  PQ_CHECK_ARG(pb->P, "pq_factor_large: P missing");
  PQ_CHECK_ARG(pb->mg >= 0 && pb->mg <= 64, "pq_factor_large: mg must be in [0, 64] (mg=%d)", pb->mg);
  PQ_CHECK_ARG(pb->mg == 0 || (pb->Cg && pb->lg && pb->ug), "pq_factor_large: Cg/lg/ug missing");
  PQ_CHECK_ARG((pb->lb == nullptr) == (pb->ub == nullptr), "pq_factor_large: lb/ub must both be set or both NULL");
  PQ_CHECK_ARG(st->K && st->Dt && st->rho && st->info && st->status, "pq_factor_large: state buffers missing");
  PQ_CHECK_ARG(st->K_stride >= (int64_t)pb->ld * pb->ld && st->Dt_stride >= (int64_t)(pb->ld / 64) * 4096,
               "pq_factor_large: K / Dt strides too small");
  PQ_CHECK_ARG(invert == 0 || (scratch && scratch_stride >= (int64_t)pb->ld * pb->ld),
               "pq_factor_large: invert needs an ld x ld scratch per problem");
  PQ_CHECK_ARG(invert >= 0 && invert <= 2, "pq_factor_large: invert must be 0, 1 or 2");
  const int grid = idx ? nidx : pb->batch;
  if (grid <= 0) return 0;
  PQ_CHECK_ARG(grid <= 65535, "pq_factor_large: at most 65535 problems per call");
  hipStream_t str = (hipStream_t)stream;
  pq::LargeCtx c;
  c.pb = *pb;
  c.st = *st;
  c.idx = idx;
  c.s = *s;
  c.W = scratch;
  c.W_stride = scratch_stride;
  const int nb = pb->ld / 64;
  const dim3 blk(256);
  hipLaunchKernelGGL(pq::k_l_form, dim3(nb * (nb + 1) / 2, grid), blk, 0, str, c);
  for (int J = 0; J < nb; ++J) {
    hipLaunchKernelGGL(pq::k_l_diag, dim3(1, grid), blk, 0, str, c, J);
    const int m = nb - J - 1;
    if (m > 0) {
      hipLaunchKernelGGL(pq::k_l_panel, dim3(m, grid), blk, 0, str, c, J);
      hipLaunchKernelGGL(pq::k_l_update, dim3(m * (m + 1) / 2, grid), blk, 0, str, c, J);
    }
  }
  if (invert) {
    for (int J = nb - 1; J >= 0; --J)
      hipLaunchKernelGGL(pq::k_l_trtri, dim3(nb - J, grid), blk, 0, str, c, J);
    hipLaunchKernelGGL(pq::k_l_lauum, dim3(nb * (nb + 1) / 2, grid), blk, 0, str, c, nb, invert);
  }
  PQ_CHECK_LAUNCH("pq_factor_large");
  return 0;
}
