// K2: batched KKT formation + blocked Cholesky (+ explicit inverse) on FP64 MFMA.
//
// One 256-thread workgroup per problem (problems are independent rebalance dates; a
// daily backtest has thousands, >> 256 CUs).  Left-looking blocked Cholesky with 64-wide
// block columns: for block column J the update  W_IJ = K_IJ - L_I,<J L_J,<J'  is a
// 64 x 64 x 64J MFMA tile GEMM streamed through LDS; the 64 x 64 diagonal block is
// factored and inverted in LDS; off-diagonal blocks are finished as L_IJ = W_IJ Dinv_J'.
// K = P_eff + sigma I + Cg' R Cg + R_box is formed on the fly the first (and only) time
// each lower tile is read, so the KKT matrix never makes a separate HBM round trip.
// With `invert`, K^-1 = L^-T L^-1 is formed in place (right-to-left trtri, then a
// row-ordered lauum that also mirrors the upper triangle) for the ADMM mat-vecs.
//
// Replaces: isPD's np.linalg.cholesky (src/helper_functions.py:61-67) and the KKT
// factorisation inside qpsolvers' backends (src/qp_problems.py:211-214).
#include "chol_dev.h"
#include "capi_util.h"

namespace pq {

__global__ __launch_bounds__(256, 2) void k_factor(pq_problem pb, pq_state st, const int32_t* idx,
                                                int nidx, pq_settings s, int invert) {
  // exactly CHOL_LDS (80 KiB): two workgroups per CU
  __shared__ __attribute__((aligned(16))) double smem[CHOL_LDS];
  double* stg = smem;                      // 4*STAGE: stream buffers / W image / diag tile
  double* sD = smem + 4 * STAGE;           // 64 x LDW: Dinv image for the current column

  const int b = idx ? idx[blockIdx.x] : (int)blockIdx.x;
  const int ld = pb.ld, n = pb.n, nb = ld / TB;
  double* K = st.K + (int64_t)b * st.K_stride;
  double* Dt = st.Dt + (int64_t)b * st.Dt_stride;
  const double rho = st.rho[b];

  FormCtx f;
  f.P = pb.P + (int64_t)b * pb.P_stride;
  f.ld = ld; f.n = n; f.mg = pb.mg;
  f.ps = pb.p_scale ? pb.p_scale[b] : 1.0;
  f.pd = pb.p_diag ? pb.p_diag[b] : 0.0;
  f.sigma = s.sigma;
  f.Cg = pb.Cg ? pb.Cg + (int64_t)b * pb.Cg_stride : nullptr;
  f.lb = pb.lb ? pb.lb + (int64_t)b * pb.box_stride : nullptr;
  f.ub = pb.ub ? pb.ub + (int64_t)b * pb.box_stride : nullptr;
  f.rho = rho; f.rho_min = s.rho_min; f.eq_scale = s.eq_scale;
  f.lg = pb.mg ? pb.lg + (int64_t)b * pb.g_stride : nullptr;
  f.ug = pb.mg ? pb.ug + (int64_t)b * pb.g_stride : nullptr;

  int info = wg_cholesky(FormOp{&f}, K, ld, nb, n, Dt, smem);
  if (threadIdx.x == 0) {
    st.info[b] = info;
    if (info) st.status[b] = PQ_NON_CONVEX;
  }
  if (info || !invert) return;

  // ---- trtri: W = L^-1 in place, block columns right to left ------------------------
  for (int J = nb - 1; J >= 0; --J) {
    __syncthreads();
    // image SB[k][j] = Dinv[k][j] = Dt[j][k]
    for (int e = threadIdx.x; e < TB * TB; e += blockDim.x) {
      const int k = e >> 6, j = e & 63;
      sD[k * LDW + j] = Dt[(int64_t)J * TB * TB + j * TB + k];
    }
    for (int I = nb - 1; I > J; --I) {
      Acc acc;
      acc.zero();
      // sum_{k=J+1..I} W_Ik L_kJ :  A(i,kk) = W[64I+i][kk] (IK), B(kk,j) = L[kk][64J+j] (KI)
      gemm_stream<MODE_IK, MODE_KI>(acc, stg, K, ld, I * TB, (J + 1) * TB, K, ld, J * TB,
                                    (J + 1) * TB, (I - J) * TB);
      __syncthreads();
      acc_to_lds_T(acc, stg, -1.0);
      __syncthreads();
      Acc o;
      o.zero();
      mma_lds(o, stg, sD, TB);
      acc_store(o, K, ld, I * TB, J * TB);
    }
    __syncthreads();
    for (int e = threadIdx.x; e < TB * TB; e += blockDim.x) {
      const int r = e >> 6, c = e & 63;
      K[(int64_t)(J * TB + r) * ld + J * TB + c] = (c <= r) ? Dt[(int64_t)J * TB * TB + c * TB + r] : 0.0;
    }
  }
  __syncthreads();
  // ---- lauum: K^-1 = W' W, row blocks top to bottom, mirrored ----------------------
  for (int I = 0; I < nb; ++I) {
    for (int J = 0; J <= I; ++J) {
      Acc acc;
      acc.zero();
      gemm_stream<MODE_KI, MODE_KI>(acc, stg, K, ld, I * TB, I * TB, K, ld, J * TB, I * TB,
                                    (nb - I) * TB);
      acc_store(acc, K, ld, I * TB, J * TB);
      if (J < I && invert == 2) acc_store_T(acc, K, ld, J * TB, I * TB);
    }
  }
}

}  // namespace pq

extern "C" int pq_factor_batched(const pq_problem* pb, pq_state* st, const int32_t* idx,
                                 int32_t nidx, const pq_settings* s, int32_t invert,
                                 void* stream) {
  PQ_CHECK_ARG(pb && st && s, "pq_factor_batched: null argument");
  PQ_CHECK_ARG(pb->n > 0 && pb->ld >= pb->n && pb->ld % 64 == 0,
               "pq_factor_batched: need n > 0 and ld a multiple of 64 >= n (n=%d ld=%d)", pb->n, pb->ld);
  PQ_CHECK_ARG(pb->mg >= 0 && pb->mg <= 64, "pq_factor_batched: mg must be in [0, 64] (mg=%d)", pb->mg);
  PQ_CHECK_ARG(pb->mg == 0 || (pb->Cg && pb->lg && pb->ug), "pq_factor_batched: Cg/lg/ug missing");
  PQ_CHECK_ARG((pb->lb == nullptr) == (pb->ub == nullptr), "pq_factor_batched: lb/ub must both be set or both NULL");
  PQ_CHECK_ARG(st->K && st->Dt && st->rho && st->info && st->status, "pq_factor_batched: state buffers missing");
  const int grid = idx ? nidx : pb->batch;
  if (grid <= 0) return 0;
  hipLaunchKernelGGL(pq::k_factor, dim3(grid), dim3(256), 0, (hipStream_t)stream, *pb, *st, idx,
                     nidx, *s, invert);
  PQ_CHECK_LAUNCH("pq_factor_batched");
  return 0;
}
