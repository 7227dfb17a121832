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


// ---- split-K form for few problems (the slide groups' M_U: 250 at config 3) -------------
// One problem per CU leaves k_factor a single 256-thread workgroup per CU whose streamed tile
// GEMMs wait on one chunk's global loads at a time (latency-bound: ~2 us per 16-deep chunk,
// 300 chunks in sequence for a 320 x 320 factor + inverse).  Here a 512-thread workgroup runs
// two 256-thread teams over the same helpers; every streamed GEMM splits its contraction
// between them (team 0 the first half of the chunks, team 1 the second, in lockstep), and
// team 1's partial tile is added through LDS.  The epilogues (diagonal block, L_IJ = W_IJ
// Dinv', trtri / lauum stores) run on team 0 with the same barriers for both teams.
template <int MA, int MB>
__device__ void gemm_sk(Acc& acc, double* lds2, const double* GA, int64_t lda, int a_i0, int ka0,
                        const double* GB, int64_t ldb, int b_j0, int kb0, int K) {
  const int nc = K / KC;
  if (nc <= 0) return;   // uniform
  const int team = threadIdx.x >> 8;
  const int n0 = (nc + 1) >> 1;
  const int my = team ? nc - n0 : n0;
  const int kofs = team ? n0 * KC : 0;
  double* lds = lds2 + team * 4 * STAGE;
  Stage4 ra, rb;
  __syncthreads();   // (gemm_stream's contract: tiles just stored by other waves, buffers free)
  if (my > 0) {
    stage_load<MA, MB>(ra, rb, GA, lda, a_i0, GB, ldb, b_j0, kofs, ka0, kb0);
    stage_store<MA, MB>(ra, rb, lds, lds + STAGE);
  }
  __syncthreads();
  int buf = 0;
  for (int c = 0; c < n0; ++c) {
    const bool act = c < my, more = c + 1 < my;
    if (more) stage_load<MA, MB>(ra, rb, GA, lda, a_i0, GB, ldb, b_j0, kofs + (c + 1) * KC, ka0, kb0);
    if (act) mma_lds(acc, lds + buf * 2 * STAGE, lds + buf * 2 * STAGE + STAGE, KC);
    if (more) stage_store<MA, MB>(ra, rb, lds + (buf ^ 1) * 2 * STAGE, lds + (buf ^ 1) * 2 * STAGE + STAGE);
    __syncthreads();
    buf ^= 1;
  }
  if (nc > 1) {   // team 1's partial into team 0's accumulator (through team 1's stage buffers)
    double* red = lds2 + 4 * STAGE;
    if (team == 1) acc_to_lds(acc, red, TB, 1.0);
    __syncthreads();
    if (team == 0) {
#pragma unroll
      for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int n = 0; n < 2; ++n)
#pragma unroll
          for (int r = 0; r < 4; ++r) acc.c[m][n][r] += red[acc_row(m, r) * TB + acc_col(n)];
    }
    __syncthreads();
  }
}

__global__ __launch_bounds__(512, 1) void k_factor_sk(pq_problem pb, pq_state st, const int32_t* idx,
                                                   int nidx, pq_settings s, int invert) {
  // 153 KiB (one workgroup per CU): two teams' stage buffers (team 0's also the diagonal
  // tile / W image, team 1's the reduction tile), the Dinv image, the diagonal inverse
  __shared__ __attribute__((aligned(16))) double smem[8 * STAGE + TB * LDW + TB * DP];
  double* stg = smem;
  double* sD = smem + 8 * STAGE;
  double* sX = sD + TB * LDW;
  const int team = threadIdx.x >> 8;
  const int b = idx ? idx[blockIdx.x] : (int)blockIdx.x;
  const int ld = pb.ld, n = pb.n, nb = ld / TB;
  double* K = st.K + (int64_t)b * st.K_stride;
  double* Dt = st.Dt + (int64_t)b * st.Dt_stride;
  FormCtx f;
  f.P = pb.P + (int64_t)b * pb.P_stride;
  f.ld = ld; f.n = n; f.mg = pb.mg;
  f.ps = pb.p_scale ? pb.p_scale[b] : 1.0;
  f.pd = pb.p_diag ? pb.p_diag[b] : 0.0;
  f.sigma = s.sigma;
  f.Cg = pb.Cg ? pb.Cg + (int64_t)b * pb.Cg_stride : nullptr;
  f.lb = pb.lb ? pb.lb + (int64_t)b * pb.box_stride : nullptr;
  f.ub = pb.ub ? pb.ub + (int64_t)b * pb.box_stride : nullptr;
  f.rho = st.rho[b]; f.rho_min = s.rho_min; f.eq_scale = s.eq_scale;
  f.lg = pb.mg ? pb.lg + (int64_t)b * pb.g_stride : nullptr;
  f.ug = pb.mg ? pb.ug + (int64_t)b * pb.g_stride : nullptr;

  // ---- potrf (wg_cholesky's left-looking form) --------------------------------------------
  int info = 0;
  for (int J = 0; J < nb; ++J) {
    Acc acc;
    acc.zero();
    gemm_sk<MODE_IK, MODE_IK>(acc, smem, K, ld, J * TB, 0, K, ld, J * TB, 0, J * TB);
    __syncthreads();
    if (team == 0) {
#pragma unroll
      for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int nn = 0; nn < 2; ++nn)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int i = acc_row(m, r), j = acc_col(nn);
            stg[i * DP + j] = form_elem(f, J * TB + i, J * TB + j) - acc.c[m][nn][r];
          }
    }
    const int bad = tile_chol_inv64(stg, sX, n - J * TB);   // (all 512 threads; waves 4.. idle)
    if (bad) {
      info = J * TB + bad;
      break;   // uniform
    }
    for (int e = threadIdx.x; e < TB * TB; e += blockDim.x) {
      const int i = e >> 6, j = e & 63;
      K[(int64_t)(J * TB + i) * ld + J * TB + j] = (j <= i) ? stg[i * DP + j] : 0.0;
      const double x = sX[i * DP + j];                   // (T^-1)[j][i]
      Dt[(int64_t)J * TB * TB + i * TB + j] = x;         // Dt[c][r] = Dinv[r][c]
      sD[i * LDW + j] = x;                               // image SB[k][j] = Dinv[j][k]
    }
    __syncthreads();
    for (int I = J + 1; I < nb; ++I) {
      acc.zero();
      gemm_sk<MODE_IK, MODE_IK>(acc, smem, K, ld, I * TB, 0, K, ld, J * TB, 0, J * TB);
      __syncthreads();
      if (team == 0) {
#pragma unroll
        for (int m = 0; m < 2; ++m)
#pragma unroll
          for (int nn = 0; nn < 2; ++nn)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int i = acc_row(m, r), k = acc_col(nn);
              stg[k * LDW + i] = form_elem(f, I * TB + i, J * TB + k) - acc.c[m][nn][r];
            }
      }
      __syncthreads();
      if (team == 0) {
        Acc o;
        o.zero();
        mma_lds(o, stg, sD, TB);
        acc_store(o, K, ld, I * TB, J * TB);
      }
    }
  }
  if (threadIdx.x == 0) {
    st.info[b] = info;
    if (info) st.status[b] = PQ_NON_CONVEX;
  }
  if (info || !invert) return;   // uniform

  // ---- trtri: W = L^-1 in place, block columns right to left --------------------------------
  for (int J = nb - 1; J >= 0; --J) {
    __syncthreads();
    for (int e = threadIdx.x; e < TB * TB; e += blockDim.x) {
      const int k = e >> 6, j = e & 63;
      sD[k * LDW + j] = Dt[(int64_t)J * TB * TB + j * TB + k];
    }
    for (int I = nb - 1; I > J; --I) {
      Acc acc;
      acc.zero();
      gemm_sk<MODE_IK, MODE_KI>(acc, smem, K, ld, I * TB, (J + 1) * TB, K, ld, J * TB, (J + 1) * TB, (I - J) * TB);
      __syncthreads();
      if (team == 0) acc_to_lds_T(acc, stg, -1.0);
      __syncthreads();
      if (team == 0) {
        Acc o;
        o.zero();
        mma_lds(o, stg, sD, TB);
        acc_store(o, K, ld, I * TB, J * TB);
      }
    }
    __syncthreads();
    for (int e = threadIdx.x; e < TB * TB; e += blockDim.x) {
      const int r = e >> 6, c = e & 63;
      K[(int64_t)(J * TB + r) * ld + J * TB + c] = (c <= r) ? Dt[(int64_t)J * TB * TB + c * TB + r] : 0.0;
    }
  }
  __syncthreads();
  // ---- lauum: K^-1 = W' W, row blocks top to bottom, mirrored ------------------------------
  for (int I = 0; I < nb; ++I) {
    for (int J = 0; J <= I; ++J) {
      Acc acc;
      acc.zero();
      gemm_sk<MODE_KI, MODE_KI>(acc, smem, K, ld, I * TB, I * TB, K, ld, J * TB, I * TB, (nb - I) * TB);
      if (team == 0) {
        acc_store(acc, K, ld, I * TB, J * TB);
        if (J < I && invert == 2) acc_store_T(acc, K, ld, J * TB, I * TB);
      }
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
  // few problems (at most one per CU: the slide groups' M_U) with an inverse: the split-K
  // 512-thread form; PQ_FACTOR_SK = 0 / 1 forces the choice (A/B)
  static const int sk_env = [] {
    const char* e = getenv("PQ_FACTOR_SK");
    return e ? atoi(e) : -1;
  }();
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const bool sk = sk_env >= 0 ? sk_env > 0 : (invert != 0 && grid <= cus);
  if (sk)
    hipLaunchKernelGGL(pq::k_factor_sk, dim3(grid), dim3(512), 0, (hipStream_t)stream, *pb, *st, idx,
                       nidx, *s, invert);
  else
    hipLaunchKernelGGL(pq::k_factor, dim3(grid), dim3(256), 0, (hipStream_t)stream, *pb, *st, idx,
                       nidx, *s, invert);
  PQ_CHECK_LAUNCH("pq_factor_batched");
  return 0;
}
