// Batched symmetric eigensolver (two-sided block Jacobi, FP64) and the PSD projection of
// nearestPD (src/helper_functions.py:29-58) on the device.
//
// The reference repairs a non-PD covariance with Higham's projection: B = (A + A')/2,
// H = V' diag(s) V from B's SVD, A2 = (B + H)/2.  For symmetric B = Q L Q' the SVD gives
// s = |L| and H = Q |L| Q', so A2 = Q max(L, 0) Q': one symmetric eigendecomposition.  The
// shift loop then needs the smallest eigenvalue of the repaired matrix (np.linalg.eigvals).
//
// Algorithm: the ld x ld matrix (zero padded beyond n; ld a multiple of 64) is cut into
// nbk = ld / 32 column blocks.  A sweep is nbk - 1 rounds of the round-robin tournament; in a
// round every pair (I, J) of blocks is one 64 x 64 subproblem [A_II A_IJ; A_JI A_JJ]:
//   k_jac_pairs   one workgroup per pair: the subproblem is diagonalised in LDS by cyclic
//                 Jacobi (32 disjoint rotations per step, round-robin order, until no
//                 off-diagonal entry exceeds tol sqrt|a_pp a_qq|), its 64 x 64 rotation W_P
//                 is written out;
//   k_jac_apply   one workgroup per 64 x 64 tile of the pair grid: A[P, Q] <- W_P' A[P, Q] W_Q
//                 (two MFMA tile products), and V[R, Q] <- V[R, Q] W_Q for the eigenvectors.
// Sweeps repeat until a whole sweep rotates nothing (device flags: the launches of a
// converged matrix return at once, so the host queues max_sweeps sweeps without syncing).
// Padding rows / columns are exactly zero and never rotate (their eigenvalues stay 0 at
// positions >= n).  eigenvalues = diag(A) on exit, unsorted.
#include "common.h"
#include "capi_util.h"

namespace pq {

constexpr int JB = 32;          // column block
constexpr int JS = 64;          // subproblem edge (2 blocks)
constexpr int JP = 65;          // LDS pitch of the subproblem / rotation

struct JacCtx {
  double* A; int64_t a_stride;
  double* V; int64_t v_stride;  // NULL: eigenvalues only
  double* work;                 // per matrix: npairs x 64 x 64 rotations + 2 x nrounds x npairs flags
  int64_t w_stride;
  int ld, n, nbk, npairs, nrounds;
  double tol;
};

// round-robin pairing (circle method): block of position k in round r
__device__ __forceinline__ int rr_member(int k, int r, int nb) {
  return k == 0 ? 0 : ((k - 1 + r) % (nb - 1)) + 1;
}
__device__ __forceinline__ void rr_pair(int i, int r, int nb, int& a, int& b) {
  a = rr_member(i, r, nb);
  b = rr_member(nb - 1 - i, r, nb);
  if (a > b) { const int t = a; a = b; b = t; }
}

__device__ __forceinline__ double* jac_rot(const JacCtx& c, int b, int pair) {
  return c.work + (int64_t)b * c.w_stride + (int64_t)pair * JS * JS;
}
__device__ __forceinline__ double* jac_flags(const JacCtx& c, int b, int parity) {
  return c.work + (int64_t)b * c.w_stride + (int64_t)c.npairs * JS * JS +
         (int64_t)parity * c.nrounds * c.npairs;
}

// did sweep `sweep - 1` rotate anything in matrix b?  (sweep 0: yes)
__device__ bool jac_active(const JacCtx& c, int b, int sweep, double* red) {
  if (sweep == 0) return true;
  const double* f = jac_flags(c, b, (sweep - 1) & 1);
  double any = 0.0;
  for (int i = threadIdx.x; i < c.nrounds * c.npairs; i += blockDim.x) any = fmax(any, f[i]);
  return block_max(any, red) > 0.0;
}

// row index (in the matrix) of subproblem index k of pair blocks (I, J)
__device__ __forceinline__ int sub_row(int k, int I, int J) { return (k < JB ? I : J) * JB + (k & (JB - 1)); }

__global__ __launch_bounds__(256) void k_jac_pairs(JacCtx c, int sweep, int round) {
  __shared__ double S[JS * JP];
  __shared__ double W[JS * JP];
  __shared__ double cs[JS / 2], sn[JS / 2];
  __shared__ int pp[JS / 2], qq[JS / 2];
  __shared__ double red[16];
  __shared__ int rot_flag;
  const int b = blockIdx.y, pair = blockIdx.x;
  double* flag = jac_flags(c, b, sweep & 1) + round * c.npairs + pair;
  if (!jac_active(c, b, sweep, red)) {
    if (threadIdx.x == 0) *flag = 0.0;
    return;
  }
  int I, J;
  rr_pair(pair, round, c.nbk, I, J);
  const double* A = c.A + (int64_t)b * c.a_stride;
  for (int e = threadIdx.x; e < JS * JS; e += blockDim.x) {   // symmetrised: the tile products of
    const int i = e >> 6, j = e & 63;                          // k_jac_apply leave A[P,Q] and A[Q,P]'
    const int ri = sub_row(i, I, J), rj = sub_row(j, I, J);    // equal only to rounding
    S[i * JP + j] = 0.5 * (A[(int64_t)ri * c.ld + rj] + A[(int64_t)rj * c.ld + ri]);
    W[i * JP + j] = (i == j) ? 1.0 : 0.0;
  }
  if (threadIdx.x == 0) rot_flag = 0;
  __syncthreads();
  int any_rot = 0;
  for (int isw = 0; isw < 30; ++isw) {
    int swept = 0;
    for (int step = 0; step < JS - 1; ++step) {
      // thread k < 32: pair k of this step, its rotation (c, s) zeroing S[p][q]
      if (threadIdx.x < JS / 2) {
        const int k = threadIdx.x;
        int p, q;
        rr_pair(k, step, JS, p, q);
        const double apq = S[p * JP + q], app = S[p * JP + p], aqq = S[q * JP + q];
        double cc = 1.0, ss = 0.0;
        if (fabs(apq) > c.tol * sqrt(fabs(app) * fabs(aqq)) && fabs(apq) > 1e-300) {
          const double tau = (aqq - app) / (2.0 * apq);
          const double t = (tau >= 0.0 ? 1.0 : -1.0) / (fabs(tau) + sqrt(1.0 + tau * tau));
          cc = 1.0 / sqrt(1.0 + t * t);
          ss = t * cc;
          rot_flag = 1;   // benign race: every writer stores 1
        }
        cs[k] = cc; sn[k] = ss; pp[k] = p; qq[k] = q;
      }
      __syncthreads();
      // rows: S <- G' S  (row_p' = c row_p - s row_q, row_q' = s row_p + c row_q)
      for (int e = threadIdx.x; e < (JS / 2) * JS; e += blockDim.x) {
        const int k = e >> 6, j = e & 63;
        const double cc = cs[k], ss = sn[k];
        if (ss == 0.0) continue;
        const int p = pp[k], q = qq[k];
        const double a = S[p * JP + j], bq = S[q * JP + j];
        S[p * JP + j] = cc * a - ss * bq;
        S[q * JP + j] = ss * a + cc * bq;
      }
      __syncthreads();
      // columns: S <- S G, W <- W G
      for (int e = threadIdx.x; e < (JS / 2) * JS; e += blockDim.x) {
        const int k = e >> 6, i = e & 63;
        const double cc = cs[k], ss = sn[k];
        if (ss == 0.0) continue;
        const int p = pp[k], q = qq[k];
        const double a = S[i * JP + p], bq = S[i * JP + q];
        S[i * JP + p] = cc * a - ss * bq;
        S[i * JP + q] = ss * a + cc * bq;
        const double wa = W[i * JP + p], wb = W[i * JP + q];
        W[i * JP + p] = cc * wa - ss * wb;
        W[i * JP + q] = ss * wa + cc * wb;
      }
      __syncthreads();
      if (threadIdx.x < JS / 2 && sn[threadIdx.x] != 0.0) {   // the rotated pair is exactly zero
        const int p = pp[threadIdx.x], q = qq[threadIdx.x];
        S[p * JP + q] = 0.0;
        S[q * JP + p] = 0.0;
      }
      __syncthreads();
    }
    swept = rot_flag;
    __syncthreads();
    if (threadIdx.x == 0) rot_flag = 0;
    __syncthreads();
    if (!swept) break;
    any_rot = 1;
  }
  double* R = jac_rot(c, b, pair);
  for (int e = threadIdx.x; e < JS * JS; e += blockDim.x) {
    const int i = e >> 6, j = e & 63;
    R[e] = W[i * JP + j];
  }
  if (threadIdx.x == 0) *flag = any_rot ? 1.0 : 0.0;
}

// tiles 0 .. npairs^2 - 1: A[P, Q] <- W_P' A[P, Q] W_Q; then (with V) tiles of V[R, Q] <- V[R, Q] W_Q
__global__ __launch_bounds__(256) void k_jac_apply(JacCtx c, int sweep, int round) {
  __shared__ __attribute__((aligned(16))) double SA[TB * LDW];
  __shared__ __attribute__((aligned(16))) double SB[TB * LDW];
  __shared__ __attribute__((aligned(16))) double SC[TB * LDW];
  const int b = blockIdx.y;
  const int t = blockIdx.x;
  const int np = c.npairs;
  const double* flags = jac_flags(c, b, sweep & 1) + round * np;
  const bool vtile = t >= np * np;
  const int P = vtile ? -1 : t / np;
  const int Q = vtile ? (t - np * np) % np : t % np;
  const int Rb = vtile ? (t - np * np) / np : -1;
  const bool rq = flags[Q] > 0.0, rp = (P >= 0) && flags[P] > 0.0;
  if (!rq && !rp) return;   // uniform: flags written by the previous launch
  int QI, QJ;
  rr_pair(Q, round, c.nbk, QI, QJ);
  const double* WQ = jac_rot(c, b, Q);
  // SB[k][j] = W_Q[k][j]
  for (int e = threadIdx.x; e < TB * TB; e += blockDim.x) SB[(e >> 6) * LDW + (e & 63)] = WQ[e];
  if (vtile) {
    double* Vm = c.V + (int64_t)b * c.v_stride;
    // SA[k][i] = V[64 Rb + i][sub_row(k)]
    for (int e = threadIdx.x; e < TB * TB; e += blockDim.x) {
      const int i = e >> 6, k = e & 63;
      SA[k * LDW + i] = Vm[(int64_t)(Rb * TB + i) * c.ld + sub_row(k, QI, QJ)];
    }
    __syncthreads();
    Acc o;
    o.zero();
    mma_lds(o, SA, SB, TB);
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int nn = 0; nn < 2; ++nn)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          Vm[(int64_t)(Rb * TB + acc_row(m, r)) * c.ld + sub_row(acc_col(nn), QI, QJ)] = o.c[m][nn][r];
    return;
  }
  int PI, PJ;
  rr_pair(P, round, c.nbk, PI, PJ);
  double* A = c.A + (int64_t)b * c.a_stride;
  // Y = X W_Q: SA[k][i] = X[i][k] = A[sub_row(i, P)][sub_row(k, Q)]
  for (int e = threadIdx.x; e < TB * TB; e += blockDim.x) {
    const int i = e >> 6, k = e & 63;
    SA[k * LDW + i] = A[(int64_t)sub_row(i, PI, PJ) * c.ld + sub_row(k, QI, QJ)];
  }
  __syncthreads();
  Acc y;
  y.zero();
  mma_lds(y, SA, SB, TB);
  __syncthreads();
  acc_to_lds(y, SC, LDW, 1.0);                       // SC[k][j] = Y[k][j]
  const double* WP = jac_rot(c, b, P);
  for (int e = threadIdx.x; e < TB * TB; e += blockDim.x) SA[(e >> 6) * LDW + (e & 63)] = WP[e];   // SA[k][i] = W_P[k][i]
  __syncthreads();
  Acc o;
  o.zero();
  mma_lds(o, SA, SC, TB);
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int nn = 0; nn < 2; ++nn)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        A[(int64_t)sub_row(acc_row(m, r), PI, PJ) * c.ld + sub_row(acc_col(nn), QI, QJ)] = o.c[m][nn][r];
}

// padding rows / columns of A zeroed, V <- I (elementwise; A itself must be symmetric)
__global__ __launch_bounds__(256) void k_jac_init(JacCtx c) {
  const int b = blockIdx.y;
  double* A = c.A + (int64_t)b * c.a_stride;
  const int64_t total = (int64_t)c.ld * c.ld;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int i = (int)(e / c.ld), j = (int)(e % c.ld);
    if (i >= c.n || j >= c.n) A[e] = 0.0;
    if (c.V) c.V[(int64_t)b * c.v_stride + e] = (i == j) ? 1.0 : 0.0;
  }
}

__global__ __launch_bounds__(256) void k_jac_diag(JacCtx c, double* evals, int64_t e_stride) {
  const int b = blockIdx.y;
  const double* A = c.A + (int64_t)b * c.a_stride;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < c.ld; i += gridDim.x * blockDim.x)
    evals[(int64_t)b * e_stride + i] = A[(int64_t)i * c.ld + i];
}

// conv[b] = 1 iff the last queued sweep (index last) rotated nothing in matrix b: every
// off-diagonal entry of every subproblem met the tolerance, i.e. the matrix converged
__global__ __launch_bounds__(256) void k_jac_conv(JacCtx c, int last, int32_t* conv) {
  __shared__ double red[16];
  const int b = blockIdx.x;
  const double* f = jac_flags(c, b, last & 1);
  double any = 0.0;
  for (int i = threadIdx.x; i < c.nrounds * c.npairs; i += blockDim.x) any = fmax(any, f[i]);
  any = block_max(any, red);
  if (threadIdx.x == 0) conv[b] = any > 0.0 ? 0 : 1;
}

// out = V diag(max(lam, 0)) V' (tile (I, J) of the full matrix): Vs = V sqrt(max(lam, 0))
// staged column-scaled into LDS, one MFMA tile product of depth ld
__global__ __launch_bounds__(256) void k_psd_form(const double* V, int64_t v_stride, const double* evals,
                                                  int64_t e_stride, int ld, int n, double* out, int64_t o_stride) {
  __shared__ __attribute__((aligned(16))) double SA[TB * LDW];
  __shared__ __attribute__((aligned(16))) double SB[TB * LDW];
  const int b = blockIdx.y;
  const int nbt = ld / TB;
  const int I = blockIdx.x / nbt, J = blockIdx.x % nbt;
  const double* Vb = V + (int64_t)b * v_stride;
  const double* lam = evals + (int64_t)b * e_stride;
  Acc acc;
  acc.zero();
  for (int k0 = 0; k0 < ld; k0 += TB) {
    __syncthreads();
    for (int e = threadIdx.x; e < TB * TB; e += blockDim.x) {
      const int i = e >> 6, k = e & 63;
      const int kk = k0 + k;
      const double sc = kk < n ? sqrt(fmax(lam[kk], 0.0)) : 0.0;
      SA[k * LDW + i] = Vb[(int64_t)(I * TB + i) * ld + kk] * sc;
      SB[k * LDW + i] = Vb[(int64_t)(J * TB + i) * ld + kk] * sc;
    }
    __syncthreads();
    mma_lds(acc, SA, SB, TB);
  }
  acc_store(acc, out + (int64_t)b * o_stride, ld, I * TB, J * TB);
}

// C = op(A) op(B), all ld x ld (batched; ta / tb: 1 = transposed)
template <int MA, int MB>
__global__ __launch_bounds__(256) void k_tile_gemm(const double* A, int64_t sa, const double* B, int64_t sb,
                                                   double* C, int64_t sc, int ld) {
  __shared__ __attribute__((aligned(16))) double stg[4 * STAGE];
  const int b = blockIdx.y;
  const int nbt = ld / TB;
  const int I = blockIdx.x / nbt, J = blockIdx.x % nbt;
  Acc acc;
  acc.zero();
  // MA == IK: A(i, k) = A[i][k]; KI: A(i, k) = A[k][i].  MB == KI: B(k, j) = B[k][j]; IK: B[j][k]
  gemm_stream<MA, MB>(acc, stg, A + (int64_t)b * sa, ld, I * TB, 0, B + (int64_t)b * sb, ld, J * TB, 0, ld);
  acc_store(acc, C + (int64_t)b * sc, ld, I * TB, J * TB);
}

}  // namespace pq

extern "C" int64_t pq_sym_eig_work_doubles(int32_t ld) {
  const int nbk = ld / pq::JB, np = nbk / 2, nr = nbk - 1;
  return (int64_t)np * pq::JS * pq::JS + 2 * (int64_t)nr * np;
}

extern "C" int pq_sym_eig_batched(double* A, int32_t ld, int64_t a_stride, int32_t n, int32_t batch, double* V,
                                  int64_t v_stride, double* evals, int64_t e_stride, double* work,
                                  int64_t w_stride, int32_t max_sweeps, double tol, void* stream) {
  PQ_CHECK_ARG(A && evals && work, "pq_sym_eig_batched: null argument");
  PQ_CHECK_ARG(ld % 64 == 0 && ld >= n && n > 0 && batch >= 0 && batch <= 65535,
               "pq_sym_eig_batched: need ld a multiple of 64 >= n > 0 (n=%d ld=%d)", n, ld);
  PQ_CHECK_ARG(a_stride >= (int64_t)ld * ld && (!V || v_stride >= (int64_t)ld * ld) && e_stride >= ld,
               "pq_sym_eig_batched: strides too small");
  PQ_CHECK_ARG(w_stride >= pq_sym_eig_work_doubles(ld), "pq_sym_eig_batched: work stride too small");
  PQ_CHECK_ARG(max_sweeps >= 1 && tol > 0.0, "pq_sym_eig_batched: max_sweeps >= 1, tol > 0");
  if (batch == 0) return 0;
  hipStream_t str = (hipStream_t)stream;
  pq::JacCtx c;
  c.A = A; c.a_stride = a_stride; c.V = V; c.v_stride = v_stride;
  c.work = work; c.w_stride = w_stride;
  c.ld = ld; c.n = n; c.nbk = ld / pq::JB; c.npairs = c.nbk / 2; c.nrounds = c.nbk - 1;
  c.tol = tol;
  const dim3 blk(256);
  hipLaunchKernelGGL(pq::k_jac_init, dim3(64, batch), blk, 0, str, c);
  const int ntile = c.npairs * c.npairs + (V ? (ld / 64) * c.npairs : 0);
  for (int s = 0; s < max_sweeps; ++s)
    for (int r = 0; r < c.nrounds; ++r) {
      hipLaunchKernelGGL(pq::k_jac_pairs, dim3(c.npairs, batch), blk, 0, str, c, s, r);
      hipLaunchKernelGGL(pq::k_jac_apply, dim3(ntile, batch), blk, 0, str, c, s, r);
    }
  hipLaunchKernelGGL(pq::k_jac_diag, dim3((ld + 255) / 256, batch), blk, 0, str, c, evals, e_stride);
  PQ_CHECK_LAUNCH("pq_sym_eig_batched");
  return 0;
}

extern "C" int pq_sym_eig_converged(const double* work, int32_t ld, int64_t w_stride, int32_t batch,
                                    int32_t max_sweeps, int32_t* conv, void* stream) {
  PQ_CHECK_ARG(work && conv && ld % 64 == 0 && ld > 0 && batch >= 0 && max_sweeps >= 1,
               "pq_sym_eig_converged: bad arguments");
  PQ_CHECK_ARG(w_stride >= pq_sym_eig_work_doubles(ld), "pq_sym_eig_converged: work stride too small");
  if (batch == 0) return 0;
  pq::JacCtx c{};
  c.work = const_cast<double*>(work); c.w_stride = w_stride;
  c.ld = ld; c.nbk = ld / pq::JB; c.npairs = c.nbk / 2; c.nrounds = c.nbk - 1;
  hipLaunchKernelGGL(pq::k_jac_conv, dim3(batch), dim3(256), 0, (hipStream_t)stream, c, max_sweeps - 1, conv);
  PQ_CHECK_LAUNCH("pq_sym_eig_converged");
  return 0;
}

extern "C" int pq_psd_form_batched(const double* V, int64_t v_stride, const double* evals, int64_t e_stride,
                                   int32_t ld, int32_t n, int32_t batch, double* out, int64_t o_stride, void* stream) {
  PQ_CHECK_ARG(V && evals && out && ld % 64 == 0 && ld >= n && n > 0 && batch >= 0 && batch <= 65535,
               "pq_psd_form_batched: bad arguments");
  if (batch == 0) return 0;
  const int nbt = ld / 64;
  hipLaunchKernelGGL(pq::k_psd_form, dim3(nbt * nbt, batch), dim3(256), 0, (hipStream_t)stream, V, v_stride, evals,
                     e_stride, ld, n, out, o_stride);
  PQ_CHECK_LAUNCH("pq_psd_form_batched");
  return 0;
}

extern "C" int pq_tile_gemm_batched(const double* A, int64_t sa, int32_t ta, const double* B, int64_t sb, int32_t tb,
                                    double* C, int64_t sc, int32_t ld, int32_t batch, void* stream) {
  PQ_CHECK_ARG(A && B && C && ld % 64 == 0 && ld > 0 && batch >= 0 && batch <= 65535,
               "pq_tile_gemm_batched: bad arguments");
  if (batch == 0) return 0;
  const int nbt = ld / 64;
  const dim3 g(nbt * nbt, batch), blk(256);
  hipStream_t str = (hipStream_t)stream;
  if (!ta && !tb) hipLaunchKernelGGL((pq::k_tile_gemm<pq::MODE_IK, pq::MODE_KI>), g, blk, 0, str, A, sa, B, sb, C, sc, ld);
  else if (ta && !tb) hipLaunchKernelGGL((pq::k_tile_gemm<pq::MODE_KI, pq::MODE_KI>), g, blk, 0, str, A, sa, B, sb, C, sc, ld);
  else if (!ta && tb) hipLaunchKernelGGL((pq::k_tile_gemm<pq::MODE_IK, pq::MODE_IK>), g, blk, 0, str, A, sa, B, sb, C, sc, ld);
  else hipLaunchKernelGGL((pq::k_tile_gemm<pq::MODE_KI, pq::MODE_IK>), g, blk, 0, str, A, sa, B, sb, C, sc, ld);
  PQ_CHECK_LAUNCH("pq_tile_gemm_batched");
  return 0;
}
