// Shared device helpers for the PorQua MI355X engine (gfx950 / CDNA4, wave64).
//
// FP64 matrix work uses v_mfma_f64_16x16x4_f64.  Lane maps (verified on MI355X by
// tools/microbench.hip, exact-integer check):
//   A operand (16x4):  lane l holds A[i = l & 15][k = l >> 4]
//   B operand (4x16):  lane l holds B[k = l >> 4][j = l & 15]
//   C/D (16x16, 4 regs): reg r of lane l is C[row = (l >> 4) + 4 r][col = l & 15]
// (the f64 C/D map differs from the f32/bf16 maps; see cdna_hip_programming.md §3).
//
// Per-workgroup 64x64 tile GEMM: 256 threads = 4 waves, each wave owns a 32x32 quadrant
// (2x2 MFMA tiles).  Operands are staged through LDS as K-major images S[k][i] with a
// row pitch of 80 doubles (64 + 16 pad): the two 16-lane halves of a ds_read_b64 lane
// group then land 32 banks apart, so fragment reads are bank-conflict free.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// The device helpers a kernel calls from several places (window passes, tile Cholesky,
// P_FF forms): forced inline -- a real call makes the callee keep the calling convention's
// register split and save / restore through scratch (k_admm: 92-308 bytes of scratch per
// lane before).  -DPQ_DEVFN=__device__ leaves the choice to the compiler (A/B builds).
#ifndef PQ_DEVFN
#define PQ_DEVFN __device__ __forceinline__
#endif

namespace pq {

typedef double f64x4 __attribute__((ext_vector_type(4)));

constexpr int TB = 64;          // tile edge
constexpr int KC = 16;          // K chunk staged per step
constexpr int LDW = 80;         // LDS row pitch (doubles) for K-major operand images
constexpr int STAGE = KC * LDW; // doubles per staged operand chunk
constexpr int NTHR = 256;       // threads of a tile-GEMM workgroup

struct Acc {
  f64x4 c[2][2];
  __device__ __forceinline__ void zero() {
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int n = 0; n < 2; ++n) c[m][n] = f64x4{0.0, 0.0, 0.0, 0.0};
  }
};

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }
__device__ __forceinline__ int wave_id() { return threadIdx.x >> 6; }

// Row / column of accumulator element (m, n, r) inside the 64x64 tile for this lane.
// (wave_id() & 3, threadIdx.x & 255 below: a 512-thread workgroup runs the tile GEMM as two
// 256-thread teams, k_factor_sk; the identity for the 256-thread workgroups)
__device__ __forceinline__ int acc_row(int m, int r) {
  return ((wave_id() & 3) >> 1) * 32 + m * 16 + (lane_id() >> 4) + 4 * r;
}
__device__ __forceinline__ int acc_col(int n) {
  return (wave_id() & 1) * 32 + n * 16 + (lane_id() & 15);
}

// acc += SA^T-image x SB-image over `kdepth` (multiple of 4) k rows of the images.
// SA[k][i] holds A[i][k]; SB[k][j] holds B[k][j]; both with pitch LDW.
__device__ __forceinline__ void mma_lds(Acc& acc, const double* SA, const double* SB, int kdepth) {
  const int l = lane_id();
  const int w = wave_id() & 3;
  const int i0 = (w >> 1) * 32 + (l & 15);
  const int j0 = (w & 1) * 32 + (l & 15);
  const int kr = l >> 4;
  for (int kk = 0; kk < kdepth; kk += 4) {
    const double* ra = SA + (kk + kr) * LDW;
    const double* rb = SB + (kk + kr) * LDW;
    double a0 = ra[i0], a1 = ra[i0 + 16];
    double b0 = rb[j0], b1 = rb[j0 + 16];
    acc.c[0][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b0, acc.c[0][0], 0, 0, 0);
    acc.c[0][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b1, acc.c[0][1], 0, 0, 0);
    acc.c[1][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b0, acc.c[1][0], 0, 0, 0);
    acc.c[1][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b1, acc.c[1][1], 0, 0, 0);
  }
}

// ---- staging of one K chunk (KC deep, 64 wide) into an LDS image S[k][i] -------------
// Mode KI: global element (k, i) at G[(k0 + k) * ld + i0 + i]   (contraction index = row)
// Mode IK: global element (k, i) at G[(i0 + i) * ld + k0 + k]   (contraction index = col)
// Each thread moves 4 doubles; all indices inside padded storage (no bounds checks).
struct Stage4 {
  double v[4];
};

__device__ __forceinline__ void load_ki(Stage4& s, const double* G, int64_t ld, int k0, int i0) {
  const int t = threadIdx.x & (NTHR - 1);
  const int k = t >> 4, i = (t & 15) * 4;
  const double2* p = reinterpret_cast<const double2*>(G + (int64_t)(k0 + k) * ld + i0 + i);
  double2 a = p[0], b = p[1];
  s.v[0] = a.x; s.v[1] = a.y; s.v[2] = b.x; s.v[3] = b.y;
}
__device__ __forceinline__ void store_ki(const Stage4& s, double* S) {
  const int t = threadIdx.x & (NTHR - 1);
  const int k = t >> 4, i = (t & 15) * 4;
  double2* p = reinterpret_cast<double2*>(S + k * LDW + i);
  p[0] = double2{s.v[0], s.v[1]};
  p[1] = double2{s.v[2], s.v[3]};
}
__device__ __forceinline__ void load_ik(Stage4& s, const double* G, int64_t ld, int k0, int i0) {
  const int t = threadIdx.x & (NTHR - 1);
  const int i = t >> 2, k = (t & 3) * 4;
  const double2* p = reinterpret_cast<const double2*>(G + (int64_t)(i0 + i) * ld + k0 + k);
  double2 a = p[0], b = p[1];
  s.v[0] = a.x; s.v[1] = a.y; s.v[2] = b.x; s.v[3] = b.y;
}
__device__ __forceinline__ void store_ik(const Stage4& s, double* S) {
  const int t = threadIdx.x & (NTHR - 1);
  const int i = t >> 2, k = (t & 3) * 4;
#pragma unroll
  for (int e = 0; e < 4; ++e) S[(k + e) * LDW + i] = s.v[e];
}

enum { MODE_KI = 0, MODE_IK = 1 };

template <int MA, int MB>
__device__ __forceinline__ void stage_load(Stage4& sa, Stage4& sb, const double* GA, int64_t lda,
                                           int a_i0, const double* GB, int64_t ldb, int b_j0,
                                           int k0, int ka0, int kb0) {
  if (MA == MODE_KI) load_ki(sa, GA, lda, ka0 + k0, a_i0); else load_ik(sa, GA, lda, ka0 + k0, a_i0);
  if (MB == MODE_KI) load_ki(sb, GB, ldb, kb0 + k0, b_j0); else load_ik(sb, GB, ldb, kb0 + k0, b_j0);
}
template <int MA, int MB>
__device__ __forceinline__ void stage_store(const Stage4& sa, const Stage4& sb, double* SA, double* SB) {
  if (MA == MODE_KI) store_ki(sa, SA); else store_ik(sa, SA);
  if (MB == MODE_KI) store_ki(sb, SB); else store_ik(sb, SB);
}

// acc += A(64 x K) * B(K x 64) streamed from global memory through the two LDS stage
// buffers `lds` (4 * STAGE doubles).  A element (i, k) and B element (k, j) are addressed
// per the modes with the contraction index starting at ka0 / kb0 and running K (multiple
// of KC).  Double buffered: the next chunk's global loads are in flight during the MFMAs.
template <int MA, int MB>
__device__ void gemm_stream(Acc& acc, double* lds, const double* GA, int64_t lda, int a_i0, int ka0,
                            const double* GB, int64_t ldb, int b_j0, int kb0, int K) {
  if (K <= 0) return;
  Stage4 ra, rb;
  // Barrier BEFORE the first global load: callers stream tiles that other waves of the
  // workgroup have just stored (e.g. L_{J,J-1} in wg_cholesky), and the stage buffers'
  // previous users must be done before they are overwritten.
  __syncthreads();
  stage_load<MA, MB>(ra, rb, GA, lda, a_i0, GB, ldb, b_j0, 0, ka0, kb0);
  stage_store<MA, MB>(ra, rb, lds, lds + STAGE);
  __syncthreads();
  int buf = 0;
  for (int k0 = 0; k0 < K; k0 += KC) {
    const bool more = (k0 + KC) < K;
    if (more) stage_load<MA, MB>(ra, rb, GA, lda, a_i0, GB, ldb, b_j0, k0 + KC, ka0, kb0);
    mma_lds(acc, lds + buf * 2 * STAGE, lds + buf * 2 * STAGE + STAGE, KC);
    if (more) stage_store<MA, MB>(ra, rb, lds + (buf ^ 1) * 2 * STAGE, lds + (buf ^ 1) * 2 * STAGE + STAGE);
    __syncthreads();
    buf ^= 1;
  }
}

// Write the accumulator (scaled by `alpha`) into a row-major LDS tile T[i][j] (pitch ldt).
__device__ __forceinline__ void acc_to_lds(const Acc& acc, double* T, int ldt, double alpha) {
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int r = 0; r < 4; ++r) T[acc_row(m, r) * ldt + acc_col(n)] = alpha * acc.c[m][n][r];
}
// Write the accumulator into an LDS image S[k][i] = acc(i, k), i.e. as the A operand
// of a following product (transposed placement, pitch LDW).
__device__ __forceinline__ void acc_to_lds_T(const Acc& acc, double* S, double alpha) {
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int r = 0; r < 4; ++r) S[acc_col(n) * LDW + acc_row(m, r)] = alpha * acc.c[m][n][r];
}

// Global tile store of the accumulator: G[(row0 + i) * ld + col0 + j] = acc(i, j).
__device__ __forceinline__ void acc_store(const Acc& acc, double* G, int64_t ld, int row0, int col0) {
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        G[(int64_t)(row0 + acc_row(m, r)) * ld + col0 + acc_col(n)] = acc.c[m][n][r];
}
// Transposed global store: G[(row0 + j) * ld + col0 + i] = acc(i, j).
__device__ __forceinline__ void acc_store_T(const Acc& acc, double* G, int64_t ld, int row0, int col0) {
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        G[(int64_t)(row0 + acc_col(n)) * ld + col0 + acc_row(m, r)] = acc.c[m][n][r];
}

// An opaque zero, re-materialised every time it is evaluated.  Lane ids rebuilt from it at
// the top of an iteration loop (threadIdx.x + loop_zero()) keep LICM from hoisting every
// per-lane address derived from them above the loop, where they stay live across all
// phases and were spilled to scratch (k_admm_gcap: 207 spilled VGPRs -> 41, ADMM 10.8 ->
// 8.6 ms on config 3)
__device__ __forceinline__ int loop_zero() {
  int z;
  asm volatile("s_mov_b32 %0, 0" : "=s"(z));
  return z;
}

// ---- wave-level helpers ---------------------------------------------------------------
__device__ __forceinline__ double readlane_f64(double v, int lane) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), lane);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), lane);
  return __hiloint2double(hi, lo);
}

// lane (l & ~15) | k of every 16-lane row (DPP row_newbcast; k folds to an immediate in
// unrolled loops)
template <int K>
__device__ __forceinline__ double row_bcast16_k(double v) {
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), 0x150 + K, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), 0x150 + K, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double row_bcast16(double v, int k) {
  switch (k) {
    case 0: return row_bcast16_k<0>(v);
    case 1: return row_bcast16_k<1>(v);
    case 2: return row_bcast16_k<2>(v);
    case 3: return row_bcast16_k<3>(v);
    case 4: return row_bcast16_k<4>(v);
    case 5: return row_bcast16_k<5>(v);
    case 6: return row_bcast16_k<6>(v);
    case 7: return row_bcast16_k<7>(v);
    case 8: return row_bcast16_k<8>(v);
    case 9: return row_bcast16_k<9>(v);
    case 10: return row_bcast16_k<10>(v);
    case 11: return row_bcast16_k<11>(v);
    case 12: return row_bcast16_k<12>(v);
    case 13: return row_bcast16_k<13>(v);
    case 14: return row_bcast16_k<14>(v);
    default: return row_bcast16_k<15>(v);
  }
}


// One wave, a 16x16 SPD block in the MFMA C layout (lane l holds A[(l>>4) + 4q][l&15], both
// triangles; identity padding): right-looking Cholesky with the inverse of the factor built
// in the same serial chain of 16 steps -- the pivot by readlane, row kk by one cross-lane
// permute, column kk by a DPP row broadcast (lane kk of every 16-lane row), the trailing
// update and the inverse's row operations in registers.  On return A holds L (lower, column
// layout as above; the strictly upper part is stale) and Bv = L^-1; returns 1 when a pivot is
// not positive (uniform), 0 otherwise.
// (l: the lane id; callers that inline several chains pass one rebuilt from loop_zero(), so
// the chain's per-lane masks are not hoisted and held live across all of them)
__device__ __forceinline__ int wave_chol_inv16(double (&A)[4], double (&Bv)[4], const int l) {
  const int cc = l & 15, gg = l >> 4;
  int bad = 0;
#pragma unroll
  for (int kk = 0; kk < 16; ++kk) {
    const int src = ((kk & 3) << 4);
    const double akk = A[kk >> 2];
    const double piv = readlane_f64(akk, src | kk);
    const double rowk = __shfl(akk, src | cc, 64);                   // A[kk][cc] = A[cc][kk]
    const double bkr = __shfl(Bv[kk >> 2], src | cc, 64);            // row kk of the inverse, unscaled
    double colv[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) colv[q] = row_bcast16(A[q], kk);     // A[gg + 4q][kk]
    if (!(piv > 0.0) || !isfinite(piv)) bad = 1;
    double rs = __builtin_amdgcn_rsq(piv);                           // 1/sqrt, two Newton steps
    rs = rs * fma(-0.5 * piv * rs, rs, 1.5);
    rs = rs * fma(-0.5 * piv * rs, rs, 1.5);
    const double bk = bkr * rs;                                      // final row kk of L^-1
    const double lck = cc > kk ? rowk * rs : 0.0;                    // L[cc][kk], trailing columns
    // branch-free updates (selects, no exec-mask branches): the masked factors leave every
    // element outside the trailing block unchanged (fma(-0, x, a) = a); register blocks q
    // whose rows all lie above kk have nothing left to update
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (4 * q + 3 < kk) continue;                                  // (compile time)
      const int r = gg + 4 * q;
      const double lrk = colv[q] * rs;                               // L[r][kk]
      const double lrt = r > kk ? lrk : 0.0;
      const double upd = fma(-lrt, lck, A[q]);
      A[q] = (cc == kk && r >= kk) ? lrk : upd;
      const double bu = fma(-lrt, bk, Bv[q]);
      Bv[q] = r == kk ? bk : bu;
    }
  }
  return bad;
}
__device__ __forceinline__ int wave_chol_inv16(double (&A)[4], double (&Bv)[4]) {
  return wave_chol_inv16(A, Bv, lane_id());
}

// XCD-contiguous block order: the hardware deals workgroups round-robin over the 8 XCDs
// (each with its own L2); slot g' = xcd_slot(blockIdx.x) gives XCD x a contiguous range of
// slots, so neighbouring problems (overlapping windows) share one L2.
__device__ __forceinline__ int xcd_slot(int g, int N) {
  const int x = g & 7, q = N >> 3, r = N & 7;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (g >> 3);
}

// ---- workgroup reductions (any block size that is a multiple of 64, <= 1024) ----------
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
  return v;
}
// red must hold >= 16 doubles of LDS.  Result broadcast to every thread.
__device__ __forceinline__ double block_sum(double v, double* red) {
  v = wave_sum(v);
  const int nw = blockDim.x >> 6;
  __syncthreads();
  if (lane_id() == 0) red[wave_id()] = v;
  __syncthreads();
  double s = 0.0;
  for (int w = 0; w < nw; ++w) s += red[w];
  return s;
}
__device__ __forceinline__ double block_max(double v, double* red) {
  v = wave_max(v);
  const int nw = blockDim.x >> 6;
  __syncthreads();
  if (lane_id() == 0) red[wave_id()] = v;
  __syncthreads();
  double s = red[0];
  for (int w = 1; w < nw; ++w) s = fmax(s, red[w]);
  return s;
}

}  // namespace pq
