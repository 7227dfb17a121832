// Device helpers of the K4 polish kernels (polish.hip: dense P; polish_w.hip: window form).
#pragma once
#include "chol_dev.h"
#include "../../include/porqua_hip.h"

namespace pq {

constexpr int PT = 256;
constexpr int PW = PT / 64;

// Optional phase timing (build with -DPQ_PROFILE): wall-clock ticks per phase accumulated
// into the 16 doubles after the work layout of each problem (tools/prof_polish.py).
#ifdef PQ_PROFILE
#define PQ_STAMP(k)                                              \
  do {                                                           \
    __syncthreads();                                             \
    if (threadIdx.x == 0) {                                      \
      const long long now_ = wall_clock64();                     \
      prof[k] += (double)(now_ - t_last_);                       \
      t_last_ = now_;                                            \
    }                                                            \
  } while (0)
#else
#define PQ_STAMP(k) do { } while (0)
#endif


// ---- the compact P_FF storage of the window-form polish (polish_w.hip, and the large free
//      sets of the grouped pipeline, polish_g.hip): diagonal 64x64 tiles of P_FF in full,
//      off-diagonal tiles transposed into the upper half, the Cholesky factor's off-diagonal
//      tiles in the lower half (wg_cholesky<false>) ----------------------------------------
// P_FF (+ dadd on the diagonal) in the compact polish storage described above
struct FormW {
  const double* K;
  int64_t ld;
  int k;
  double dadd;
  __device__ __forceinline__ double operator()(int gi, int gj) const {
    if (gi >= k || gj >= k) return gi == gj ? 1.0 : 0.0;
    double v = ((gi >> 6) == (gj >> 6)) ? K[(int64_t)gi * ld + gj] : K[(int64_t)min(gi, gj) * ld + max(gi, gj)];
    if (gi == gj) v += dadd;
    return v;
  }
};

__device__ __forceinline__ double pc_at(const double* K, int64_t ld, int p, int q) {
  return ((p >> 6) == (q >> 6)) ? K[(int64_t)p * ld + q] : K[(int64_t)min(p, q) * ld + max(p, q)];
}

// P_FF = psw Xc_F' Xc_F + pd I into the compact storage (lower tiles computed; diagonal
// tiles stored in full, off-diagonal tiles transposed into the upper half).  One MFMA
// tile product per lower tile, contracted over the window in 16-row chunks staged into LDS.
PQ_DEVFN void form_pff(const pq_lowrank& lr, int b, const int* Fl, int k, int nbk, double psw,
                         double pd, double* Ks, int64_t ldk, double* smem) {
  const int T = lr.tlen[b];
  const int32_t* rws = lr.rows + (int64_t)b * lr.tmax;
  const double* mu = lr.mu ? lr.mu + (int64_t)b * lr.mu_stride : nullptr;
  const int t = threadIdx.x;
  const int kr = t >> 4, i4 = (t & 15) * 4;
  double* SA = smem;
  double* SB = smem + STAGE;
  const int ntile = nbk * (nbk + 1) / 2;
  for (int tile = 0; tile < ntile; ++tile) {
    int I = (int)((sqrt(8.0 * tile + 1.0) - 1.0) * 0.5);
    while ((I + 1) * (I + 2) / 2 <= tile) ++I;
    while (I * (I + 1) / 2 > tile) --I;
    const int J = tile - I * (I + 1) / 2;
    int ca[4], cb[4];
    double ma[4], mb[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int pa = I * TB + i4 + e, pb_ = J * TB + i4 + e;
      ca[e] = pa < k ? Fl[pa] : -1;
      cb[e] = pb_ < k ? Fl[pb_] : -1;
      ma[e] = (ca[e] >= 0 && mu) ? mu[ca[e]] : 0.0;
      mb[e] = (cb[e] >= 0 && mu) ? mu[cb[e]] : 0.0;
    }
    Acc acc;
    acc.zero();
    // unconditional loads from a clamped row / column, zeroed by a factor after the load (a
    // conditional load makes the compiler wait for every outstanding load there), two chunks
    // ahead of the MFMAs in registers
    auto gather = [&](int t0, double (&va)[4], double (&vb)[4]) {
      const int tt = t0 + kr;
      const bool ok = tt < T;
      const double* row = lr.panel + (int64_t)rws[ok ? tt : 0] * lr.ldp;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const double xa = row[ca[e] >= 0 ? ca[e] : 0], xb = row[cb[e] >= 0 ? cb[e] : 0];
        va[e] = (xa - ma[e]) * ((ok && ca[e] >= 0) ? 1.0 : 0.0);
        vb[e] = (xb - mb[e]) * ((ok && cb[e] >= 0) ? 1.0 : 0.0);
      }
    };
    auto stage = [&](const double (&va)[4], const double (&vb)[4]) {
      __syncthreads();   // the previous chunk's MFMAs are done with SA / SB
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        SA[kr * LDW + i4 + e] = va[e];
        SB[kr * LDW + i4 + e] = vb[e];
      }
      __syncthreads();
    };
    double va0[4], vb0[4], va1[4], vb1[4];
    gather(0, va0, vb0);
    if (KC < T) gather(KC, va1, vb1);
    for (int t0 = 0; t0 < T; t0 += 2 * KC) {
      stage(va0, vb0);
      if (t0 + 2 * KC < T) gather(t0 + 2 * KC, va0, vb0);
      mma_lds(acc, SA, SB, KC);
      if (t0 + KC >= T) break;
      stage(va1, vb1);
      if (t0 + 3 * KC < T) gather(t0 + 3 * KC, va1, vb1);
      mma_lds(acc, SA, SB, KC);
    }
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int nn = 0; nn < 2; ++nn)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int gi = I * TB + acc_row(m, r), gj = J * TB + acc_col(nn);
          const double v = psw * acc.c[m][nn][r] + (gi == gj ? pd : 0.0);
          if (I == J) Ks[(int64_t)gi * ldk + gj] = v;
          else Ks[(int64_t)gj * ldk + gi] = v;
        }
  }
  __syncthreads();
}

// y = L^-1 r  (L in K with ld, block inverses in Dt); r, y, t64 in LDS, length nbk*64.
__device__ void fwd_solve(const double* K, int64_t ld, const double* Dt, int nbk, const double* r,
                          double* y, double* t64, double* y64p) {
  const int t = threadIdx.x, w = wave_id(), l = lane_id();
  const int g4 = l >> 4, c16 = l & 15;
  for (int I = 0; I < nbk; ++I) {
    // t_I = r_I - L[I, :I] y[:I]: 16 lanes per row, four rows per wave at a time (a 16-lane sum
    // per row instead of one full-wave sum per row: a quarter of the serial reductions)
    for (int i0 = 4 * w; i0 < TB; i0 += 4 * PW) {
      const int i = i0 + g4;
      const double* row = K + (int64_t)(I * TB + i) * ld;
      double s = 0.0, s2 = 0.0;   // (two chains; the loop unrolled so its loads issue together)
#pragma unroll 4
      for (int c = c16; c < I * TB; c += 32) {
        const bool in2 = c + 16 < I * TB;   // (clamped, unconditional second load)
        s = fma(row[c], y[c], s);
        s2 = fma(row[in2 ? c + 16 : c], in2 ? y[c + 16] : 0.0, s2);
      }
      s += s2;
#pragma unroll
      for (int o = 8; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
      if (c16 == 0) t64[i] = r[I * TB + i] - s;
    }
    __syncthreads();
    {  // y_I = Dinv_I t_I : 4 threads per output row, 16 independent loads each
      const double* D = Dt + (int64_t)I * TB * TB;
      const int o = t & 63, part = t >> 6;
      double s = 0.0;
#pragma unroll
      for (int c = part * 16; c < part * 16 + 16; ++c) s += D[c * TB + o] * t64[c];   // Dinv[o][c] = Dt[c][o]
      y64p[part * TB + o] = s;
    }
    __syncthreads();
    if (t < TB) y[I * TB + t] = (y64p[t] + y64p[TB + t]) + (y64p[2 * TB + t] + y64p[3 * TB + t]);
    __syncthreads();
  }
}

// fwd_solve for two right-hand sides at once (y = L^-1 r, y2 = L^-1 r2): one pass over L's
// rows and the block inverses instead of two.  t64: 2*64, y64p: 2*4*64 LDS scratch.
__device__ void fwd_solve2(const double* K, int64_t ld, const double* Dt, int nbk, const double* r,
                           const double* r2, double* y, double* y2, double* t64, double* y64p) {
  const int t = threadIdx.x, w = wave_id(), l = lane_id();
  const int g4 = l >> 4, c16 = l & 15;
  for (int I = 0; I < nbk; ++I) {
    for (int i0 = 4 * w; i0 < TB; i0 += 4 * PW) {
      const int i = i0 + g4;
      const double* row = K + (int64_t)(I * TB + i) * ld;
      double s = 0.0, s2 = 0.0, u = 0.0, u2 = 0.0;
#pragma unroll 4
      for (int c = c16; c < I * TB; c += 32) {
        const bool in2 = c + 16 < I * TB;   // (clamped, unconditional second load)
        const double a = row[c], b = row[in2 ? c + 16 : c];
        s = fma(a, y[c], s);
        u = fma(a, y2[c], u);
        s2 = fma(b, in2 ? y[c + 16] : 0.0, s2);
        u2 = fma(b, in2 ? y2[c + 16] : 0.0, u2);
      }
      s += s2;
      u += u2;
#pragma unroll
      for (int o = 8; o > 0; o >>= 1) {
        s += __shfl_xor(s, o, 64);
        u += __shfl_xor(u, o, 64);
      }
      if (c16 == 0) {
        t64[i] = r[I * TB + i] - s;
        t64[TB + i] = r2[I * TB + i] - u;
      }
    }
    __syncthreads();
    {  // y_I = Dinv_I t_I for both
      const double* D = Dt + (int64_t)I * TB * TB;
      const int o = t & 63, part = t >> 6;
      double v = 0.0, v2 = 0.0;
#pragma unroll
      for (int c = part * 16; c < part * 16 + 16; ++c) {
        const double d = D[c * TB + o];   // Dinv[o][c] = Dt[c][o]
        v = fma(d, t64[c], v);
        v2 = fma(d, t64[TB + c], v2);
      }
      y64p[part * TB + o] = v;
      y64p[4 * TB + part * TB + o] = v2;
    }
    __syncthreads();
    if (t < TB) {
      y[I * TB + t] = (y64p[t] + y64p[TB + t]) + (y64p[2 * TB + t] + y64p[3 * TB + t]);
      y2[I * TB + t] = (y64p[4 * TB + t] + y64p[5 * TB + t]) + (y64p[6 * TB + t] + y64p[7 * TB + t]);
    }
    __syncthreads();
  }
}

// x = L^-T y ; part[] is 4*64 LDS scratch.
__device__ void bwd_solve(const double* K, int64_t ld, const double* Dt, int nbk, const double* y,
                          double* x, double* t64, double* part, double* part_out) {
  const int t = threadIdx.x, w = wave_id(), l = lane_id();
  for (int I = nbk - 1; I >= 0; --I) {
    // t_I = y_I - sum_{r >= 64(I+1)} L[r][64I + i] x[r]   (lanes over i, waves split r)
    double s = 0.0, s2 = 0.0;   // (two chains; unrolled so the row loads issue together)
#pragma unroll 4
    for (int r = (I + 1) * TB + w; r < nbk * TB; r += 2 * PW) {
      const bool in2 = r + PW < nbk * TB;   // (clamped, unconditional second load)
      s = fma(K[(int64_t)r * ld + I * TB + l], x[r], s);
      s2 = fma(K[(int64_t)(in2 ? r + PW : r) * ld + I * TB + l], in2 ? x[r + PW] : 0.0, s2);
    }
    part[w * TB + l] = s + s2;
    __syncthreads();
    if (t < TB) t64[t] = y[I * TB + t] - (part[t] + part[TB + t] + part[2 * TB + t] + part[3 * TB + t]);
    __syncthreads();
    {  // x_I = Dinv_I' t_I : (Dinv')[o][c] = Dt[o][c], 4 threads per output
      const double* D = Dt + (int64_t)I * TB * TB;
      const int o = t & 63, part = t >> 6;
      double v = 0.0;
#pragma unroll
      for (int c = part * 16; c < part * 16 + 16; ++c) v += D[o * TB + c] * t64[c];
      part_out[part * TB + o] = v;
    }
    __syncthreads();
    if (t < TB) x[I * TB + t] = (part_out[t] + part_out[TB + t]) + (part_out[2 * TB + t] + part_out[3 * TB + t]);
    __syncthreads();
  }
}

__device__ __forceinline__ int block_or(int v, double* red) {
  return block_max((double)v, red) > 0.5;
}

// emit(p, P[row(p)] . v) for p < cnt: full rows of the dense symmetric P (n <= 1024
// columns), v held in registers (lane l owns columns 128 q + 2 l, 2 l + 1; v must be zero
// from n up to the next even index), 16-B loads, two rows per wave in flight.  Called by
// every thread; emit runs on lane 0 of the wave that owns the row.
template <typename RowF, typename EmitF>
__device__ __forceinline__ void rows_dot_vec(const double* P, int64_t ld, int n, int cnt, RowF row_of,
                                             const double* v, EmitF emit) {
  constexpr int NQ = 8;
  const int w = wave_id(), l = lane_id();
  double2 vr[NQ];
#pragma unroll
  for (int qq = 0; qq < NQ; ++qq) {
    const int c = 128 * qq + 2 * l;
    vr[qq] = c < n ? reinterpret_cast<const double2*>(v + c)[0] : double2{0.0, 0.0};
  }
  for (int p = w; p < cnt; p += 2 * PW) {
    const int p1 = p + PW;
    const bool two = p1 < cnt;
    const double2* r0 = reinterpret_cast<const double2*>(P + (int64_t)row_of(p) * ld) + l;
    const double2* r1 = reinterpret_cast<const double2*>(P + (int64_t)row_of(two ? p1 : p) * ld) + l;
    double2 a[NQ], b[NQ];
#pragma unroll
    for (int qq = 0; qq < NQ; ++qq) {
      const bool ok = 128 * qq + 2 * l < n;
      a[qq] = ok ? r0[64 * qq] : double2{0.0, 0.0};
      b[qq] = (ok && two) ? r1[64 * qq] : double2{0.0, 0.0};
    }
    double d0 = 0.0, d1 = 0.0;
#pragma unroll
    for (int qq = 0; qq < NQ; ++qq) {
      d0 = fma(a[qq].x, vr[qq].x, fma(a[qq].y, vr[qq].y, d0));
      d1 = fma(b[qq].x, vr[qq].x, fma(b[qq].y, vr[qq].y, d1));
    }
    d0 = wave_sum(d0);
    d1 = wave_sum(d1);
    if (l == 0) {
      emit(p, d0);
      if (two) emit(p1, d1);
    }
  }
}

// Window passes of P = w_scale Xc'Xc (pq_lowrank), shared by neighbouring dates, so the
// rows are L2-resident.  Columns go in chunks of 1024 (lane l owns columns
// c0 + 128 q + 2 l, + 1 of a chunk; 16-B loads), so n is unbounded.  Vectors in global
// memory must be zero from n to the next even index.
//
// lr_pass1: u_t = Xc_t . x = X_t . x - mu . x for t < T (u in LDS, >= T doubles).  Row t
// is always owned by the same wave, so its partial dot products accumulate across column
// chunks in u[t] without barriers.  Ends with a barrier.
PQ_DEVFN void lr_pass1(const pq_lowrank& lr, int b, int n, const double* x, double* u, double* red) {
  constexpr int NQ = 8, RU = 4, LM = NQ * 128;
  const int t = threadIdx.x, w = wave_id(), l = lane_id();
  const int T = lr.tlen[b];
  const int32_t* rws = lr.rows + (int64_t)b * lr.tmax;
  const double* mu = lr.mu ? lr.mu + (int64_t)b * lr.mu_stride : nullptr;
  double mux = 0.0;
  if (mu) {
    double a = 0.0;
    for (int i = t; i < n; i += PT) a += mu[i] * x[i];
    mux = block_sum(a, red);
  }
  for (int c0 = 0; c0 < n; c0 += LM) {
    double2 vr[NQ];
#pragma unroll
    for (int qq = 0; qq < NQ; ++qq) {
      const int c = c0 + 128 * qq + 2 * l;
      vr[qq] = c < n ? reinterpret_cast<const double2*>(x + c)[0] : double2{0.0, 0.0};
    }
    for (int t0 = w; t0 < T; t0 += RU * PW) {
      double2 r[RU][NQ];
#pragma unroll
      for (int e = 0; e < RU; ++e) {
        const int tt = t0 + e * PW;
        const double2* rp =
            reinterpret_cast<const double2*>(lr.panel + (tt < T ? (int64_t)rws[tt] : 0) * lr.ldp + c0) + l;
#pragma unroll
        for (int qq = 0; qq < NQ; ++qq)
          r[e][qq] = (tt < T && c0 + 128 * qq + 2 * l < n) ? rp[64 * qq] : double2{0.0, 0.0};
      }
      double d[RU];
#pragma unroll
      for (int e = 0; e < RU; ++e) {
        double s0 = 0.0;
#pragma unroll
        for (int qq = 0; qq < NQ; ++qq) s0 = fma(r[e][qq].x, vr[qq].x, fma(r[e][qq].y, vr[qq].y, s0));
        d[e] = wave_sum(s0);
      }
      if (l == 0) {
#pragma unroll
        for (int e = 0; e < RU; ++e)
          if (t0 + e * PW < T) u[t0 + e * PW] = (c0 == 0 ? -mux : u[t0 + e * PW]) + d[e];
      }
    }
  }
  __syncthreads();
}

// lr_pass2: emit(i, (Xc' u)_i) = sum_t u_t X_ti - mu_i sum_t u_t for i < n (u in LDS,
// T entries).  Register accumulators per chunk, then a fixed-order wave tree in `tree`
// (LDS >= 2 * 1024 doubles): bit-reproducible.  emit runs on wave 0.
template <typename EmitF>
__device__ void lr_pass2(const pq_lowrank& lr, int b, int n, const double* u, double* tree, double* red,
                         EmitF emit) {
  constexpr int NQ = 8, RU = 4, LM = NQ * 128;
  const int t = threadIdx.x, w = wave_id(), l = lane_id();
  const int T = lr.tlen[b];
  const int32_t* rws = lr.rows + (int64_t)b * lr.tmax;
  const double* mu = lr.mu ? lr.mu + (int64_t)b * lr.mu_stride : nullptr;
  double su = 0.0;
  if (mu) {
    double a = 0.0;
    for (int tt = t; tt < T; tt += PT) a += u[tt];
    su = block_sum(a, red);
  }
  for (int c0 = 0; c0 < n; c0 += LM) {
    double2 acc[NQ];
#pragma unroll
    for (int qq = 0; qq < NQ; ++qq) acc[qq] = double2{0.0, 0.0};
    for (int t0 = w; t0 < T; t0 += RU * PW) {
      double2 r[RU][NQ];
      double a[RU];
#pragma unroll
      for (int e = 0; e < RU; ++e) {
        const int tt = t0 + e * PW;
        a[e] = tt < T ? u[tt] : 0.0;
        const double2* rp =
            reinterpret_cast<const double2*>(lr.panel + (tt < T ? (int64_t)rws[tt] : 0) * lr.ldp + c0) + l;
#pragma unroll
        for (int qq = 0; qq < NQ; ++qq)
          r[e][qq] = (tt < T && c0 + 128 * qq + 2 * l < n) ? rp[64 * qq] : double2{0.0, 0.0};
      }
#pragma unroll
      for (int e = 0; e < RU; ++e)
#pragma unroll
        for (int qq = 0; qq < NQ; ++qq) {
          acc[qq].x = fma(a[e], r[e][qq].x, acc[qq].x);
          acc[qq].y = fma(a[e], r[e][qq].y, acc[qq].y);
        }
    }
#pragma unroll
    for (int half = PW / 2; half >= 1; half >>= 1) {
      if (w >= half && w < 2 * half) {
        double2* dst = reinterpret_cast<double2*>(tree + (w - half) * LM) + l;
#pragma unroll
        for (int qq = 0; qq < NQ; ++qq) dst[64 * qq] = acc[qq];
      }
      __syncthreads();
      if (w < half) {
        const double2* src = reinterpret_cast<const double2*>(tree + w * LM) + l;
#pragma unroll
        for (int qq = 0; qq < NQ; ++qq) {
          const double2 vv = src[64 * qq];
          acc[qq].x += vv.x;
          acc[qq].y += vv.y;
        }
      }
      __syncthreads();
    }
    if (w == 0) {
#pragma unroll
      for (int qq = 0; qq < NQ; ++qq) {
        const int c = c0 + 128 * qq + 2 * l;
        if (c < n) emit(c, acc[qq].x - (mu ? mu[c] * su : 0.0));
        if (c + 1 < n) emit(c + 1, acc[qq].y - (mu ? mu[c + 1] * su : 0.0));
      }
    }
  }
}

// lr_pass1 for an x supported on k listed columns (x_F compact in LDS, index list Fl in
// LDS): u_t = sum_p X_t,F[p] x_F[p] - mu . x, gathered from the window rows -- k
// instead of n loads per row.  4 rows per wave in flight.  Ends with a barrier.
PQ_DEVFN void lr_pass1_sparse(const pq_lowrank& lr, int b, const int* Fl, int k, const double* xF,
                                double* u, double* red) {
  constexpr int RU = 4;
  const int t = threadIdx.x, w = wave_id(), l = lane_id();
  const int T = lr.tlen[b];
  const int32_t* rws = lr.rows + (int64_t)b * lr.tmax;
  const double* mu = lr.mu ? lr.mu + (int64_t)b * lr.mu_stride : nullptr;
  double mux = 0.0;
  if (mu) {
    double a = 0.0;
    for (int p = t; p < k; p += PT) a += mu[Fl[p]] * xF[p];
    mux = block_sum(a, red);
  }
  for (int t0 = w * RU; t0 < T; t0 += RU * PW) {
    double a[RU];
    const double* row[RU];
#pragma unroll
    for (int e = 0; e < RU; ++e) {
      a[e] = 0.0;
      row[e] = lr.panel + (int64_t)rws[t0 + e < T ? t0 + e : 0] * lr.ldp;
    }
    for (int p = l; p < k; p += 64) {
      const int c = Fl[p];
      const double xv = xF[p];
#pragma unroll
      for (int e = 0; e < RU; ++e) a[e] = fma(row[e][c], xv, a[e]);
    }
#pragma unroll
    for (int e = 0; e < RU; ++e) {
      const double d = wave_sum(a[e]);
      if (l == 0 && t0 + e < T) u[t0 + e] = d - mux;
    }
  }
  __syncthreads();
}

// emit(i, w_scale * (Xc' Xc x)_i) for i < n: both passes (u: LDS >= tmax doubles).
template <typename EmitF>
PQ_DEVFN void lr_px(const pq_lowrank& lr, int b, int n, const double* x, double* u, double* tree,
                      double* red, EmitF emit) {
  const double wsc = lr.w_scale ? lr.w_scale[b] : 1.0;
  lr_pass1(lr, b, n, x, u, red);
  lr_pass2(lr, b, n, u, tree, red, [&](int i, double v) { emit(i, wsc * v); });
}

}  // namespace pq
