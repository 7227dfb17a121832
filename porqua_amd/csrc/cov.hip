// K1: batched windowed covariance / Gram on FP64 MFMA, plus the O(T n) window reductions.
//
// The return panel (D_total x n, row-major, resident in HBM) is read through per-date row
// index lists, so a window is `data[index <= rebdate].tail(width)` with weekend rows
// removed exactly as src/builders.py:208-211 selects it; consecutive daily windows share
// T-1 of their T rows, so the panel is served from L2 / Infinity Cache, not HBM.
// Sigma = (X - 1 mu')'(X - 1 mu') * (1/(T-1)) is the two-pass np.cov that
// DataFrame.cov() runs (src/covariance.py:65-66): the mean comes from pq_window_mean and
// is subtracted while staging each 16-row chunk into LDS.  One 256-thread workgroup per
// lower 64x64 output tile and date; each tile is written twice (tile and mirror) so the
// result is the full symmetric matrix PorQua's Covariance.estimate returns.
#include "common.h"
#include "capi_util.h"

namespace pq {

__global__ __launch_bounds__(256) void k_window_mean(const double* panel, int64_t ldp, int n,
                                                     const int32_t* rows, const int32_t* tlen,
                                                     int tmax, double* mu, int64_t mu_stride,
                                                     int geo) {
  const int b = blockIdx.y;
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const int T = tlen[b];
  const int32_t* rw = rows + (int64_t)b * tmax;
  double s = 0.0;
  // (unrolled: eight rows' loads in flight per thread instead of one round trip per row -- the
  // same sums in the same order)
  if (geo) {   // (the loads gathered before the logarithms, whose branches would otherwise
               // wait for every outstanding load)
    int k = 0;
    for (; k + 8 <= T; k += 8) {
      double v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = panel[(int64_t)rw[k + u] * ldp + j];
#pragma unroll
      for (int u = 0; u < 8; ++u) s += log(1.0 + v[u]);
    }
    for (; k < T; ++k) s += log(1.0 + panel[(int64_t)rw[k] * ldp + j]);
    mu[(int64_t)b * mu_stride + j] = exp(s / T) - 1.0;
  } else {
#pragma unroll 8
    for (int k = 0; k < T; ++k) s += panel[(int64_t)rw[k] * ldp + j];
    mu[(int64_t)b * mu_stride + j] = s / T;
  }
}

// diag(Xc'Xc): sum_t (X_tj - mu_j)^2 (mu == NULL: sum_t X_tj^2), one thread per column
__global__ __launch_bounds__(256) void k_window_sumsq(const double* panel, int64_t ldp, int n,
                                                      const int32_t* rows, const int32_t* tlen,
                                                      int tmax, const double* mu, int64_t mu_stride,
                                                      double* out, int64_t out_stride) {
  const int b = blockIdx.y;
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const int T = tlen[b];
  const int32_t* rw = rows + (int64_t)b * tmax;
  const double m = mu ? mu[(int64_t)b * mu_stride + j] : 0.0;
  double s = 0.0;
#pragma unroll 8
  for (int k = 0; k < T; ++k) {
    const double d = panel[(int64_t)rw[k] * ldp + j] - m;
    s = fma(d, d, s);
  }
  out[(int64_t)b * out_stride + j] = s;
}

// Window means and diag(Xc'Xc) of a slide group's dates in one pass over its union rows
// (engine.GroupPlan: date b's window is union[uoff_b, uoff_b + T), offsets nondecreasing,
// one T per group).  One thread per column: the first window is summed directly, each later
// window by adding the rows that enter and subtracting the rows that leave -- T + 2 (G - 1)
// row reads per group instead of G T.  Sums are shifted by the column's first value c
// (sa = sum (x - c), sb = sum (x - c)^2; mu = c + sa / T, dg = sb - sa^2 / T), so neither
// the sliding updates nor the centring cancel: the results match pq_window_mean /
// pq_window_sumsq to a few ulps.
__global__ __launch_bounds__(256) void k_window_moments_grp(const double* panel, int64_t ldp, int n,
                                                            const int32_t* gdates, const int32_t* urows,
                                                            int umax, const int32_t* uoff,
                                                            const int32_t* tlen, double* mu,
                                                            int64_t mu_stride, double* dg,
                                                            int64_t dg_stride) {
  const int g = blockIdx.y;
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const int d0 = gdates[g], d1 = gdates[g + 1];
  const int32_t* ur = urows + (int64_t)g * umax;
  const int T = tlen[d0];
  auto x = [&](int u) { return panel[(int64_t)ur[u] * ldp + j]; };
  int lo = uoff[d0], hi = lo + T;
  const double c = x(lo);
  double sa = 0.0, sb = 0.0;
#pragma unroll 8
  for (int u = lo; u < hi; ++u) {
    const double v = x(u) - c;
    sa += v;
    sb = fma(v, v, sb);
  }
  for (int b = d0;; ) {
    mu[(int64_t)b * mu_stride + j] = c + sa / T;
    dg[(int64_t)b * dg_stride + j] = sb - sa * sa / T;
    if (++b >= d1) break;
    const int nlo = uoff[b], nhi = nlo + T;
    for (int u = hi; u < nhi; ++u) {   // entering
      const double v = x(u) - c;
      sa += v;
      sb = fma(v, v, sb);
    }
    for (int u = lo; u < nlo; ++u) {   // leaving
      const double v = x(u) - c;
      sa -= v;
      sb = fma(-v, v, sb);
    }
    lo = nlo;
    hi = nhi;
  }
}

// Geometric window means of a slide group's dates (src/mean_estimation.py:39-48, the
// k_window_mean geo arithmetic: exp(sum log(1 + x) / T) - 1) in one sliding pass over the
// group's union rows: the first window's log sum directly, each later one by the rows that
// enter and leave -- T + 2 (G - 1) logarithms per column and group instead of G T.
__global__ __launch_bounds__(256) void k_window_geomean_grp(const double* panel, int64_t ldp, int n,
                                                            const int32_t* gdates, const int32_t* urows,
                                                            int umax, const int32_t* uoff,
                                                            const int32_t* tlen, double* mu,
                                                            int64_t mu_stride) {
  const int g = blockIdx.y;
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const int d0 = gdates[g], d1 = gdates[g + 1];
  const int32_t* ur = urows + (int64_t)g * umax;
  const int T = tlen[d0];
  // the rows' loads gathered before their logarithms (whose branches would otherwise wait for
  // every outstanding load): 8 at a time for the first window, 4 for the entering / leaving
  // runs -- the same sums in the same order
  auto xv = [&](int u) { return panel[(int64_t)ur[u] * ldp + j]; };
  int lo = uoff[d0], hi = lo + T;
  double s = 0.0;
  {
    int u = lo;
    for (; u + 8 <= hi; u += 8) {
      double v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = xv(u + e);
#pragma unroll
      for (int e = 0; e < 8; ++e) s += log(1.0 + v[e]);
    }
    for (; u < hi; ++u) s += log(1.0 + xv(u));
  }
  for (int b = d0;; ) {
    mu[(int64_t)b * mu_stride + j] = exp(s / T) - 1.0;
    if (++b >= d1) break;
    const int nlo = uoff[b], nhi = nlo + T;
    for (int u = hi; u < nhi; u += 4) {   // entering
      double v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = xv(min(u + e, nhi - 1));
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (u + e < nhi) s += log(1.0 + v[e]);
    }
    for (int u = lo; u < nlo; u += 4) {   // leaving
      double v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = xv(min(u + e, nlo - 1));
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (u + e < nlo) s -= log(1.0 + v[e]);
    }
    lo = nlo;
    hi = nhi;
  }
}

__device__ __forceinline__ void tri_index(int t, int& I, int& J) {
  // t enumerates lower tiles row by row: (0,0),(1,0),(1,1),(2,0),...
  I = (int)((sqrt(8.0 * t + 1.0) - 1.0) * 0.5);
  while ((I + 1) * (I + 2) / 2 <= t) ++I;
  while (I * (I + 1) / 2 > t) --I;
  J = t - I * (I + 1) / 2;
}

// stage one 16-row chunk of window columns [c0, c0+64) into image S[k][i] (centred)
__device__ __forceinline__ void load_win(double (&v)[4], const double* panel, int64_t ldp, int n,
                                         const int32_t* rw, int T, int k0, int c0,
                                         const double* mu) {
  const int t = threadIdx.x;
  const int k = t >> 4, i = (t & 15) * 4;
  const int kk = k0 + k;
  const int64_t row = kk < T ? (int64_t)rw[kk] : -1;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int c = c0 + i + e;
    double x = 0.0;
    if (row >= 0 && c < n) {
      x = panel[row * ldp + c];
      if (mu) x -= mu[c];
    }
    v[e] = x;
  }
}
__device__ __forceinline__ void store_win(const double (&v)[4], double* S) {
  const int t = threadIdx.x;
  const int k = t >> 4, i = (t & 15) * 4;
  double2* p = reinterpret_cast<double2*>(S + k * LDW + i);
  p[0] = double2{v[0], v[1]};
  p[1] = double2{v[2], v[3]};
}

__global__ __launch_bounds__(256) void k_syrk(const double* panel, int64_t ldp, int n,
                                              const int32_t* rows, const int32_t* tlen, int tmax,
                                              int mode, const double* mu, int64_t mu_stride,
                                              double* out, int ld, int64_t out_stride) {
  __shared__ __attribute__((aligned(16))) double smem[4 * STAGE];
  const int b = blockIdx.y;
  int I, J;
  tri_index(blockIdx.x, I, J);
  const int T = tlen[b];
  const int32_t* rw = rows + (int64_t)b * tmax;
  const double* m = (mode == 0) ? mu + (int64_t)b * mu_stride : nullptr;
  Acc acc;
  acc.zero();
  double va[4], vb[4];
  load_win(va, panel, ldp, n, rw, T, 0, I * TB, m);
  load_win(vb, panel, ldp, n, rw, T, 0, J * TB, m);
  store_win(va, smem);
  store_win(vb, smem + STAGE);
  __syncthreads();
  int buf = 0;
  for (int k0 = 0; k0 < T; k0 += KC) {
    const bool more = (k0 + KC) < T;
    if (more) {
      load_win(va, panel, ldp, n, rw, T, k0 + KC, I * TB, m);
      load_win(vb, panel, ldp, n, rw, T, k0 + KC, J * TB, m);
    }
    mma_lds(acc, smem + buf * 2 * STAGE, smem + buf * 2 * STAGE + STAGE, KC);
    if (more) {
      store_win(va, smem + (buf ^ 1) * 2 * STAGE);
      store_win(vb, smem + (buf ^ 1) * 2 * STAGE + STAGE);
    }
    __syncthreads();
    buf ^= 1;
  }
  if (mode == 0) {
    const double sc = 1.0 / (double)(T - 1);  // numpy: c *= 1/(N - ddof)
#pragma unroll
    for (int mm = 0; mm < 2; ++mm)
#pragma unroll
      for (int nn = 0; nn < 2; ++nn) acc.c[mm][nn] *= sc;
  }
  double* o = out + (int64_t)b * out_stride;
  acc_store(acc, o, ld, I * TB, J * TB);
  if (I != J) acc_store_T(acc, o, ld, J * TB, I * TB);
}

// ---- windows with missing values: pandas' pairwise-complete covariance -------------------
//
// DataFrame.cov() on a window with NaN (src/covariance.py:65-66, pandas nancorr with cov=True)
// uses, for each pair (i, j), only the rows where both are present: their own pairwise means
// and N_ij - 1 degrees of freedom.  With X~ = (X - c) on present entries and 0 elsewhere
// (c: the column's mean over its present rows, a shift that keeps the correction term small)
// and M the presence mask, every entry follows from four masked Grams:
//     N = M'M,  S_A = X~'M,  S_B = M'X~,  S_2 = X~'X~,
//     Sigma_ij = (S_2 - S_A S_B / N)_ij / (N_ij - 1)      (NaN when N_ij < 2, as pandas)
// -- four 64x64 MFMA tile products per workgroup over the same staged rows.
__device__ __forceinline__ void load_win_masked(double (&v)[4], double (&m)[4], const double* panel, int64_t ldp,
                                                int n, const int32_t* rw, int T, int k0, int c0,
                                                const double* c) {
  const int t = threadIdx.x;
  const int k = t >> 4, i = (t & 15) * 4;
  const int kk = k0 + k;
  const int64_t row = kk < T ? (int64_t)rw[kk] : -1;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int col = c0 + i + e;
    double x = 0.0, p = 0.0;
    if (row >= 0 && col < n) {
      const double v0 = panel[row * ldp + col];
      if (!isnan(v0)) {
        x = v0 - (c ? c[col] : 0.0);
        p = 1.0;
      }
    }
    v[e] = x;
    m[e] = p;
  }
}

__global__ __launch_bounds__(256) void k_syrk_pairwise(const double* panel, int64_t ldp, int n,
                                                       const int32_t* rows, const int32_t* tlen, int tmax,
                                                       const double* shift, int64_t shift_stride, double* out,
                                                       int ld, int64_t out_stride) {
  __shared__ __attribute__((aligned(16))) double smem[8 * STAGE];   // 2 buffers x (xa, ma, xb, mb)
  const int b = blockIdx.y;
  int I, J;
  tri_index(blockIdx.x, I, J);
  const int T = tlen[b];
  const int32_t* rw = rows + (int64_t)b * tmax;
  const double* c = shift ? shift + (int64_t)b * shift_stride : nullptr;
  Acc s2, sa, sb, cn;
  s2.zero();
  sa.zero();
  sb.zero();
  cn.zero();
  double xa[4], ma[4], xb[4], mb[4];
  auto stage = [&](double* S) {
    store_win(xa, S);
    store_win(ma, S + STAGE);
    store_win(xb, S + 2 * STAGE);
    store_win(mb, S + 3 * STAGE);
  };
  load_win_masked(xa, ma, panel, ldp, n, rw, T, 0, I * TB, c);
  load_win_masked(xb, mb, panel, ldp, n, rw, T, 0, J * TB, c);
  stage(smem);
  __syncthreads();
  int buf = 0;
  for (int k0 = 0; k0 < T; k0 += KC) {
    const bool more = (k0 + KC) < T;
    if (more) {
      load_win_masked(xa, ma, panel, ldp, n, rw, T, k0 + KC, I * TB, c);
      load_win_masked(xb, mb, panel, ldp, n, rw, T, k0 + KC, J * TB, c);
    }
    const double* S = smem + buf * 4 * STAGE;
    mma_lds(s2, S, S + 2 * STAGE, KC);
    mma_lds(sa, S, S + 3 * STAGE, KC);
    mma_lds(sb, S + STAGE, S + 2 * STAGE, KC);
    mma_lds(cn, S + STAGE, S + 3 * STAGE, KC);
    if (more) stage(smem + (buf ^ 1) * 4 * STAGE);
    __syncthreads();
    buf ^= 1;
  }
  const double qnan = __builtin_nan("");
#pragma unroll
  for (int mm = 0; mm < 2; ++mm)
#pragma unroll
    for (int nn = 0; nn < 2; ++nn)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const double N = cn.c[mm][nn][r];
        s2.c[mm][nn][r] = N >= 2.0 ? (s2.c[mm][nn][r] - sa.c[mm][nn][r] * sb.c[mm][nn][r] / N) / (N - 1.0) : qnan;
      }
  double* o = out + (int64_t)b * out_stride;
  // padding rows / columns >= n stay 0 like the dense kernel's
#pragma unroll
  for (int mm = 0; mm < 2; ++mm)
#pragma unroll
    for (int nn = 0; nn < 2; ++nn)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (I * TB + acc_row(mm, r) >= n || J * TB + acc_col(nn) >= n) s2.c[mm][nn][r] = 0.0;
  acc_store(s2, o, ld, I * TB, J * TB);
  if (I != J) acc_store_T(s2, o, ld, J * TB, I * TB);
}

// column means over the present (non-NaN) rows of each window (NaN when none): the shift
// of k_syrk_pairwise and pandas' skipna DataFrame.mean(); geo: exp(mean log(1 + x)) - 1,
// MeanEstimator.estimate_geometric on a window with gaps (src/mean_estimation.py:39-48)
__global__ __launch_bounds__(256) void k_window_nanmean(const double* panel, int64_t ldp, int n,
                                                        const int32_t* rows, const int32_t* tlen, int tmax,
                                                        double* mu, int64_t mu_stride, int geo) {
  const int b = blockIdx.y;
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const int T = tlen[b];
  const int32_t* rw = rows + (int64_t)b * tmax;
  double s = 0.0;
  int cnt = 0;
  for (int k = 0; k < T; ++k) {
    const double v = panel[(int64_t)rw[k] * ldp + j];
    if (!isnan(v)) {
      s += geo ? log1p(v) : v;
      ++cnt;
    }
  }
  mu[(int64_t)b * mu_stride + j] = cnt ? (geo ? expm1(s / cnt) : s / cnt) : __builtin_nan("");
}

// ---- sliding windows: anchor SYRK + rank-2s updates -----------------------------------
//
// A daily backtest's consecutive windows share T - s of their T rows (s = 1 for daily,
// 21 for monthly rebalancing).  Dates are cut into groups; the first date of a group (the
// anchor) is a full SYRK of its window, shifted by the anchor's own mean c; every later
// date d of the group updates the shifted Gram in registers,
//     S_d = S_{d-1} + sum_{added rows} (x - c)(x - c)' - sum_{dropped rows} (x - c)(x - c)',
// as one MFMA pass over a 2s-deep [added; -dropped] operand, and is written out centred
// by its own two-pass mean mu_d (pq_window_mean):
//     Sigma_d = (S_d - T (mu_d - c)(mu_d - c)') / (T - 1)
// -- algebraically np.cov's two-pass result (src/covariance.py:65-66); the shift keeps
// the correction term at the size of the drift of the mean inside one group.  mode 1
// (uncentred Gram X'X, src/optimization.py:215) uses c = 0 and no correction.  Flops per
// date: 2 s n^2 instead of 2 T n^2; the output (8 n^2 B per date) is the remaining cost,
// written through an LDS tile with 16-B row stores (tile and mirror).
constexpr int SP = 65;   // pitch of the LDS output tile

__device__ __forceinline__ void slide_load(double (&va)[4], double (&vb)[4], const double* panel,
                                           int64_t ldp, int n, const int32_t* add, const int32_t* drop,
                                           int na, int i0, int j0, const double* c) {
  // rows k < na: added (+), na <= k < 2 na: dropped (- on the A side), else zero
  const int t = threadIdx.x;
  const int k = t >> 4, i = (t & 15) * 4;
  int64_t row = -1;
  double sg = 1.0;
  if (k < na) row = add[k];
  else if (k < 2 * na) { row = drop[k - na]; sg = -1.0; }
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    double a = 0.0, b = 0.0;
    if (row >= 0) {
      const int ca = i0 + i + e, cb = j0 + i + e;
      if (ca < n) a = sg * (panel[row * ldp + ca] - (c ? c[ca] : 0.0));
      if (cb < n) b = panel[row * ldp + cb] - (c ? c[cb] : 0.0);
    }
    va[e] = a;
    vb[e] = b;
  }
}

__global__ __launch_bounds__(256) void k_syrk_slide(const double* panel, int64_t ldp, int n,
                                                    const int32_t* rows, const int32_t* tlen, int tmax,
                                                    int mode, const double* mu, int64_t mu_stride,
                                                    double* out, int ld, int64_t out_stride,
                                                    const int32_t* gstart, const int32_t* shift,
                                                    int mirror) {
  __shared__ __attribute__((aligned(16))) double smem[4 * STAGE + TB * SP];
  double* tile = smem + 4 * STAGE;
  int I, J;
  tri_index(blockIdx.x, I, J);
  const int g = blockIdx.y;
  const int d0 = gstart[g], d1 = gstart[g + 1];
  const int T = tlen[d0];
  const double* c = (mode == 0) ? mu + (int64_t)d0 * mu_stride : nullptr;   // the shift
  const int t = threadIdx.x;
  // ---- anchor: full SYRK of the anchor window (identical to k_syrk) ---------------------
  Acc acc;
  acc.zero();
  {
    const int32_t* rw = rows + (int64_t)d0 * tmax;
    double va[4], vb[4];
    load_win(va, panel, ldp, n, rw, T, 0, I * TB, c);
    load_win(vb, panel, ldp, n, rw, T, 0, J * TB, c);
    store_win(va, smem);
    store_win(vb, smem + STAGE);
    __syncthreads();
    int buf = 0;
    for (int k0 = 0; k0 < T; k0 += KC) {
      const bool more = (k0 + KC) < T;
      if (more) {
        load_win(va, panel, ldp, n, rw, T, k0 + KC, I * TB, c);
        load_win(vb, panel, ldp, n, rw, T, k0 + KC, J * TB, c);
      }
      mma_lds(acc, smem + buf * 2 * STAGE, smem + buf * 2 * STAGE + STAGE, KC);
      if (more) {
        store_win(va, smem + (buf ^ 1) * 2 * STAGE);
        store_win(vb, smem + (buf ^ 1) * 2 * STAGE + STAGE);
      }
      __syncthreads();
      buf ^= 1;
    }
  }
  const double sc = (mode == 0) ? 1.0 / (double)(T - 1) : 1.0;
  for (int d = d0; d < d1; ++d) {
    if (d > d0) {
      // ---- slide: + rows entering the window, - rows leaving it (chunks of 8 each) ------
      const int s = shift[d];
      const int32_t* add = rows + (int64_t)d * tmax + (T - s);
      const int32_t* drop = rows + (int64_t)(d - 1) * tmax;
      for (int k0 = 0; k0 < s; k0 += KC / 2) {
        const int na = min(KC / 2, s - k0);
        double va[4], vb[4];
        slide_load(va, vb, panel, ldp, n, add + k0, drop + k0, na, I * TB, J * TB, c);
        store_win(va, smem);
        store_win(vb, smem + STAGE);
        __syncthreads();
        mma_lds(acc, smem, smem + STAGE, (2 * na + 3) & ~3);
        __syncthreads();
      }
    }
    // ---- emit date d: centre by its own mean, scale, stage through LDS ----------------
    const double* md = (mode == 0) ? mu + (int64_t)d * mu_stride : nullptr;
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int nn = 0; nn < 2; ++nn)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int i = acc_row(m, r), j = acc_col(nn);
          double v = acc.c[m][nn][r];
          if (md && d > d0) {
            const int gi = I * TB + i, gj = J * TB + j;
            const double di = gi < n ? md[gi] - c[gi] : 0.0;
            const double dj = gj < n ? md[gj] - c[gj] : 0.0;
            v -= (double)T * (di * dj);   // (di dj) first: bitwise symmetric tiles
          }
          tile[i * SP + j] = v * sc;
        }
    __syncthreads();
    double* o = out + (int64_t)d * out_stride;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int idx = t + 256 * e;
      const int r = idx >> 5, c2 = (idx & 31) * 2;
      reinterpret_cast<double2*>(o + (int64_t)(I * TB + r) * ld + J * TB)[c2 >> 1] =
          double2{tile[r * SP + c2], tile[r * SP + c2 + 1]};
      if (I != J && mirror)
        reinterpret_cast<double2*>(o + (int64_t)(J * TB + r) * ld + I * TB)[c2 >> 1] =
            double2{tile[c2 * SP + r], tile[(c2 + 1) * SP + r]};
    }
    __syncthreads();
  }
}

__global__ __launch_bounds__(256) void k_gram_xy(const double* panel, int64_t ldp, int n,
                                                 const double* bm, const int32_t* rows,
                                                 const int32_t* tlen, int tmax, double* xty,
                                                 int64_t xty_stride, double* yty) {
  __shared__ double red[16];
  const int b = blockIdx.y;
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  const int T = tlen[b];
  const int32_t* rw = rows + (int64_t)b * tmax;
  if (j < n) {
    double s = 0.0;
    for (int k = 0; k < T; ++k) s += panel[(int64_t)rw[k] * ldp + j] * bm[rw[k]];
    xty[(int64_t)b * xty_stride + j] = s;
  }
  if (blockIdx.x == 0) {
    double s = 0.0;
    for (int k = threadIdx.x; k < T; k += blockDim.x) {
      const double v = bm[rw[k]];
      s += v * v;
    }
    s = block_sum(s, red);
    if (threadIdx.x == 0) yty[b] = s;
  }
}

// X'y and y'y for the dates of slide groups (k_window_moments_grp's layout): the first window
// summed, the later ones by the entering / leaving union rows
__global__ __launch_bounds__(256) void k_gram_xy_grp(const double* panel, int64_t ldp, int n, const double* bm,
                                                     const int32_t* gdates, const int32_t* urows, int umax,
                                                     const int32_t* uoff, const int32_t* tlen, double* xty,
                                                     int64_t xty_stride, double* yty, double* dg,
                                                     int64_t dg_stride) {
  const int g = blockIdx.y;
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  const int d0 = gdates[g], d1 = gdates[g + 1];
  const int32_t* ur = urows + (int64_t)g * umax;
  const int T = tlen[d0];
  if (blockIdx.x == 0 && (int)threadIdx.x < d1 - d0) {   // y'y: one thread per date, direct sum
    const int b = d0 + threadIdx.x, lo = uoff[b];
    double s = 0.0;
    for (int u = lo; u < lo + T; ++u) {
      const double v = bm[ur[u]];
      s = fma(v, v, s);
    }
    yty[b] = s;
  }
  if (j >= n) return;
  int lo = uoff[d0], hi = lo + T;
  double s = 0.0, q = 0.0;
#pragma unroll 8
  for (int u = lo; u < hi; ++u) {
    const int r = ur[u];
    const double x = panel[(int64_t)r * ldp + j];
    s = fma(x, bm[r], s);
    q = fma(x, x, q);
  }
  for (int b = d0;; ) {
    xty[(int64_t)b * xty_stride + j] = s;
    if (dg) dg[(int64_t)b * dg_stride + j] = q;
    if (++b >= d1) break;
    const int nlo = uoff[b], nhi = nlo + T;
    for (int u = hi; u < nhi; ++u) {   // entering
      const int r = ur[u];
      const double x = panel[(int64_t)r * ldp + j];
      s = fma(x, bm[r], s);
      q = fma(x, x, q);
    }
    for (int u = lo; u < nlo; ++u) {   // leaving
      const int r = ur[u];
      const double x = panel[(int64_t)r * ldp + j];
      s = fma(-x, bm[r], s);
      q = fma(-x, x, q);
    }
    lo = nlo;
    hi = nhi;
  }
}

}  // namespace pq

static int check_win(const double* panel, int32_t n, const int32_t* rows, const int32_t* tlen,
                     int32_t tmax, int32_t batch) {
  PQ_CHECK_ARG(panel && rows && tlen, "window kernels: null pointer");
  PQ_CHECK_ARG(n > 0 && tmax > 0 && batch >= 0, "window kernels: bad sizes n=%d tmax=%d batch=%d", n, tmax, batch);
  return 0;
}

extern "C" int pq_window_mean(const double* panel, int64_t ldp, int32_t n, const int32_t* rows,
                              const int32_t* tlen, int32_t tmax, int32_t batch, double* mu,
                              int64_t mu_stride, void* stream) {
  if (int e = check_win(panel, n, rows, tlen, tmax, batch)) return e;
  PQ_CHECK_ARG(mu != nullptr, "pq_window_mean: mu is null");
  if (batch == 0) return 0;
  hipLaunchKernelGGL(pq::k_window_mean, dim3((n + 255) / 256, batch), dim3(256), 0,
                     (hipStream_t)stream, panel, ldp, n, rows, tlen, tmax, mu, mu_stride, 0);
  PQ_CHECK_LAUNCH("pq_window_mean");
  return 0;
}

extern "C" int pq_window_sumsq(const double* panel, int64_t ldp, int32_t n, const int32_t* rows,
                               const int32_t* tlen, int32_t tmax, int32_t batch, const double* mu,
                               int64_t mu_stride, double* out, int64_t out_stride, void* stream) {
  if (int e = check_win(panel, n, rows, tlen, tmax, batch)) return e;
  PQ_CHECK_ARG(out != nullptr, "pq_window_sumsq: out is null");
  if (batch == 0) return 0;
  hipLaunchKernelGGL(pq::k_window_sumsq, dim3((n + 255) / 256, batch), dim3(256), 0,
                     (hipStream_t)stream, panel, ldp, n, rows, tlen, tmax, mu, mu_stride, out, out_stride);
  PQ_CHECK_LAUNCH("pq_window_sumsq");
  return 0;
}

extern "C" int pq_window_moments_grouped(const double* panel, int64_t ldp, int32_t n, const int32_t* gdates,
                                         int32_t ngroups, const int32_t* urows, int32_t umax,
                                         const int32_t* uoff, const int32_t* tlen, double* mu,
                                         int64_t mu_stride, double* dg, int64_t dg_stride, void* stream) {
  PQ_CHECK_ARG(panel && gdates && urows && uoff && tlen && mu && dg, "pq_window_moments_grouped: null pointer");
  PQ_CHECK_ARG(n > 0 && umax > 0 && ngroups >= 0, "pq_window_moments_grouped: bad sizes n=%d umax=%d ngroups=%d",
               n, umax, ngroups);
  if (ngroups == 0) return 0;
  hipLaunchKernelGGL(pq::k_window_moments_grp, dim3((n + 255) / 256, ngroups), dim3(256), 0,
                     (hipStream_t)stream, panel, ldp, n, gdates, urows, umax, uoff, tlen, mu, mu_stride, dg,
                     dg_stride);
  PQ_CHECK_LAUNCH("pq_window_moments_grouped");
  return 0;
}

extern "C" int pq_window_geomean_grouped(const double* panel, int64_t ldp, int32_t n, const int32_t* gdates,
                                         int32_t ngroups, const int32_t* urows, int32_t umax,
                                         const int32_t* uoff, const int32_t* tlen, double* mu,
                                         int64_t mu_stride, void* stream) {
  PQ_CHECK_ARG(panel && gdates && urows && uoff && tlen && mu, "pq_window_geomean_grouped: null pointer");
  PQ_CHECK_ARG(n > 0 && umax > 0 && ngroups >= 0, "pq_window_geomean_grouped: bad sizes n=%d umax=%d ngroups=%d",
               n, umax, ngroups);
  if (ngroups == 0) return 0;
  hipLaunchKernelGGL(pq::k_window_geomean_grp, dim3((n + 255) / 256, ngroups), dim3(256), 0,
                     (hipStream_t)stream, panel, ldp, n, gdates, urows, umax, uoff, tlen, mu, mu_stride);
  PQ_CHECK_LAUNCH("pq_window_geomean_grouped");
  return 0;
}

extern "C" int pq_window_nanmean(const double* panel, int64_t ldp, int32_t n, const int32_t* rows,
                                 const int32_t* tlen, int32_t tmax, int32_t batch, double* mu, int64_t mu_stride,
                                 int32_t geometric, void* stream) {
  if (int e = check_win(panel, n, rows, tlen, tmax, batch)) return e;
  PQ_CHECK_ARG(mu != nullptr, "pq_window_nanmean: mu is null");
  if (batch == 0) return 0;
  hipLaunchKernelGGL(pq::k_window_nanmean, dim3((n + 255) / 256, batch), dim3(256), 0, (hipStream_t)stream, panel,
                     ldp, n, rows, tlen, tmax, mu, mu_stride, geometric);
  PQ_CHECK_LAUNCH("pq_window_nanmean");
  return 0;
}

extern "C" int pq_cov_pairwise_batched(const double* panel, int64_t ldp, int32_t n, const int32_t* rows,
                                       const int32_t* tlen, int32_t tmax, int32_t batch, const double* shift,
                                       int64_t shift_stride, double* out, int32_t ld, int64_t out_stride,
                                       void* stream) {
  if (int e = check_win(panel, n, rows, tlen, tmax, batch)) return e;
  PQ_CHECK_ARG(out && ld >= n && ld % 64 == 0, "pq_cov_pairwise_batched: ld must be a multiple of 64 >= n");
  if (batch == 0) return 0;
  const int nb = ld / 64;
  hipLaunchKernelGGL(pq::k_syrk_pairwise, dim3(nb * (nb + 1) / 2, batch), dim3(256), 0, (hipStream_t)stream, panel,
                     ldp, n, rows, tlen, tmax, shift, shift_stride, out, ld, out_stride);
  PQ_CHECK_LAUNCH("pq_cov_pairwise_batched");
  return 0;
}

extern "C" int pq_window_geomean(const double* panel, int64_t ldp, int32_t n, const int32_t* rows,
                                 const int32_t* tlen, int32_t tmax, int32_t batch, double* mu,
                                 int64_t mu_stride, void* stream) {
  if (int e = check_win(panel, n, rows, tlen, tmax, batch)) return e;
  PQ_CHECK_ARG(mu != nullptr, "pq_window_geomean: mu is null");
  if (batch == 0) return 0;
  hipLaunchKernelGGL(pq::k_window_mean, dim3((n + 255) / 256, batch), dim3(256), 0,
                     (hipStream_t)stream, panel, ldp, n, rows, tlen, tmax, mu, mu_stride, 1);
  PQ_CHECK_LAUNCH("pq_window_geomean");
  return 0;
}

extern "C" int pq_cov_batched(const double* panel, int64_t ldp, int32_t n, const int32_t* rows,
                              const int32_t* tlen, int32_t tmax, int32_t batch, int32_t mode,
                              const double* mu, int64_t mu_stride, double* out, int32_t ld,
                              int64_t out_stride, void* stream) {
  if (int e = check_win(panel, n, rows, tlen, tmax, batch)) return e;
  PQ_CHECK_ARG(mode == 0 || mode == 1, "pq_cov_batched: mode must be 0 (centred cov) or 1 (Gram)");
  PQ_CHECK_ARG(mode == 1 || mu != nullptr, "pq_cov_batched: mode 0 needs the window means");
  PQ_CHECK_ARG(out && ld >= n && ld % 64 == 0, "pq_cov_batched: ld must be a multiple of 64 >= n");
  if (batch == 0) return 0;
  const int nb = ld / 64;
  hipLaunchKernelGGL(pq::k_syrk, dim3(nb * (nb + 1) / 2, batch), dim3(256), 0,
                     (hipStream_t)stream, panel, ldp, n, rows, tlen, tmax, mode, mu, mu_stride,
                     out, ld, out_stride);
  PQ_CHECK_LAUNCH("pq_cov_batched");
  return 0;
}

extern "C" int pq_cov_slide_batched(const double* panel, int64_t ldp, int32_t n, const int32_t* rows,
                                    const int32_t* tlen, int32_t tmax, int32_t batch, int32_t mode,
                                    const double* mu, int64_t mu_stride, double* out, int32_t ld,
                                    int64_t out_stride, const int32_t* gstart, int32_t ngroups,
                                    const int32_t* shift, int32_t lower_only, void* stream) {
  if (int e = check_win(panel, n, rows, tlen, tmax, batch)) return e;
  PQ_CHECK_ARG(mode == 0 || mode == 1, "pq_cov_slide_batched: mode must be 0 (centred cov) or 1 (Gram)");
  PQ_CHECK_ARG(mode == 1 || mu != nullptr, "pq_cov_slide_batched: mode 0 needs the window means");
  PQ_CHECK_ARG(out && ld >= n && ld % 64 == 0, "pq_cov_slide_batched: ld must be a multiple of 64 >= n");
  PQ_CHECK_ARG(gstart && shift && ngroups >= 0, "pq_cov_slide_batched: slide plan missing");
  if (batch == 0 || ngroups == 0) return 0;
  const int nb = ld / 64;
  hipLaunchKernelGGL(pq::k_syrk_slide, dim3(nb * (nb + 1) / 2, ngroups), dim3(256), 0,
                     (hipStream_t)stream, panel, ldp, n, rows, tlen, tmax, mode, mu, mu_stride,
                     out, ld, out_stride, gstart, shift, lower_only ? 0 : 1);
  PQ_CHECK_LAUNCH("pq_cov_slide_batched");
  return 0;
}

extern "C" int pq_gram_xy_grouped(const double* panel, int64_t ldp, int32_t n, const double* bm,
                                  const int32_t* gdates, int32_t ngroups, const int32_t* urows, int32_t umax,
                                  const int32_t* uoff, const int32_t* tlen, double* xty, int64_t xty_stride,
                                  double* yty, double* dg, int64_t dg_stride, void* stream) {
  PQ_CHECK_ARG(panel && bm && gdates && urows && uoff && tlen && xty && yty, "pq_gram_xy_grouped: null pointer");
  PQ_CHECK_ARG(n > 0 && umax > 0 && ngroups >= 0, "pq_gram_xy_grouped: bad sizes n=%d umax=%d ngroups=%d", n,
               umax, ngroups);
  if (ngroups == 0) return 0;
  hipLaunchKernelGGL(pq::k_gram_xy_grp, dim3((n + 255) / 256, ngroups), dim3(256), 0, (hipStream_t)stream, panel,
                     ldp, n, bm, gdates, urows, umax, uoff, tlen, xty, xty_stride, yty, dg, dg_stride);
  PQ_CHECK_LAUNCH("pq_gram_xy_grouped");
  return 0;
}

extern "C" int pq_gram_xy_batched(const double* panel, int64_t ldp, int32_t n, const double* bm,
                                  const int32_t* rows, const int32_t* tlen, int32_t tmax,
                                  int32_t batch, double* xty, int64_t xty_stride, double* yty,
                                  void* stream) {
  if (int e = check_win(panel, n, rows, tlen, tmax, batch)) return e;
  PQ_CHECK_ARG(bm && xty && yty, "pq_gram_xy_batched: null pointer");
  if (batch == 0) return 0;
  hipLaunchKernelGGL(pq::k_gram_xy, dim3((n + 255) / 256, batch), dim3(256), 0,
                     (hipStream_t)stream, panel, ldp, n, bm, rows, tlen, tmax, xty, xty_stride, yty);
  PQ_CHECK_LAUNCH("pq_gram_xy_batched");
  return 0;
}
