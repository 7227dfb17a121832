// K4, window form: the active-set polish of polish.hip for the low-rank (backtest) path,
// with no n x n matrix anywhere.
//
// P_eff = p_scale w_scale Xc'Xc + p_diag I is only available through the date's window
// (pq_lowrank).  Each active-set round gathers the free columns of the window (T x k,
// from the L2-resident panel rows) and forms the reduced matrix P_FF = p_scale w_scale
// Xc_F'Xc_F + p_diag I with FP64 MFMA tile products (the same SYRK as K1, restricted to
// the free set) into a compact per-problem scratch of leading dimension ldk >= k:
//   - the diagonal 64x64 tiles hold P_FF in full,
//   - the strictly-upper tiles hold P_FF's lower tiles transposed,
//   - the strictly-lower tiles receive the Cholesky factor L of P_FF + delta I
//     (wg_cholesky<false>: the diagonal tiles of L are never stored; the solves use Dt),
// so one k x k buffer serves both the factorisation and the exact residuals of the
// proximal iterative refinement.  Every n-length quantity (P x_B, the final exact
// gradient) comes from two passes over the window rows (lr_px); per-variable bookkeeping
// lives in the work buffer, so n is unbounded and only the free set (k <= min(ldk, 1024))
// is bounded.  A problem whose free set outgrows ldk is left untouched with
// out[PQ_OUT_ROUNDS] = -1 so the caller can relaunch it with a larger scratch
// (final_try = 1: polish fails instead and the ADMM point is scored).
//
// Replaces, with polish.hip, the accuracy of qpsolvers' interior-point answer
// (src/qp_problems.py:211-214); scoring as in polish.hip (src/qp_problems.py:219-221,
// example/compare_solver.ipynb:212-216).
#include "polish_dev.h"
#include "capi_util.h"

namespace pq {

constexpr int KMAX = 1024;   // free variables held in LDS

// Woodbury mode: C = cdiag I + Xc diag(free) Xc' (T x T) into the lower tiles (diagonal
// tiles in full) of Ks; rows / columns >= T are the identity.  Contraction over all n
// columns (free-masked), 16 at a time through LDS, one MFMA tile product per lower tile.
__device__ void form_cwood(const pq_lowrank& lr, int b, int n, const int* fl, int nbt, double cdiag,
                           double* Ks, int64_t ldk, double* smem) {
  const int T = lr.tlen[b];
  const int32_t* rws = lr.rows + (int64_t)b * lr.tmax;
  const double* mu = lr.mu ? lr.mu + (int64_t)b * lr.mu_stride : nullptr;
  const int t = threadIdx.x;
  const int i = t >> 2, cc = (t & 3) * 4;
  double* SA = smem;
  double* SB = smem + STAGE;
  const int ntile = nbt * (nbt + 1) / 2;
  for (int tile = 0; tile < ntile; ++tile) {
    int I = (int)((sqrt(8.0 * tile + 1.0) - 1.0) * 0.5);
    while ((I + 1) * (I + 2) / 2 <= tile) ++I;
    while (I * (I + 1) / 2 > tile) --I;
    const int J = tile - I * (I + 1) / 2;
    const double* ra = I * TB + i < T ? lr.panel + (int64_t)rws[I * TB + i] * lr.ldp : nullptr;
    const double* rb = J * TB + i < T ? lr.panel + (int64_t)rws[J * TB + i] * lr.ldp : nullptr;
    Acc acc;
    acc.zero();
    for (int c0 = 0; c0 < n; c0 += KC) {
      double va[4], vb[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int c = c0 + cc + e;
        const bool m = c < n && fl[c] == 0;
        const double mc = (m && mu) ? mu[c] : 0.0;
        va[e] = (m && ra) ? ra[c] - mc : 0.0;
        vb[e] = (m && rb) ? rb[c] - mc : 0.0;
      }
      __syncthreads();
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        SA[(cc + e) * LDW + i] = va[e];
        SB[(cc + e) * LDW + i] = vb[e];
      }
      __syncthreads();
      mma_lds(acc, SA, SB, KC);
    }
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int nn = 0; nn < 2; ++nn)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int gi = I * TB + acc_row(m, r), gj = J * TB + acc_col(nn);
          Ks[(int64_t)gi * ldk + gj] = acc.c[m][nn][r] + (gi == gj ? (gi < T ? cdiag : 1.0) : 0.0);
        }
  }
  __syncthreads();
}

// The same C from the row-band Gram of the panel (pq_lr_band_gram: band[r - r0][d] =
// x_r . x_{r-d}) when every column is free: X_F X_F' is then the window's whole Gram, an
// O(T^2) gather instead of form_cwood's O(T^2 n) product (config 4: n = 3000, every
// variable free).  Centred windows: Xc Xc' = G - s 1' - 1 s' + (mu.mu) 1 1', s_t = x_t . mu.
// A few fixed columns (a later active-set round: k = n - nfix, nfix <= NFIX_MAX, listed in
// fx) are then downdated, Xc_F Xc_F' = Xc Xc' - sum_{j fixed} xc_j xc_j', from DC-column
// chunks of the window staged in LDS -- O(T^2 nfix) instead of form_cwood's O(T^2 n).
constexpr int NFIX_MAX = 128;
constexpr int DC = 8;
static_assert(KMAX + DC * KMAX <= CHOL_LDS, "form_cwood_band: sx | column chunk must fit the Cholesky LDS");
__device__ void form_cwood_band(const pq_lowrank& lr, int b, int n, int nbt, double cdiag, double* Ks,
                                int64_t ldk, const double* band, int64_t ldo, int r0, const int* fx, int nfix,
                                double* sx, double* red) {
  const int T = lr.tlen[b];
  const int32_t* rws = lr.rows + (int64_t)b * lr.tmax;
  const double* mu = lr.mu ? lr.mu + (int64_t)b * lr.mu_stride : nullptr;
  const int t = threadIdx.x, w = wave_id(), l = lane_id();
  double mm = 0.0;
  if (mu) {
    for (int i = w; i < T; i += PW) {
      const double* row = lr.panel + (int64_t)rws[i] * lr.ldp;
      double a = 0.0;
      for (int c = l; c < n; c += 64) a = fma(row[c], mu[c], a);
      a = wave_sum(a);
      if (l == 0) sx[i] = a;
    }
    double a = 0.0;
    for (int c = t; c < n; c += PT) a = fma(mu[c], mu[c], a);
    mm = block_sum(a, red);   // barrier: sx complete
  }
  const int ntile = nbt * (nbt + 1) / 2;
  for (int tile = 0; tile < ntile; ++tile) {
    int I = (int)((sqrt(8.0 * tile + 1.0) - 1.0) * 0.5);
    while ((I + 1) * (I + 2) / 2 <= tile) ++I;
    while (I * (I + 1) / 2 > tile) --I;
    const int J = tile - I * (I + 1) / 2;
    for (int e = t; e < TB * TB; e += PT) {
      const int gi = I * TB + (e >> 6), gj = J * TB + (e & 63);
      double v;
      if (gi < T && gj < T) {
        const int ri = rws[gi], rj = rws[gj];
        const int hi = ri > rj ? ri : rj;
        v = band[(int64_t)(hi - r0) * ldo + (ri > rj ? ri - rj : rj - ri)];
        if (mu) v += mm - sx[gi] - sx[gj];
        if (gi == gj) v += cdiag;
      } else {
        v = gi == gj ? 1.0 : 0.0;
      }
      Ks[(int64_t)gi * ldk + gj] = v;
    }
  }
  double* cs = sx + KMAX;   // T x DC: centred window columns of a chunk of fixed variables
  for (int j0 = 0; j0 < nfix; j0 += DC) {
    const int nc = min(DC, nfix - j0);
    __syncthreads();
    for (int e = t; e < T * DC; e += PT) {
      const int i = e / DC, c = e - i * DC;
      double v = 0.0;
      if (c < nc) {
        const int j = fx[j0 + c];
        v = lr.panel[(int64_t)rws[i] * lr.ldp + j] - (mu ? mu[j] : 0.0);
      }
      cs[e] = v;
    }
    __syncthreads();
    for (int tile = 0; tile < ntile; ++tile) {   // same tile / element map as above
      int I = (int)((sqrt(8.0 * tile + 1.0) - 1.0) * 0.5);
      while ((I + 1) * (I + 2) / 2 <= tile) ++I;
      while (I * (I + 1) / 2 > tile) --I;
      const int J = tile - I * (I + 1) / 2;
      for (int e = t; e < TB * TB; e += PT) {
        const int gi = I * TB + (e >> 6), gj = J * TB + (e & 63);
        if (gi >= T || gj >= T) continue;
        const double* a = cs + gi * DC;
        const double* c = cs + gj * DC;
        double d = 0.0;
#pragma unroll
        for (int q = 0; q < DC; ++q) d = fma(a[q], c[q], d);
        Ks[(int64_t)gi * ldk + gj] -= d;
      }
    }
  }
  __syncthreads();
}

struct FormRead {   // the lower tiles (diagonal tiles in full) as written
  const double* K;
  int64_t ld;
  __device__ __forceinline__ double operator()(int gi, int gj) const { return K[(int64_t)gi * ld + gj]; }
};

// P_FF for k <= 128 (one or two column blocks): each 32-row chunk of the window is
// gathered ONCE for all (NB (NB + 1) / 2) tiles into one LDS image of pitch NB*64 + 16,
// double-buffered so the next chunk's gathers (2 rows x 4 NB columns per thread, all in
// flight together) overlap the MFMAs: 8 dependent gather round trips for T = 252.
template <int NB>
PQ_DEVFN void form_pff_small(const pq_lowrank& lr, int b, const int* Fl, int k, double psw, double pd,
                               double* Ks, int64_t ldk, double* smem) {
  constexpr int PIT = NB * TB + 16;
  constexpr int NT = NB * (NB + 1) / 2;
  constexpr int KCH = 32;             // window rows per chunk (2 x 32 x PIT <= CHOL_LDS)
  constexpr int RS = KCH / 16;        // rows per thread and chunk
  static_assert(2 * KCH * PIT <= CHOL_LDS, "form_pff_small: stage buffers exceed the LDS region");
  const int T = lr.tlen[b];
  const int32_t* rws = lr.rows + (int64_t)b * lr.tmax;
  const double* mu = lr.mu ? lr.mu + (int64_t)b * lr.mu_stride : nullptr;
  const int t = threadIdx.x, kr = t >> 4, c4 = (t & 15) * 4;
  int col[NB][4];
  double mc[NB][4];
#pragma unroll
  for (int h = 0; h < NB; ++h)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int p = h * TB + c4 + e;
      col[h][e] = p < k ? Fl[p] : -1;
      mc[h][e] = (col[h][e] >= 0 && mu) ? mu[col[h][e]] : 0.0;
    }
  double v[RS][NB][4];
  auto gather = [&](int t0) {
#pragma unroll
    for (int s = 0; s < RS; ++s) {
      const int tt = t0 + kr + 16 * s;
      const double* row = tt < T ? lr.panel + (int64_t)rws[tt] * lr.ldp : nullptr;
#pragma unroll
      for (int h = 0; h < NB; ++h)
#pragma unroll
        for (int e = 0; e < 4; ++e) v[s][h][e] = (row && col[h][e] >= 0) ? row[col[h][e]] - mc[h][e] : 0.0;
    }
  };
  auto put = [&](double* S) {
#pragma unroll
    for (int s = 0; s < RS; ++s)
#pragma unroll
      for (int h = 0; h < NB; ++h)
#pragma unroll
        for (int e = 0; e < 4; ++e) S[(kr + 16 * s) * PIT + h * TB + c4 + e] = v[s][h][e];
  };
  // acc[tile] for tiles (0,0), (1,0), (1,1); mma over an image of pitch PIT
  Acc acc[NT];
#pragma unroll
  for (int q = 0; q < NT; ++q) acc[q].zero();
  const int l = lane_id(), w = wave_id();
  const int i0 = (w >> 1) * 32 + (l & 15), j0 = (w & 1) * 32 + (l & 15), krd = l >> 4;
  auto mma = [&](const double* S) {
#pragma unroll
    for (int kk = 0; kk < KCH; kk += 4) {
      const double* r = S + (kk + krd) * PIT;
      double a[NB][2];
#pragma unroll
      for (int h = 0; h < NB; ++h) {
        a[h][0] = r[h * TB + i0];
        a[h][1] = r[h * TB + i0 + 16];
      }
      double bj[NB][2];
#pragma unroll
      for (int h = 0; h < NB; ++h) {
        bj[h][0] = r[h * TB + j0];
        bj[h][1] = r[h * TB + j0 + 16];
      }
      int q = 0;
#pragma unroll
      for (int I = 0; I < NB; ++I)
#pragma unroll
        for (int J = 0; J <= I; ++J, ++q)
#pragma unroll
          for (int m = 0; m < 2; ++m)
#pragma unroll
            for (int nn = 0; nn < 2; ++nn)
              acc[q].c[m][nn] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[I][m], bj[J][nn], acc[q].c[m][nn], 0, 0, 0);
    }
  };
  double* S0 = smem;
  double* S1 = smem + KCH * PIT;
  gather(0);
  __syncthreads();   // the stage buffers' previous users are done
  put(S0);
  __syncthreads();
  int buf = 0;
  for (int t0 = 0; t0 < T; t0 += KCH) {
    const bool more = t0 + KCH < T;
    if (more) gather(t0 + KCH);
    mma(buf ? S1 : S0);
    if (more) put(buf ? S0 : S1);
    __syncthreads();
    buf ^= 1;
  }
  int q = 0;
#pragma unroll
  for (int I = 0; I < NB; ++I)
#pragma unroll
    for (int J = 0; J <= I; ++J, ++q)
#pragma unroll
      for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int nn = 0; nn < 2; ++nn)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int gi = I * TB + acc_row(m, r), gj = J * TB + acc_col(nn);
            const double vv = psw * acc[q].c[m][nn][r] + (gi == gj ? pd : 0.0);
            if (I == J) Ks[(int64_t)gi * ldk + gj] = vv;
            else Ks[(int64_t)gj * ldk + gi] = vv;
          }
  __syncthreads();
}

__global__ __launch_bounds__(PT) void k_polish_w(pq_lowrank lr, pq_problem pb, pq_state st,
                                                 const int32_t* idx, int nidx, pq_settings s, int ldk,
                                                 int final_try, const double* band, int64_t ldo, int r0) {
  __shared__ __attribute__((aligned(16))) double smem[CHOL_LDS + 2 * KMAX + 15 * 64 + KMAX / 2 + 256];
  double* stg = smem;                  // Cholesky / SYRK stream buffers; S factor; lr_px tree
  double* vec = smem + 4 * STAGE;      // 3 KMAX vectors during refinement; lr_px u
  double* solx = smem + CHOL_LDS;      // compact solution x_F
  double* rF = solx + KMAX;            // compact rhs of the F rows
  double* solL = rF + KMAX;            // 64: multipliers of the active rows
  double* dA = solL + 64;              // 64: rhs of the active rows
  double* rl = dA + 64;                // 64
  double* wl = rl + 64;                // 64
  double* t64 = wl + 64;               // 64
  double* part = t64 + 64;             // 4*64 (also reduction scratch)
  double* red = part + 4 * 64;         // 64
  double* lamF = red + 64;             // 64: multipliers of all general rows (by row)
  double* y64p = lamF + 64;            // 4*64 partial sums of the diagonal-block products
  int* Fl = reinterpret_cast<int*>(y64p + 4 * 64);   // KMAX: free-variable list
  int* act = Fl + KMAX;                               // 64
  int* Al = act + 64;                                 // 64
  int* cnt = Al + 64;                                 // PT + 8

  const int slot = xcd_slot(blockIdx.x, gridDim.x);   // neighbouring dates share an XCD L2
  const int b = idx ? idx[slot] : slot;
  const int st0 = st.status[b];
  if (st0 != PQ_SOLVED && st0 != PQ_MAX_ITER) return;
  const int n = pb.n, ld = pb.ld, mg = pb.mg;
  const int t = threadIdx.x, w = wave_id(), l = lane_id();
  const double ps = pb.p_scale ? pb.p_scale[b] : 1.0;
  const double pd = pb.p_diag ? pb.p_diag[b] : 0.0;
  const double wsc = lr.w_scale ? lr.w_scale[b] : 1.0;
  const double psw = ps * wsc;
  const double* q = pb.q + (int64_t)b * pb.q_stride;
  const double* Cg = pb.Cg ? pb.Cg + (int64_t)b * pb.Cg_stride : nullptr;
  const double* lg = pb.lg ? pb.lg + (int64_t)b * pb.g_stride : nullptr;
  const double* ug = pb.ug ? pb.ug + (int64_t)b * pb.g_stride : nullptr;
  const bool has_box = pb.lb != nullptr;
  const double* lb = has_box ? pb.lb + (int64_t)b * pb.box_stride : nullptr;
  const double* ub = has_box ? pb.ub + (int64_t)b * pb.box_stride : nullptr;
  // compact scratch: one slot per launched workgroup (a relaunch passes a smaller buffer)
  double* K = st.K + (int64_t)blockIdx.x * st.K_stride;
  double* Dt = st.Dt + (int64_t)blockIdx.x * st.Dt_stride;
  double* sx = st.x + (int64_t)b * ld;
  double* sz = st.z + (int64_t)b * st.m_ld;
  double* sy = st.y + (int64_t)b * st.m_ld;
  // work layout (doubles): xs | xb | g | Px | wr wx wt wd (Woodbury mode) | U (mg_pad rows:
  // ldk-strided L^-1 C_aF' in compact mode, n-length A^-1 C_aF' in Woodbury mode) | fl (ld ints)
  double* W = st.work + (int64_t)b * st.work_stride;
  double* xs = W;
  double* xb = xs + ld;
  double* g = xb + ld;
  double* Px = g + ld;
  double* U = W + 8 * (int64_t)ld;
  int* fl = reinterpret_cast<int*>(U + (int64_t)st.mg_pad * ld);   // 0 free, 1 at lower, 2 at upper
#ifdef PQ_PROFILE
  double* prof = W + PQ_WORK_PROF(ld, st.mg_pad);
  if (t < 16) prof[t] = 0.0;
  long long t_last_ = wall_clock64();
#endif

  // ---- problem scale -> tolerances (diag P from the window's sums of squares) ----------
  const double* dgb = lr.dg + (int64_t)b * lr.dg_stride;
  double sc = 0.0;
  for (int i = t; i < n; i += PT) sc = fmax(sc, fmax(fabs(q[i]), fabs(psw * dgb[i] + pd)));
  sc = block_max(sc, red);
  sc = fmax(sc, 1e-300);
  const double dtol = s.dual_tol * sc;
  const double delta = s.delta * sc;
  const double ptol = 1e-12;

  // ---- classification from the ADMM point -------------------------------------------
  for (int i = t; i < ld; i += PT) {
    int f = 0;
    if (i < n && has_box) {
      const double zi = sz[st.mg_pad + i], yi = sy[st.mg_pad + i];
      if (!isinf(lb[i]) && zi - lb[i] < -yi) f = 1;
      else if (!isinf(ub[i]) && ub[i] - zi < yi) f = 2;
      if (lb[i] == ub[i]) f = 1;
    }
    fl[i] = (i < n) ? f : 1;  // padding never free
    xs[i] = (i < n) ? sx[i] : 0.0;
  }
  if (t < mg) {
    const double zr = sz[t], yr = sy[t];
    int a = 0;
    if (lg[t] == ug[t]) a = 2;
    else if (!isinf(lg[t]) && zr - lg[t] < -yr) a = 1;
    else if (!isinf(ug[t]) && ug[t] - zr < yr) a = 2;
    act[t] = a;
    lamF[t] = yr;   // multipliers start at the ADMM duals
  }
  __syncthreads();
  PQ_STAMP(0);

  // exact P x and gradient g = P x + q + Cg' lam of the point in xs
  auto emit_g = [&](int i, double sum) {
    const double pxi = ps * sum + pd * xs[i];
    double gi = pxi + q[i];
    for (int r = 0; r < mg; ++r) gi += Cg[(int64_t)r * ld + i] * lamF[r];
    Px[i] = pxi;
    g[i] = gi;
  };
  auto full_px = [&]() { lr_px(lr, b, n, xs, vec, stg, red, emit_g); };

  // At least two proximal refinement steps per round in Woodbury mode: one step from the
  // ADMM point left config 4's budget row outside the 1e-10 equality check on every date,
  // and the second active-set round that followed (new capacitance, Cholesky, Z) cost 1.5x
  // the extra step (polish 33 -> 22 ms per 2000 dates).  A converged step breaks early.
  // Compact mode takes s.refine_iters steps as given: the caller chooses them (the grouped
  // polish's own dates take 1; the dates it hands to this kernel are relaunched with at least
  // 2, engine.solve_lowrank polish_grouped, so those may take more steps than grouped dates).
  const int refine_steps = max(s.refine_iters, 2);
  // Woodbury mode (free set beyond the compact scratch) needs the T x T capacitance to fit
  const bool wood_ok = ((lr.tmax + TB - 1) / TB) * TB <= ldk && lr.tmax <= KMAX;
  int accepted = 0, rounds = 0, nfree = 0, overflow = 0;
  for (int round = 0; round < s.polish_rounds && !accepted; ++round) {
    rounds = round + 1;
    // ---- free list (stable compaction) ------------------------------------------------
    const int chunk = (n + PT - 1) / PT;
    int c0 = 0;
    for (int i = t * chunk; i < min(n, (t + 1) * chunk); ++i) c0 += (fl[i] == 0);
    cnt[t] = c0;
    __syncthreads();
    if (t == 0) {
      int acc = 0;
      for (int u = 0; u < PT; ++u) { const int v = cnt[u]; cnt[u] = acc; acc += v; }
      cnt[PT] = acc;
      int a = 0;
      for (int r = 0; r < mg; ++r) if (act[r]) Al[a++] = r;
      cnt[PT + 1] = a;
    }
    __syncthreads();
    const int k = cnt[PT];
    const int ma = cnt[PT + 1];
    nfree = k;
    const bool compact = k <= ldk && k <= KMAX;   // uniform (k from LDS)
    if (!compact && !wood_ok) {   // neither the compact nor the Woodbury scratch fits
      overflow = 1;
      break;
    }
    if (compact) {
      int p = cnt[t];
      for (int i = t * chunk; i < min(n, (t + 1) * chunk); ++i)
        if (fl[i] == 0) Fl[p++] = i;
    }
    const int nbk = (k + TB - 1) / TB;
    int px_ready = 0;   // g holds w Xc'Xc xs (uniform)
    int nzb = 0;
    for (int i = t; i < ld; i += PT) {
      const double v = i < n ? (fl[i] == 1 ? lb[i] : (fl[i] == 2 ? ub[i] : 0.0)) : 0.0;
      xb[i] = v;
      nzb |= (v != 0.0);
    }
    nzb = block_or(nzb, red);
    PQ_STAMP(1);
    __builtin_amdgcn_s_dcache_inv();
    if (!compact) {
      // ---- Woodbury mode: A = P_FF + delta I = psw Xc_F'Xc_F + dl I on F, applied as
      //      A^-1 v = (v - Xc_F' C^-1 Xc_F v) / dl with C = (dl / psw) I + Xc_F Xc_F' (T x T);
      //      every vector is n-length in the work buffer (zero outside F) ------------------
      const int T = lr.tlen[b];
      const int nbt = (T + TB - 1) / TB;
      const double dl = pd + delta;
      double* wr = W + 4 * (int64_t)ld;    // rF on F
      double* wx = wr + ld;                // x_F
      double* wt = wx + ld;                // A^-1 rx
      double* wd = wt + ld;                // rx (also the C_aF' staging)
      double* u = vec;                     // T (+ padding): Xc v
      double* y1 = vec + KMAX;
      double* y2 = vec + 2 * KMAX;
      double* tree = solx;                 // solx | rF (2 KMAX doubles) are unused in this mode
      if (nzb) {
        lr_px(lr, b, n, xb, u, tree, red, [&](int i, double sum) { g[i] = sum; });
        __syncthreads();
      }
      for (int i = t; i < ld; i += PT) {
        const bool f = i < n && fl[i] == 0;
        wr[i] = f ? -q[i] - (nzb ? ps * g[i] : 0.0) : 0.0;
        wx[i] = f ? xs[i] : 0.0;
        wt[i] = 0.0;
        wd[i] = 0.0;
      }
      for (int a = w; a < ma; a += PW) {
        const int r = Al[a];
        const double* c = Cg + (int64_t)r * ld;
        double sum = 0.0;
        for (int j = l; j < n; j += 64) sum += c[j] * xb[j];
        sum = wave_sum(sum);
        if (l == 0) dA[a] = (act[r] == 1 ? lg[r] : ug[r]) - sum;
      }
      if (t < ma) solL[t] = lamF[Al[t]];
      __syncthreads();
      PQ_STAMP(2);
      const int nfix = n - k;
      if (band && nfix <= NFIX_MAX) {
        if (nfix > 0 && w == 0) {   // fixed-column list in Fl (unused in this mode), ascending
          int base = 0;
          for (int i0 = 0; i0 < n; i0 += 64) {
            const int i = i0 + l;
            const bool fx = i < n && fl[i] != 0;
            const unsigned long long m = __ballot(fx);
            if (fx) Fl[base + __popcll(m & ((1ull << l) - 1ull))] = i;
            base += __popcll(m);
          }
        }
        __syncthreads();
        form_cwood_band(lr, b, n, nbt, dl / psw, K, ldk, band, ldo, r0, Fl, nfix, smem, red);
      } else {
        form_cwood(lr, b, n, fl, nbt, dl / psw, K, ldk, smem);
      }
      const int info = wg_cholesky(FormRead{K, ldk}, K, ldk, nbt, T, Dt, smem);
      if (info) break;
      PQ_STAMP(3);
      auto apply = [&](const double* v, double* out) {   // out = A^-1 v on F, 0 elsewhere
        lr_pass1(lr, b, n, v, u, red);
        for (int p = T + t; p < nbt * TB; p += PT) u[p] = 0.0;
        __syncthreads();
        fwd_solve(K, ldk, Dt, nbt, u, y1, t64, y64p);
        bwd_solve(K, ldk, Dt, nbt, y1, y2, t64, part, y64p);
        lr_pass2(lr, b, n, y2, tree, red,
                 [&](int i, double sv) { out[i] = fl[i] == 0 ? (v[i] - sv) / dl : 0.0; });
        for (int i = n + t; i < ld; i += PT) out[i] = 0.0;
        __syncthreads();
      };
      // Z_a = A^-1 C_aF' (rows of U), S = C_aF Z + delta I (lower, in stg)
      for (int a = 0; a < ma; ++a) {
        const double* c = Cg + (int64_t)Al[a] * ld;
        for (int i = t; i < n; i += PT) wd[i] = fl[i] == 0 ? c[i] : 0.0;
        __syncthreads();
        apply(wd, U + (int64_t)a * ld);
      }
      __builtin_amdgcn_s_dcache_inv();
      for (int e = w; e < ma * ma; e += PW) {
        const int i = e / ma, j = e % ma;
        if (j > i) continue;
        const double* c = Cg + (int64_t)Al[i] * ld;
        const double* z = U + (int64_t)j * ld;
        double sum = 0.0;
        for (int x = l; x < n; x += 64) sum += c[x] * z[x];
        sum = wave_sum(sum);
        if (l == 0) stg[i * DP + j] = sum + (i == j ? delta : 0.0);
      }
      __syncthreads();
      if (tile_potrf_lds(stg, ma)) break;
      PQ_STAMP(4);
      for (int itr = 0; itr < refine_steps; ++itr) {
        // wd = rF - P_FF x_F - C_aF' solL on F ;  rl = dA - C_aF x_F ;  g = w Xc'Xc x_F
        // (kept: a converged x_F with x_B = 0 is the final point, whose exact P x this is)
        lr_px(lr, b, n, wx, u, tree, red, [&](int i, double sum) {
          g[i] = sum;
          double v = 0.0;
          if (fl[i] == 0) {
            v = wr[i] - ps * sum - pd * wx[i];
            for (int a = 0; a < ma; ++a) v -= Cg[(int64_t)Al[a] * ld + i] * solL[a];
          }
          wd[i] = v;
        });
        for (int a = w; a < ma; a += PW) {
          const double* c = Cg + (int64_t)Al[a] * ld;
          double sum = 0.0;
          for (int x = l; x < n; x += 64) sum += c[x] * wx[x];
          sum = wave_sum(sum);
          if (l == 0) {
            const double v = dA[a] - sum;
            rl[a] = fabs(v) <= 1e-14 * (1.0 + fabs(dA[a]) + fabs(sum)) ? 0.0 : v;
          }
        }
        __syncthreads();
        {
          double rm = 0.0;
          for (int i = t; i < n; i += PT) rm = fmax(rm, fabs(wd[i]));
          if (t < ma) rm = fmax(rm, fabs(rl[t]));
          if (block_max(rm, red) <= 1e-13 * sc) {
            px_ready = !nzb;
            break;
          }
        }
        apply(wd, wt);
        for (int a = w; a < ma; a += PW) {   // wl = C_aF t1 - rl
          const double* c = Cg + (int64_t)Al[a] * ld;
          double sum = 0.0;
          for (int x = l; x < n; x += 64) sum += c[x] * wt[x];
          sum = wave_sum(sum);
          if (l == 0) wl[a] = sum - rl[a];
        }
        __syncthreads();
        if (t == 0) {
          for (int i = 0; i < ma; ++i) {
            double v = wl[i];
            for (int j = 0; j < i; ++j) v -= stg[i * DP + j] * wl[j];
            wl[i] = v / stg[i * DP + i];
          }
          for (int i = ma - 1; i >= 0; --i) {
            double v = wl[i];
            for (int j = i + 1; j < ma; ++j) v -= stg[j * DP + i] * wl[j];
            wl[i] = v / stg[i * DP + i];
          }
        }
        __syncthreads();
        for (int i = t; i < n; i += PT) {
          if (fl[i] == 0) {
            double v = wt[i];
            for (int a = 0; a < ma; ++a) v -= U[(int64_t)a * ld + i] * wl[a];
            wx[i] += v;
          }
        }
        if (t < ma) solL[t] += wl[t];
        __syncthreads();
      }
      PQ_STAMP(5);
      for (int i = t; i < n; i += PT) xs[i] = fl[i] == 0 ? wx[i] : xb[i];
      if (t < 64) lamF[t] = 0.0;
      __syncthreads();
      if (t < ma) lamF[Al[t]] = solL[t];
      __syncthreads();
    } else {
      // ---- reduced rhs: rF = -q_F - P_FB x_B ;  d_a = rhs_a - C_aB x_B --------------------
      if (nzb) {   // P x_B through the window (pd I does not couple F and B)
        lr_px(lr, b, n, xb, vec, stg, red, [&](int i, double sum) { g[i] = sum; });
        __syncthreads();
        for (int p = t; p < k; p += PT) rF[p] = -q[Fl[p]] - ps * g[Fl[p]];
      } else {     // (long-only: every fixed weight is 0 and P_FB x_B vanishes)
        for (int p = t; p < k; p += PT) rF[p] = -q[Fl[p]];
      }
      for (int a = w; a < ma; a += PW) {
        const int r = Al[a];
        const double* c = Cg + (int64_t)r * ld;
        double sum = 0.0;
        for (int j = l; j < n; j += 64) sum += c[j] * xb[j];
        sum = wave_sum(sum);
        if (l == 0) dA[a] = (act[r] == 1 ? lg[r] : ug[r]) - sum;
      }
      for (int p = k + t; p < nbk * TB; p += PT) rF[p] = 0.0;
      for (int p = t; p < k; p += PT) solx[p] = xs[Fl[p]];
      if (t < ma) solL[t] = lamF[Al[t]];
      __syncthreads();
      PQ_STAMP(2);
      // ---- P_FF from the window, then factor P_FF + delta I --------------------------------
      int info = 0;
      if (k > 0) {
        if (nbk == 1) form_pff_small<1>(lr, b, Fl, k, psw, pd, K, ldk, smem);
        else if (nbk == 2) form_pff_small<2>(lr, b, Fl, k, psw, pd, K, ldk, smem);
        else form_pff(lr, b, Fl, k, nbk, psw, pd, K, ldk, smem);
        PQ_STAMP(9);
        info = wg_cholesky<false>(FormW{K, ldk, k, delta}, K, ldk, nbk, k, Dt, smem);
      }
      if (info) break;
      PQ_STAMP(3);
      double* t1 = vec;                 // KMAX each, inside the sD region
      double* dx = vec + KMAX;
      double* rx = vec + 2 * KMAX;
      // ---- U = L^-1 C_aF' (columns a), S = U'U + delta I, factor S in stg ---------------
      for (int a = 0; a < ma; ++a) {
        const int r = Al[a];
        for (int p = t; p < nbk * TB; p += PT) rx[p] = p < k ? Cg[(int64_t)r * ld + Fl[p]] : 0.0;
        __syncthreads();
        fwd_solve(K, ldk, Dt, nbk, rx, t1, t64, y64p);
        for (int p = t; p < nbk * TB; p += PT) U[(int64_t)a * ldk + p] = t1[p];
        __syncthreads();
      }
      __builtin_amdgcn_s_dcache_inv();   // U is re-read below, partly at uniform addresses
      for (int e = t; e < TB * TB; e += PT) {
        const int i = e >> 6, j = e & 63;
        double v = (i == j) ? 1.0 : 0.0;
        if (i < ma && j < ma) {
          v = (i == j) ? delta : 0.0;
          if (j <= i) for (int p = 0; p < k; ++p) v += U[(int64_t)i * ldk + p] * U[(int64_t)j * ldk + p];
        }
        stg[i * DP + j] = v;
      }
      __syncthreads();
      if (tile_potrf_lds(stg, ma)) break;
      PQ_STAMP(4);
      // ---- proximal iterative refinement -------------------------------------------------
      for (int itr = 0; itr < s.refine_iters; ++itr) {
        // rx = rF - P_FF solx - C_aF' solL ;  rl = dA - C_aF solx
        for (int p = w; p < k; p += PW) {
          double sum = 0.0;
          for (int qq = l; qq < k; qq += 64) sum += pc_at(K, ldk, p, qq) * solx[qq];
          sum = wave_sum(sum);
          if (l == 0) {
            double v = rF[p] - sum;
            for (int a = 0; a < ma; ++a) v -= Cg[(int64_t)Al[a] * ld + Fl[p]] * solL[a];
            rx[p] = v;
          }
        }
        for (int p = k + t; p < nbk * TB; p += PT) rx[p] = 0.0;
        for (int a = w; a < ma; a += PW) {
          const double* c = Cg + (int64_t)Al[a] * ld;
          double sum = 0.0;
          for (int p = l; p < k; p += 64) sum += c[Fl[p]] * solx[p];
          sum = wave_sum(sum);
          if (l == 0) {
            const double v = dA[a] - sum;
            // rounding-level residuals of a row with no free support must not move lam
            rl[a] = fabs(v) <= 1e-14 * (1.0 + fabs(dA[a]) + fabs(sum)) ? 0.0 : v;
          }
        }
        __syncthreads();
        {  // converged to rounding level: further refinement steps change nothing
          double rm = 0.0;
          for (int p = t; p < k; p += PT) rm = fmax(rm, fabs(rx[p]));
          if (t < ma) rm = fmax(rm, fabs(rl[t]));
          if (block_max(rm, red) <= 1e-13 * sc) break;
        }
        fwd_solve(K, ldk, Dt, nbk, rx, t1, t64, y64p);
        // wl = U' t1 - rl ; dlam = S^-1 wl (S = Ls Ls', tiny, one thread)
        for (int a = w; a < ma; a += PW) {
          double sum = 0.0;
          for (int p = l; p < k; p += 64) sum += U[(int64_t)a * ldk + p] * t1[p];
          sum = wave_sum(sum);
          if (l == 0) wl[a] = sum - rl[a];
        }
        __syncthreads();
        if (t == 0) {
          for (int i = 0; i < ma; ++i) {            // forward Ls
            double v = wl[i];
            for (int j = 0; j < i; ++j) v -= stg[i * DP + j] * wl[j];
            wl[i] = v / stg[i * DP + i];
          }
          for (int i = ma - 1; i >= 0; --i) {       // backward Ls'
            double v = wl[i];
            for (int j = i + 1; j < ma; ++j) v -= stg[j * DP + i] * wl[j];
            wl[i] = v / stg[i * DP + i];
          }
        }
        __syncthreads();
        // t1 <- t1 - U dlam ; dx = L^-T t1
        for (int p = t; p < nbk * TB; p += PT) {
          double v = t1[p];
          for (int a = 0; a < ma; ++a) v -= U[(int64_t)a * ldk + p] * wl[a];
          t1[p] = v;
        }
        __syncthreads();
        bwd_solve(K, ldk, Dt, nbk, t1, dx, t64, part, y64p);
        for (int p = t; p < k; p += PT) solx[p] += dx[p];
        if (t < ma) solL[t] += wl[t];
        __syncthreads();
      }
      PQ_STAMP(5);
      // ---- expand, exact gradient, checks -------------------------------------------------
      for (int i = t; i < n; i += PT) xs[i] = xb[i];
      __syncthreads();
      for (int p = t; p < k; p += PT) xs[Fl[p]] = solx[p];
      if (t < 64) lamF[t] = 0.0;
      __syncthreads();
      if (t < ma) lamF[Al[t]] = solL[t];  // full-length general multipliers
      __syncthreads();
    }
    __builtin_amdgcn_s_dcache_inv();   // xs was rewritten: no stale scalar-cache reads
    PQ_STAMP(6);
    if (px_ready) {          // Woodbury mode: the converged refinement's last pass
      for (int i = t; i < n; i += PT) emit_g(i, g[i]);
    } else if (compact && !nzb) {   // x = x_F exactly: pass 1 gathers the k free columns only
      lr_pass1_sparse(lr, b, Fl, k, solx, vec, red);
      lr_pass2(lr, b, n, vec, stg, red, [&](int i, double v) { emit_g(i, wsc * v); });
    } else {
      full_px();
    }
    __syncthreads();
    PQ_STAMP(10);
    int bad = 0;
    for (int i = t; i < n; i += PT) {
      const int f = fl[i];
      const double xi = xs[i];
      if (f == 0 && has_box) {
        if (!isinf(lb[i]) && xi < lb[i] - ptol * (1.0 + fabs(lb[i]))) { fl[i] = 1; bad = 1; }
        else if (!isinf(ub[i]) && xi > ub[i] + ptol * (1.0 + fabs(ub[i]))) { fl[i] = 2; bad = 1; }
      } else if (f == 1 && lb[i] != ub[i] && -g[i] > dtol) { fl[i] = 0; bad = 1; }
      else if (f == 2 && -g[i] < -dtol) { fl[i] = 0; bad = 1; }
    }
    for (int r = w; r < mg; r += PW) {
      const double* c = Cg + (int64_t)r * ld;
      double sum = 0.0;
      for (int j = l; j < n; j += 64) sum += c[j] * xs[j];
      sum = wave_sum(sum);
      if (l == 0 && lg[r] != ug[r]) {
        const int a = act[r];
        const double lam = lamF[r];
        if (a == 0 && sum > ug[r] + ptol * (1.0 + fabs(ug[r]))) { act[r] = 2; bad = 1; }
        else if (a == 0 && sum < lg[r] - ptol * (1.0 + fabs(lg[r]))) { act[r] = 1; bad = 1; }
        else if (a == 2 && lam < -dtol) { act[r] = 0; bad = 1; }
        else if (a == 1 && lam > dtol) { act[r] = 0; bad = 1; }
      } else if (l == 0 && fabs(sum - ug[r]) > 1e-10 * (1.0 + fabs(ug[r]))) {
        bad = 1;   // an equality row the reduced system could not satisfy (no free support)
      }
    }
    bad = block_or(bad, red);
    if (!bad) accepted = 1;
    __syncthreads();
    PQ_STAMP(7);
  }
  __syncthreads();
  if (overflow && !final_try) {   // leave the problem for a relaunch with a larger ldk
    if (t == 0) {
      double* o = st.out + (int64_t)b * PQ_OUT_FIELDS;
      o[PQ_OUT_NFREE] = (double)nfree;
      o[PQ_OUT_ROUNDS] = -1.0;
    }
    return;
  }
  // ---- final point: polished or ADMM --------------------------------------------------
  if (!accepted) {
    for (int i = t; i < n; i += PT) xs[i] = sx[i];
    if (t < 64) lamF[t] = (t < mg) ? sy[t] : 0.0;
    __syncthreads();
    __builtin_amdgcn_s_dcache_inv();
    full_px();
    __syncthreads();
  }
  // z_box: polished -> -g on fixed, 0 on free; ADMM -> ADMM box duals
  double xpx = 0.0, qx = 0.0, pres = 0.0, dres = 0.0, gapb = 0.0;
  for (int i = t; i < n; i += PT) {
    const double xi = xs[i];
    double zb = 0.0;
    if (has_box) zb = accepted ? (fl[i] ? -g[i] : 0.0) : sy[st.mg_pad + i];
    xpx += xi * Px[i];
    qx += q[i] * xi;
    dres = fmax(dres, fabs(g[i] + zb));
    if (has_box) {
      if (!isinf(lb[i])) { pres = fmax(pres, lb[i] - xi); gapb += lb[i] * fmin(zb, 0.0); }
      if (!isinf(ub[i])) { pres = fmax(pres, xi - ub[i]); gapb += ub[i] * fmax(zb, 0.0); }
      sy[st.mg_pad + i] = zb;
    }
    sx[i] = xi;
  }
  for (int r = w; r < mg; r += PW) {
    const double* c = Cg + (int64_t)r * ld;
    double sum = 0.0;
    for (int j = l; j < n; j += 64) sum += c[j] * xs[j];
    sum = wave_sum(sum);
    if (l == 0) {
      const double lam = lamF[r];
      double v;
      if (lg[r] == ug[r]) v = fabs(sum - ug[r]);
      else v = fmax(isinf(ug[r]) ? 0.0 : sum - ug[r], isinf(lg[r]) ? 0.0 : lg[r] - sum);
      part[r] = v;
      part[64 + r] = (lam > 0.0 ? ug[r] : (isinf(lg[r]) ? 0.0 : lg[r])) * lam;
      sy[r] = lam;
      sz[r] = sum;
    }
  }
  __syncthreads();
  if (t < mg) { pres = fmax(pres, part[t]); gapb += part[64 + t]; }
  xpx = block_sum(xpx, red);
  qx = block_sum(qx, red);
  gapb = block_sum(gapb, red);
  pres = block_max(pres, red);
  dres = block_max(dres, red);
  if (t == 0) {
    double* o = st.out + (int64_t)b * PQ_OUT_FIELDS;
    o[PQ_OUT_OBJ] = 0.5 * xpx + qx;
    o[PQ_OUT_PRIM] = fmax(pres, 0.0);
    o[PQ_OUT_DUAL] = dres;
    o[PQ_OUT_GAP] = fabs(xpx + qx + gapb);
    o[PQ_OUT_RHO] = st.rho[b];
    o[PQ_OUT_NFREE] = (double)nfree;
    o[PQ_OUT_ROUNDS] = (double)rounds;
    if (st0 == PQ_SOLVED) st.status[b] = accepted ? PQ_SOLVED : PQ_SOLVED_INACCURATE;
    else st.status[b] = accepted ? PQ_SOLVED : PQ_MAX_ITER;
  }
  PQ_STAMP(8);
}

}  // namespace pq

extern "C" int pq_polish_w_batched(const pq_lowrank* lr, const pq_problem* pb, pq_state* st,
                                   const int32_t* idx, int32_t nidx, const pq_settings* s, int32_t ldk,
                                   int32_t final_try, const double* band, int64_t ldo, int32_t r0, void* stream) {
  PQ_CHECK_ARG(lr && pb && st && s, "pq_polish_w_batched: null argument");
  PQ_CHECK_ARG(lr->panel && lr->rows && lr->tlen && lr->tmax > 0 && lr->dg,
               "pq_polish_w_batched: window (with its diagonal dg) missing");
  PQ_CHECK_ARG((lr->ldp & 1) == 0, "pq_polish_w_batched: the window form needs an even panel stride");
  PQ_CHECK_ARG(pb->mg <= 64 && (pb->mg == 0 || (pb->Cg && pb->lg && pb->ug)), "pq_polish_w_batched: bad general rows");
  PQ_CHECK_ARG(ldk % 64 == 0 && ldk >= 64 && ldk <= pb->ld && ldk <= pq::KMAX,
               "pq_polish_w_batched: need 64 <= ldk <= min(ld, %d), multiple of 64 (ldk=%d)", pq::KMAX, ldk);
  PQ_CHECK_ARG(st->K && st->Dt && st->K_stride >= (int64_t)ldk * ldk && st->Dt_stride >= (int64_t)(ldk / 64) * 4096,
               "pq_polish_w_batched: scratch K / Dt too small for ldk=%d", ldk);
  PQ_CHECK_ARG(st->work && st->work_stride >= PQ_WORK_DOUBLES(pb->ld, st->mg_pad),
               "pq_polish_w_batched: work buffer too small");
  const int grid = idx ? nidx : pb->batch;
  if (grid <= 0) return 0;
  hipLaunchKernelGGL(pq::k_polish_w, dim3(grid), dim3(pq::PT), 0, (hipStream_t)stream, *lr, *pb, *st, idx,
                     nidx, *s, ldk, final_try, band, ldo, r0);
  PQ_CHECK_LAUNCH("pq_polish_w_batched");
  return 0;
}
