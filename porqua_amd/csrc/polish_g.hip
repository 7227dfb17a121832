// K4, grouped pipeline: the window-form active-set polish of polish_w.hip restructured as
// a few throughput kernels per active-set round over ALL dates of a backtest, instead of
// one latency-bound workgroup per date that runs every round's phases back to back.
//
// Per round (pq_polish_grouped_round), for every date still pending:
//   setup   (one workgroup per date)   free list F (stable order), active general rows,
//                                       fixed values x_B, reduced rhs pieces;
//   pass 0  (one workgroup per GROUP)  P x_B through the window for dates with x_B != 0,
//                                       both window passes as FP64 MFMA GEMMs over the union
//                                       rows of a slide group (as in the grouped ADMM);
//   form    (one workgroup per date)   P_FF = p_scale w_scale Xc_F'Xc_F + p_diag I, MFMA tile
//                                       products over the window gathered 16 rows at a time;
//   solve   (one workgroup per date)   LDS-resident packed Cholesky of P_FF + delta I
//                                       (16-column panels: one wave factors the diagonal
//                                       block, all waves the panel and the MFMA trailing
//                                       update), the Schur complement of the active rows,
//                                       proximal iterative refinement;
//   pass 1  (one workgroup per GROUP)  exact P x and gradient of the new point through the
//                                       window (MFMA over the union), the active-set checks,
//                                       and for accepted dates the final scoring.
// The arithmetic of every step is polish_w.hip's (same classification, same regularised
// reduced KKT, same refinement, same acceptance tests), so results agree with it to
// rounding.  Dates the pipeline does not take (free set outside 1..128, more than 32
// active rows, a failed factorisation, not accepted within polish_rounds) are marked
// FALLBACK and left untouched for pq_polish_w_batched, which restarts them from the ADMM
// point.
//
// Replaces, with polish_w.hip, the accuracy of qpsolvers' interior-point answer
// (src/qp_problems.py:211-214); scoring as src/qp_problems.py:219-221 and
// example/compare_solver.ipynb:212-216.
#include <cstdlib>
#include <mutex>

#include "polish_dev.h"
#include "capi_util.h"
#include "pg_record.h"

namespace pq {


// ---------------------------------------------------------------------------------------
// init: classification from the ADMM point (polish_w.hip's, verbatim) + problem scale
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(PT) void k_pg_init(pq_lowrank lr, pq_problem pb, pq_state st, double* rec,
                                                pq_settings s) {
  __shared__ double red[16];
  const int b = blockIdx.x;
  const int t = threadIdx.x;
  double* R = rec + (int64_t)b * PGR;
  const int st0 = st.status[b];
  if (st0 != PQ_SOLVED && st0 != PQ_MAX_ITER) {
    if (t == 0) R[R_STATE] = PQ_PG_SKIP;
    return;
  }
  const int n = pb.n, ld = pb.ld, mg = pb.mg;
  const double ps = pb.p_scale ? pb.p_scale[b] : 1.0;
  const double pd = pb.p_diag ? pb.p_diag[b] : 0.0;
  const double psw = ps * (lr.w_scale ? lr.w_scale[b] : 1.0);
  const double* q = pb.q + (int64_t)b * pb.q_stride;
  const double* lg = pb.lg ? pb.lg + (int64_t)b * pb.g_stride : nullptr;
  const double* ug = pb.ug ? pb.ug + (int64_t)b * pb.g_stride : nullptr;
  const bool has_box = pb.lb != nullptr;
  const double* lb = has_box ? pb.lb + (int64_t)b * pb.box_stride : nullptr;
  const double* ub = has_box ? pb.ub + (int64_t)b * pb.box_stride : nullptr;
  const double* sz = st.z + (int64_t)b * st.m_ld;
  const double* sy = st.y + (int64_t)b * st.m_ld;
  const double* sx = st.x + (int64_t)b * ld;
  PGWork wk(st, b, ld);
  const double* dgb = lr.dg + (int64_t)b * lr.dg_stride;
  double sc = 0.0;
  for (int i = t; i < n; i += PT) sc = fmax(sc, fmax(fabs(q[i]), fabs(psw * dgb[i] + pd)));
  sc = block_max(sc, red);
  sc = fmax(sc, 1e-300);
  // centred windows (the mean-variance family, sparse long-only optima): a variable far
  // below the largest distance to its lower bound starts fixed there too (s.polish_fix_rel;
  // the ADMM point of a loose eps leaves small positive weights).  Tracking windows keep
  // OSQP's rule: their free sets are large and the wide rounds border few fixed variables
  double fix_thr = -INFINITY;
  if (s.polish_fix_rel > 0.0 && has_box && lr.mu) {
    double dm = 0.0;
    for (int i = t; i < n; i += PT)
      if (!isinf(lb[i])) dm = fmax(dm, sx[i] - lb[i]);
    fix_thr = s.polish_fix_rel * block_max(dm, red);
  }
  double nfree = 0.0;
  for (int i = t; i < ld; i += PT) {
    int f = 0;
    if (i < n && has_box) {
      const double zi = sz[st.mg_pad + i], yi = sy[st.mg_pad + i];
      if (!isinf(lb[i]) && (zi - lb[i] < -yi || sx[i] - lb[i] < fix_thr)) f = 1;
      else if (!isinf(ub[i]) && ub[i] - zi < yi) f = 2;
      if (lb[i] == ub[i]) f = 1;
    }
    wk.fl[i] = (i < n) ? f : 1;
    wk.xs[i] = (i < n) ? sx[i] : 0.0;
    nfree += (i < n && f == 0) ? 1.0 : 0.0;
  }
  nfree = block_sum(nfree, red);   // the caller reads it to decide whether wide rounds can occur
  if (t < 64) {
    int a = 0;
    double lam = 0.0;
    if (t < mg) {
      const double zr = sz[t], yr = sy[t];
      if (lg[t] == ug[t]) a = 2;
      else if (!isinf(lg[t]) && zr - lg[t] < -yr) a = 1;
      else if (!isinf(ug[t]) && ug[t] - zr < yr) a = 2;
      lam = yr;
    }
    R[R_ACT + t] = a;
    R[R_LAM + t] = lam;
  }
  if (t == 0) {
    R[R_STATE] = PQ_PG_PENDING;
    R[R_ROUNDS] = 0;
    R[R_SC] = sc;
    R[R_K] = nfree;
    R[R_NZB] = 0;
    R[R_W] = 0;
    R[R_FORMED] = 0;
    R[R_REUSE] = 0;
  }
#ifdef PQ_PROFILE
  if (t >= 8 && t < 32) R[t] = 0.0;
#endif
}

// ---------------------------------------------------------------------------------------
// setup: free list, active rows, x_B, dA, the starting point of the refinement
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(PT) void k_pg_setup(pq_problem pb, pq_state st, double* rec, int kmax, int wide_ok,
                                                 int kbig) {
  __shared__ int wcnt[PW];
  __shared__ int s_al[PG_MGMAX + 1];
  __shared__ double red[16];
  const int b = blockIdx.x;
  double* R = rec + (int64_t)b * PGR;
  if (R[R_STATE] != PQ_PG_PENDING) return;   // uniform
  const int n = pb.n, ld = pb.ld, mg = pb.mg;
  const int t = threadIdx.x, w = wave_id(), l = lane_id();
  const double* q = pb.q + (int64_t)b * pb.q_stride;
  const double* Cg = pb.Cg ? pb.Cg + (int64_t)b * pb.Cg_stride : nullptr;
  const double* lg = pb.lg ? pb.lg + (int64_t)b * pb.g_stride : nullptr;
  const double* ug = pb.ug ? pb.ug + (int64_t)b * pb.g_stride : nullptr;
  const bool has_box = pb.lb != nullptr;
  const double* lb = has_box ? pb.lb + (int64_t)b * pb.box_stride : nullptr;
  const double* ub = has_box ? pb.ub + (int64_t)b * pb.box_stride : nullptr;
  PGWork wk(st, b, ld);
  // ---- stable compaction of the free variables: wave w owns a contiguous index range ----
  const int seg = ((n + PW * 64 - 1) / (PW * 64)) * 64;
  const int lo = w * seg, hi = min(n, lo + seg);
  // (every loop over a date's n entries below issues four steps' loads before using them,
  // from clamped addresses: one load round trip per step made the setup ~140 serial round
  // trips at n = 5000)
  int c = 0;
  for (int i0 = lo; i0 < hi; i0 += 4 * 64) {
    int fv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = i0 + 64 * u + l;
      fv[u] = wk.fl[i < hi ? i : lo];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) c += __popcll(__ballot(i0 + 64 * u + l < hi && fv[u] == 0));
  }
  if (l == 0) wcnt[w] = c;
  if (t == 0) {
    int a = 0;
    for (int r = 0; r < mg && a <= PG_MGMAX; ++r)
      if (R[R_ACT + r] != 0.0) s_al[a++] = r;
    s_al[PG_MGMAX] = a;
  }
  __syncthreads();
  int base = 0, k = 0;
  for (int ww = 0; ww < PW; ++ww) {
    if (ww < w) base += wcnt[ww];
    k += wcnt[ww];
  }
  const int ma = s_al[PG_MGMAX];
  // ---- wide mode (polish_gw.hip): a free set beyond the LDS solve with at most PG_WMB
  // bordered rows (active general rows + fixed variables); the group solve works in n-space
  // from x = xs, so neither the free list nor x_B is built -------------------------------
  const int nfx = n - k;
  if (wide_ok && k > kmax && mg <= PG_WG_MAX && ma + nfx <= PG_WMB) {   // uniform
    if (w == 0) {   // fixed variables, ascending
      int nb = 0;
      for (int i0 = 0; i0 < n; i0 += 64) {
        const int i = i0 + l;
        const int f = i < n ? wk.fl[i] : 0;
        const unsigned long long m = __ballot(f != 0);
        if (f != 0) {
          const int j = nb + __popcll(m & ((1ull << l) - 1ull));
          R[R_FIX + j] = i;
          R[R_FIXV + j] = f == 1 ? lb[i] : ub[i];
          R[R_FXL + j] = st.y[(int64_t)b * st.m_ld + st.mg_pad + i];   // the ADMM box dual
        }
        nb += __popcll(m);
      }
    }
    if (t < ma) {
      const int r = s_al[t];
      R[R_AL + t] = r;
      R[R_SOL + t] = R[R_LAM + r];
      R[R_DA + t] = R[R_ACT + r] == 1.0 ? lg[r] : ug[r];
    }
    if (t == 0) {
      R[R_K] = k;
      R[R_MA] = ma;
      R[R_NZB] = 0;
      R[R_W] = 1;
      R[R_NFX] = nfx;
      R[R_ROUNDS] += 1.0;
    }
    return;
  }
  // every variable at a bound (a vertex, e.g. nearly linear objectives): x = x_B, and the
  // multiplier of at most one active equality row is chosen in the post from the dual
  // feasibility interval of the bound variables (k_pg_post); otherwise the per-date kernel
  const bool vertex_ok = ma == 0 || (ma == 1 && lg[s_al[0]] == ug[s_al[0]]);
  // (kmax < k <= kbig: the large-free-set solve k_pg_big)
  if ((k == 0 && !vertex_ok) || k > kbig || ma > PG_MGMAX) {   // uniform
    if (t == 0) R[R_STATE] = PQ_PG_FALLBACK;
    return;
  }
  for (int i0 = lo; i0 < hi; i0 += 4 * 64) {
    int fv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = i0 + 64 * u + l;
      fv[u] = wk.fl[i < hi ? i : lo];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = i0 + 64 * u + l;
      const bool f = i < hi && fv[u] == 0;
      const unsigned long long m = __ballot(f);
      if (f) wk.Fl[base + __popcll(m & ((1ull << l) - 1ull))] = i;
      base += __popcll(m);
    }
  }
  // ---- P_FF reuse: every free variable in the free list of the last form (the usual later
  //      round only fixes variables) -> the solve gathers P_FF from K ---------------------------
  int reuse = 0;
  if (R[R_FORMED] == 1.0) {
    __syncthreads();   // Fl complete
    int miss = 0;
    for (int p = t; p < k; p += PT) miss |= wk.posF[wk.Fl[p]] < 0;
    reuse = !block_or(miss, red);
  }
  // ---- fixed values, nzb -------------------------------------------------------------------
  int nzb = 0;
  for (int i0 = t; i0 < ld; i0 += 4 * PT) {
    int fv[4];
    double lv[4], uv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = i0 + u * PT, ic = i < n ? i : 0;
      fv[u] = wk.fl[i < ld ? i : 0];
      lv[u] = has_box ? lb[ic] : 0.0;
      uv[u] = has_box ? ub[ic] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = i0 + u * PT;
      if (i >= ld) continue;
      const int f = fv[u];
      const double v = i < n ? (f == 1 ? lv[u] : (f == 2 ? uv[u] : 0.0)) : 0.0;
      wk.xb[i] = v;
      if (k == 0) wk.xs[i] = v;
      nzb |= (v != 0.0);
    }
  }
  nzb = block_or(nzb, red);   // barrier: Fl complete below
  // ---- d_a = rhs_a - C_aB x_B ----------------------------------------------------------------
  for (int a = w; a < ma; a += PW) {
    const int r = s_al[a];
    const double* cr = Cg + (int64_t)r * ld;
    double sum = 0.0;
    for (int j0 = l; j0 < n; j0 += 8 * 64) {   // (the same per-lane order, eight loads ahead)
      double cv[8], xv[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int j = j0 + 64 * u, jc = j < n ? j : 0;
        cv[u] = cr[jc];
        xv[u] = wk.xb[jc];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (j0 + 64 * u < n) sum += cv[u] * xv[u];
    }
    sum = wave_sum(sum);
    if (l == 0) R[R_DA + a] = (R[R_ACT + r] == 1.0 ? lg[r] : ug[r]) - sum;
  }
  const int kp = (k + 15) & ~15;
  for (int p = t; p < kp; p += PT) {
    const int i = p < k ? wk.Fl[p] : 0;
    wk.solx[p] = p < k ? wk.xs[i] : 0.0;
    wk.rF[p] = p < k ? -q[i] : 0.0;
  }
  if (t < ma) {
    R[R_AL + t] = s_al[t];
    R[R_SOL + t] = R[R_LAM + s_al[t]];
  }
  if (t == 0) {
    R[R_K] = k;
    R[R_KB] = k;
    R[R_MA] = ma;
    R[R_NZB] = nzb;
    R[R_W] = 0;
    R[R_REUSE] = reuse;
    R[R_GFORM] = 0;
    R[R_ROUNDS] += 1.0;
  }
}

// ---------------------------------------------------------------------------------------
// form: P_FF (both triangles, from the lower 16x16 tiles) into the date's K scratch (pitch
// ldk).  16-granular tiles: a free set of k needs only round16(k)^2 / 2 of MFMA work (a
// 64-granular tiling computes up to 3x more for the typical k = 65..96), and the small
// register footprint keeps several workgroups per CU to hide the gather latency.
// ---------------------------------------------------------------------------------------
constexpr int FKCH = 16;            // window rows per staged chunk
constexpr int FPIT = PG_KMAX + 4;   // LDS pitch (doubles)
constexpr int FT = 512;             // threads (8 waves)
constexpr int GMAXT = 512;          // window rows held in LDS by k_pg_form
constexpr int FNW = FT / 64;
constexpr int FTW = 5;              // 16x16 tiles per wave (36 lower tiles for k <= 128)

// group form (k_pg_form_grp): the Gram of a polish group's union rows over the union of its
// forming dates' free lists, centred by one of their means, in the group's pass scratch
// (pitch GLD), with the union free list, that mean and the union column sums beside it
constexpr int GLD = PG_KMAX;
constexpr int64_t GS_COL = (int64_t)GLD * GLD, GS_MU = GS_COL + GLD, GS_CS = GS_MU + GLD, GS_N = GS_CS + GLD;
static_assert(GS_N + 1 <= PQ_PG_PASS_SCRATCH, "group form scratch exceeds the pass scratch");
constexpr int GMO = 32;   // union rows outside a date's window (the per-date correction)
// big group form (k_pg_form_grp_big, uncentred windows, free sets of PG_KMAX + 1 .. PG_KBIG):
// the Gram of the group's union rows over the union of its forming dates' free lists (at most
// KBG columns), pitch KBG, in the group's pass scratch after the window passes' region
// (GB_OFF doubles: QSCR, checked below), with the union free list and its length beside it
constexpr int KBG = 320;   // 16-date unions of config 2's free sets: 261 mean, 313 max (r05G_diag_union.log)
constexpr int64_t GB_OFF = 20816;
constexpr int64_t GB_COL = GB_OFF + (int64_t)KBG * KBG, GB_N = GB_COL + KBG, GB_END = GB_N + 1;
static_assert(GB_END <= PQ_PG_PASS_SCRATCH, "big group form scratch exceeds the pass scratch");
constexpr int GBS = 4;    // workgroups per group of the big Gram (its lower tiles split between them)
constexpr int FKB = 8;    // union rows per staged chunk of the big Gram

// P_FF of date b from its group's Gram G (centred by mu_g over the union rows U):
//   sum_{t in W} (x_t - mu)(x_t - mu)' = G_FF - sum_{o in U \ W} x~_o x~_o'
//                                         - d s' - s d' + T d d'
// with x~ = x - mu_g, d = mu - mu_g and s = sum_{t in W} x~_t (union column sums minus the
// outside rows) -- exact for any centring vector mu.  The outside rows (U - T <= GMO) are
// staged in LDS; one thread per lower entry.
__device__ __forceinline__ void form_from_group(const pq_lowrank& lr, const pq_problem& pb, const pq_state& st,
                                                double* R, int b, int k, int ldk, const int32_t* gdates,
                                                int ngroups, const int32_t* urows_all, const int32_t* ucnt_all,
                                                const int32_t* uoff, int umax, const double* scr, double* S) {
  __shared__ int s_cu[GLD], s_pi[PG_KMAX], s_fl[PG_KMAX], s_ou[GMO];
  __shared__ double s_gmu[GLD], s_d[PG_KMAX], s_s[PG_KMAX];
  const int ld = pb.ld;
  const int t = threadIdx.x;
  const int grp = (int)R[R_GFORM] - 1;   // set by k_pg_form_grp
  const double* Gs = scr + (int64_t)grp * PQ_PG_PASS_SCRATCH;
  const int nc = (int)Gs[GS_N];
  const int U = ucnt_all[grp], off = uoff[b], T = lr.tlen[b], mo = U - T;
  PGWork wk(st, b, ld);
  const double ps = pb.p_scale ? pb.p_scale[b] : 1.0;
  const double pd = pb.p_diag ? pb.p_diag[b] : 0.0;
  const double psw = ps * (lr.w_scale ? lr.w_scale[b] : 1.0);
  const double* mu = lr.mu ? lr.mu + (int64_t)b * lr.mu_stride : nullptr;
  const int32_t* ur = urows_all + (int64_t)grp * umax;
  // the independent reads of every list first (one memory round trip; the date's means at
  // its free variables one more): union free list and centre, the date's free list, the union
  // rows outside its window
  double muF = 0.0;
  for (int c = t; c < nc; c += FT) {
    s_cu[c] = (int)Gs[GS_COL + c];
    s_gmu[c] = Gs[GS_MU + c];
  }
  for (int p = t; p < k; p += FT) {
    const int i = wk.Fl[p];
    s_fl[p] = i;
    muF = mu ? mu[i] : 0.0;   // (k <= PG_KMAX <= FT: one free variable per thread)
  }
  for (int o = t; o < mo; o += FT) s_ou[o] = ur[o < off ? o : o + T];
  __syncthreads();
  // union position of each free variable (s_cu ascending) and the outside rows' raw values
  if (t < k) {
    const int i = s_fl[t];
    int a = 0, z = nc;
    while (z - a > 1) {
      const int mid = (a + z) >> 1;
      if (s_cu[mid] <= i) a = mid; else z = mid;
    }
    s_pi[t] = a;
    s_d[t] = muF - s_gmu[a];
  }
  const int nt = (k + 15) >> 4, kp = 16 * nt, mo4 = (mo + 3) & ~3;
  for (int e = t; e < mo4 * kp; e += FT) {   // (zero beyond k, and whole zero rows up to mo4)
    const int o = e / kp, p = e - o * kp;
    S[e] = (o < mo && p < k) ? lr.panel[(int64_t)s_ou[o] * lr.ldp + s_fl[p]] : 0.0;
  }
  __syncthreads();
  // centred by the union's centre, and s = union column sums - outside rows
  for (int e = t; e < mo * kp; e += FT) {
    const int p = e % kp;
    if (p < k) S[e] -= s_gmu[s_pi[p]];
  }
  __syncthreads();
  for (int p = t; p < k; p += FT) {
    double v = Gs[GS_CS + s_pi[p]];
    for (int o = 0; o < mo; ++o) v -= S[o * kp + p];
    s_s[p] = v;
  }
  __syncthreads();
  // the lower 16 x 16 tiles, FTW per wave: acc = G_FF - X_o,F' X_o,F by MFMA over the outside
  // rows (4 per step), then the centring terms, into K (both triangles) -- instead of one
  // thread per entry summing its mo products from LDS
  double* K = st.K + (int64_t)b * st.K_stride;
  const double Td = (double)T;
  const int l = lane_id(), wu = __builtin_amdgcn_readfirstlane(wave_id());
  const int ntile = nt * (nt + 1) / 2;
#pragma unroll
  for (int j = 0; j < FTW; ++j) {
    const int q = wu + FNW * j;
    if (q >= ntile) break;   // (uniform)
    int I = (int)((sqrt(8.0 * q + 1.0) - 1.0) * 0.5);
    while ((I + 1) * (I + 2) / 2 <= q) ++I;
    while (I * (I + 1) / 2 > q) --I;
    const int J = q - I * (I + 1) / 2;
    const int gj = 16 * J + (l & 15), pj = s_pi[gj < k ? gj : 0];
    f64x4 acc;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int gi = 16 * I + (l >> 4) + 4 * r;
      acc[r] = Gs[(int64_t)s_pi[gi < k ? gi : 0] * GLD + pj];
    }
    for (int o0 = 0; o0 < mo4; o0 += 4) {
      const double* so = S + (o0 + (l >> 4)) * kp + (l & 15);
      acc = __builtin_amdgcn_mfma_f64_16x16x4f64(-so[16 * I], so[16 * J], acc, 0, 0, 0);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int gi = 16 * I + (l >> 4) + 4 * r;
      if (gi < k && gj < k && gj <= gi) {
        double v = acc[r] - (s_d[gi] * s_s[gj] + s_s[gi] * s_d[gj]);
        v = fma(Td * s_d[gi], s_d[gj], v);
        const double val = psw * v + (gi == gj ? pd : 0.0);
        K[(int64_t)gi * ldk + gj] = val;
        K[(int64_t)gj * ldk + gi] = val;
      }
    }
  }
  // positions of the formed free list, in one pass (the free list is ascending: setup builds it
  // in index order and the solves' inner steps compact it in order)
  for (int i = t; i < pb.n; i += FT) {
    int a = 0, z = k;
    while (z - a > 1) {
      const int mid = (a + z) >> 1;
      if (s_fl[mid] <= i) a = mid; else z = mid;
    }
    wk.posF[i] = (k > 0 && s_fl[a] == i) ? a : -1;
  }
  if (t == 0) R[R_FORMED] = 1.0;
}

// KF = PG_KMAX: the LDS solve's free sets (and the group form); KF = PG_KBIG: the free sets
// of k_pg_big (PG_KMAX < k <= PG_KBIG), formed here the same way -- every window chunk
// gathered once for all tiles -- instead of one window pass per 64 x 64 tile
template <int KF>
__device__ __forceinline__ void pg_form_date(int b, const pq_lowrank& lr, const pq_problem& pb, const pq_state& st,
                                             double* rec, int ldk, const int32_t* gdates, int ngroups,
                                             const int32_t* urows_all, const int32_t* ucnt_all,
                                             const int32_t* uoff, int umax, const double* scr) {
  constexpr int FPITK = KF + 4;                        // LDS pitch (doubles)
  constexpr int NCG = KF / 32;                         // gathered columns per thread and row
  constexpr int NTL = (KF / 16) * (KF / 16 + 1) / 2;   // lower 16 x 16 tiles
  constexpr int FTWK = (NTL + FNW - 1) / FNW;          // tiles per wave
  static_assert(KF != PG_KMAX || FTWK == FTW, "k_pg_form tiling");
  __shared__ __attribute__((aligned(16))) double S[2 * FKCH * FPITK];
  double* R = rec + (int64_t)b * PGR;
  if (R[R_STATE] != PQ_PG_PENDING || R[R_W] != 0.0) return;   // wide dates: polish_gw.hip
  const int k = (int)R[R_K];
  if (KF == PG_KMAX && threadIdx.x == 0) {   // the date joins its solve bucket's list
    const int kb = (int)R[R_KB], kmax = ldk < PG_KMAX ? ldk : PG_KMAX, kbig = ldk < PG_KBIG ? ldk : PG_KBIG;
    if (kb >= 1 && kb <= kbig) {
      const int bk = kb <= kmax ? pg_bucket(kb) : PG_BIGB;
      const unsigned long long i = atomicAdd(reinterpret_cast<unsigned long long*>(rec + R_CNT) + bk, 1ull);
      rec[(int64_t)i * PGR + R_LIST + bk] = (double)b;
    }
  }
  if (KF == PG_KMAX ? (k > PG_KMAX || k == 0) : (k <= PG_KMAX || k > KF)) return;
  if (R[R_REUSE] != 0.0) {   // P_FF is a principal submatrix of the formed one: nothing to form
    if (R[R_NZB] != 0.0) {   // (the reduced rhs still takes P_FB x_B from pass 0)
      PGWork wk0(st, b, pb.ld);
      const double ps0 = pb.p_scale ? pb.p_scale[b] : 1.0;
      for (int p = threadIdx.x; p < k; p += FT) wk0.rF[p] -= ps0 * wk0.pxb[wk0.Fl[p]];
    }
    return;
  }
  const int ld = pb.ld;
  const int t = threadIdx.x, w = wave_id(), l = lane_id();
  PGWork wk(st, b, ld);
  const double ps = pb.p_scale ? pb.p_scale[b] : 1.0;
  const double pd = pb.p_diag ? pb.p_diag[b] : 0.0;
  const double psw = ps * (lr.w_scale ? lr.w_scale[b] : 1.0);
  if (R[R_NZB] != 0.0)   // rF = -q_F - p_scale (w_scale Xc'Xc x_B)_F  (pass 0 left it in pxb)
    for (int p = t; p < k; p += FT) wk.rF[p] -= ps * wk.pxb[wk.Fl[p]];
  if constexpr (KF == PG_KMAX) {
    if (R[R_GFORM] != 0.0) {   // from the group Gram (k_pg_form_grp)
      form_from_group(lr, pb, st, R, b, k, ldk, gdates, ngroups, urows_all, ucnt_all, uoff, umax, scr, S);
      return;
    }
  }
  // big free sets from the group Gram (k_pg_form_grp_big, uncentred windows): P_FF =
  // G_FF - X_o,F' X_o,F over the union rows o outside the window (at most GMO), the same tile
  // MFMAs over those rows instead of the window's T, the accumulators starting at -G_FF
  const bool from_g = KF == PG_KBIG && R[R_GFORM] != 0.0;   // (uniform)
  const int grp_g = from_g ? (int)R[R_GFORM] - 1 : 0;
  const double* Gb = scr + (int64_t)grp_g * PQ_PG_PASS_SCRATCH;
  const int Tw = lr.tlen[b];
  const int T = from_g ? ucnt_all[grp_g] - Tw : Tw;   // rows accumulated
  const double* mu = (lr.mu && !from_g) ? lr.mu + (int64_t)b * lr.mu_stride : nullptr;
  // the window's row indices in LDS: a gather's row address is then one LDS read away, not a
  // dependent global load
  __shared__ int s_rws[GMAXT];
  const int32_t* g_rws = lr.rows + (int64_t)b * lr.tmax;
  const bool lds_rows = from_g || T <= GMAXT;   // (uniform; longer windows read the indices from memory)
  if (from_g) {   // the union rows outside [off, off + Tw)
    const int off = uoff[b];
    const int32_t* ur = urows_all + (int64_t)grp_g * umax;
    for (int tt = t; tt < T; tt += FT) s_rws[tt] = ur[tt < off ? tt : tt + Tw];
  } else {
    for (int tt = t; lds_rows && tt < T; tt += FT) s_rws[tt] = g_rws[tt];
  }
  __syncthreads();
  auto rws = [&](int tt) -> int { return lds_rows ? s_rws[tt] : g_rws[tt]; };
  const int nt = (k + 15) >> 4, ntile = nt * (nt + 1) / 2;
  const int kp = nt * 16;
  // gather map: thread t -> window row t / 32 of a chunk, free columns (t % 32) + 32 c
  const int gr = t >> 5, gc = t & 31;
  int col[NCG];
  double mc[NCG];
#pragma unroll
  for (int c = 0; c < NCG; ++c) {
    const int p = gc + 32 * c;
    col[c] = p < k ? wk.Fl[p] : -1;
    mc[c] = (col[c] >= 0 && mu) ? mu[col[c]] : 0.0;
  }
  double v[NCG];
  // unconditional loads (clamped row / column, zeroed by a factor after the load: a conditional
  // load makes the compiler wait for every outstanding load there)
  auto gather = [&](int t0) {
    const int tt = t0 + gr;
    const double* row = lr.panel + (int64_t)rws(tt < T ? tt : 0) * lr.ldp;
#pragma unroll
    for (int c = 0; c < NCG; ++c) {
      const double x = row[col[c] >= 0 ? col[c] : 0];
      v[c] = (x - mc[c]) * ((tt < T && col[c] >= 0) ? 1.0 : 0.0);
    }
  };
  auto put = [&](double* Sb) {
#pragma unroll
    for (int c = 0; c < NCG; ++c)
      if (gc + 32 * c < kp) Sb[gr * FPITK + gc + 32 * c] = v[c];
  };
  // this wave's tiles (I, J), I >= J, in column-major order of the lower triangle (from the
  // wave index made uniform: the tile coordinates stay in scalar registers)
  const int wu = __builtin_amdgcn_readfirstlane(w);
  int tI[FTWK], tJ[FTWK];
#pragma unroll
  for (int j = 0; j < FTWK; ++j) {
    const int q = wu + FNW * j;
    int I = (int)((sqrt(8.0 * q + 1.0) - 1.0) * 0.5);
    while ((I + 1) * (I + 2) / 2 <= q) ++I;
    while (I * (I + 1) / 2 > q) --I;
    tI[j] = I;
    tJ[j] = q - I * (I + 1) / 2;
  }
  f64x4 acc[FTWK];
#pragma unroll
  for (int j = 0; j < FTWK; ++j) acc[j] = f64x4{0.0, 0.0, 0.0, 0.0};
  if (from_g) {   // acc = -G_FF: the union position of each free variable, then the tiles' entries
    __shared__ int s_gp[KF];
    const int nc = (int)Gb[GB_N];
    for (int p = t; p < k; p += FT) {   // (the union list is ascending)
      const int i = wk.Fl[p];
      int a = 0, z = nc;
      while (z - a > 1) {
        const int mid = (a + z) >> 1;
        if ((int)Gb[GB_COL + mid] <= i) a = mid; else z = mid;
      }
      s_gp[p] = a;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < FTWK; ++j) {
      if (wu + FNW * j < ntile) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int gi = 16 * tI[j] + (l >> 4) + 4 * r, gj = 16 * tJ[j] + (l & 15);
          acc[j][r] = (gi < k && gj < k) ? -Gb[GB_OFF + (int64_t)s_gp[gi] * KBG + s_gp[gj]] : 0.0;
        }
      }
    }
  }
  auto mma = [&](const double* Sb) {
#pragma unroll
    for (int kk = 0; kk < FKCH; kk += 4) {
      const double* r = Sb + (kk + (l >> 4)) * FPITK + (l & 15);
#pragma unroll
      for (int j = 0; j < FTWK; ++j)
        if (wu + FNW * j < ntile)
          acc[j] = __builtin_amdgcn_mfma_f64_16x16x4f64(r[16 * tI[j]], r[16 * tJ[j]], acc[j], 0, 0, 0);
    }
  };
  double* S0 = S;
  double* S1 = S + FKCH * FPITK;
  gather(0);
  put(S0);
  __syncthreads();
  int buf = 0;
  for (int t0 = 0; t0 < T; t0 += FKCH) {   // (T = 0, from the group Gram alone: no chunk)
    const bool more = t0 + FKCH < T;
    if (more) gather(t0 + FKCH);
    mma(buf ? S1 : S0);
    if (more) put(buf ? S0 : S1);
    __syncthreads();
    buf ^= 1;
  }
  double* K = st.K + (int64_t)b * st.K_stride;
  for (int i = t; i < pb.n; i += FT) wk.posF[i] = -1;   // positions of the formed free list
  __syncthreads();
  for (int p = t; p < k; p += FT) wk.posF[wk.Fl[p]] = p;
  if (t == 0) R[R_FORMED] = 1.0;   // (k_pg_big factors in place and clears it again)
#pragma unroll
  for (int j = 0; j < FTWK; ++j) {
    if (wu + FNW * j < ntile) {
      // k_pg_big (KF = PG_KBIG) reads the diagonal 64-blocks in full and the off-diagonal
      // originals from the upper half only (its factor overwrites the lower off-diagonal
      // blocks with L): those lower writes are skipped
      const bool lower = KF != PG_KBIG || (tI[j] >> 2) == (tJ[j] >> 2);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int gi = 16 * tI[j] + (l >> 4) + 4 * r, gj = 16 * tJ[j] + (l & 15);
        const double v = psw * (from_g ? -acc[j][r] : acc[j][r]) + (gi == gj ? pd : 0.0);
        if (lower) K[(int64_t)gi * ldk + gj] = v;
        if (tI[j] != tJ[j]) K[(int64_t)gj * ldk + gi] = v;   // both triangles: column reads in the solve
      }
    }
  }
}

// KF = PG_KMAX: one workgroup per date (and the bucket lists' appends); KF = PG_KBIG: a
// resident grid striding over the large free sets' list (most backtests have none: one
// workgroup per date needed its 66 KB of LDS only to exit, behind the solves on the CUs)
template <int KF>
__global__ __launch_bounds__(FT) void k_pg_form(pq_lowrank lr, pq_problem pb, pq_state st, double* rec,
                                                int ldk, const int32_t* gdates, int ngroups,
                                                const int32_t* urows_all, const int32_t* ucnt_all,
                                                const int32_t* uoff, int umax, const double* scr) {
  if constexpr (KF == PG_KMAX) {
    pg_form_date<KF>(blockIdx.x, lr, pb, st, rec, ldk, gdates, ngroups, urows_all, ucnt_all, uoff, umax, scr);
  } else {
    const int cnt = (int)pg_count(rec, PG_BIGB);
    for (int i = blockIdx.x; i < cnt; i += gridDim.x) {
      pg_form_date<KF>(pg_listed(rec, PG_BIGB, i), lr, pb, st, rec, ldk, gdates, ngroups, urows_all, ucnt_all,
                       uoff, umax, scr);
      __syncthreads();   // (LDS reused by the next date)
    }
  }
}

// ---------------------------------------------------------------------------------------
// group form: one workgroup per polish group with dates that form P_FF this round (pending,
// not reusing K, 0 < |F| <= 128, at most GMO union rows outside the window).  Their free
// lists are merged in column order; when the union stays within PG_KMAX columns, the Gram of
// the group's union rows over it (centred by the first forming date's mean) is one MFMA tile
// product as in k_pg_form -- the union is gathered once for up to 16 dates instead of each
// window once per date -- and k_pg_form derives each date's P_FF from it (form_from_group).
// Otherwise the dates keep R_GFORM = 0 and k_pg_form forms them alone.
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(FT) void k_pg_form_grp(pq_lowrank lr, pq_problem pb, pq_state st, double* rec,
                                                    const int32_t* gdates, const int32_t* urows_all,
                                                    const int32_t* ucnt_all, int umax, double* scr,
                                                    int min_dates) {
  __shared__ __attribute__((aligned(16))) double S[2 * FKCH * FPIT];
  __shared__ int s_col[PG_KMAX], s_on[16], s_wcnt[FNW], s_ncol;
  __shared__ double s_gm[PG_KMAX];
  const int grp = xcd_slot(blockIdx.x, gridDim.x);
  const int d0 = gdates[grp], G = gdates[grp + 1] - d0, U = ucnt_all[grp];
  const int t = threadIdx.x, w = wave_id(), l = lane_id();
  const int n = pb.n, ld = pb.ld;
  if (t < 16) {
    int on = 0;
    if (t < G) {
      const double* R = rec + (int64_t)(d0 + t) * PGR;
      const int k = (int)R[R_K];
      on = R[R_STATE] == PQ_PG_PENDING && R[R_W] == 0.0 && R[R_REUSE] == 0.0 && k > 0 && k <= PG_KMAX &&
           U - lr.tlen[d0 + t] <= GMO;
    }
    s_on[t] = on;
  }
  if (t == 0) s_ncol = 0;
  __syncthreads();
  int first = -1, non = 0;
  for (int g = G - 1; g >= 0; --g)
    if (s_on[g]) {
      first = g;
      ++non;
    }
  if (non < min_dates) return;   // uniform: too few to pay for the union pass, they form alone
  // ---- union of the forming dates' free lists, in column order (ballot + wave prefix) ----
  for (int cb = 0; cb < n; cb += FT) {
    const int i = cb + t;
    bool f = false;
    {   // every date's flag loaded at once (clamped, unconditional), then combined
      int fv[16];
#pragma unroll
      for (int g = 0; g < 16; ++g) {
        PGWork wg(st, d0 + (g < G ? g : 0), ld);
        fv[g] = wg.fl[i < n ? i : 0];
      }
#pragma unroll
      for (int g = 0; g < 16; ++g) f |= g < G && s_on[g] && fv[g] == 0;
      f = f && i < n;
    }
    const unsigned long long bal = __ballot(f);
    if (l == 0) s_wcnt[w] = __popcll(bal);
    __syncthreads();
    int pos = s_ncol;
    for (int ww = 0; ww < w; ++ww) pos += s_wcnt[ww];
    pos += __popcll(bal & ((1ull << l) - 1ull));
    if (f && pos < PG_KMAX) s_col[pos] = i;
    __syncthreads();
    if (t == 0)
      for (int ww = 0; ww < FNW; ++ww) s_ncol += s_wcnt[ww];
    __syncthreads();
  }
  const int nc = s_ncol;
  if (nc > PG_KMAX) return;   // uniform: the dates form alone
  const double* mug = lr.mu ? lr.mu + (int64_t)(d0 + first) * lr.mu_stride : nullptr;
  for (int c = t; c < PG_KMAX; c += FT) s_gm[c] = (c < nc && mug) ? mug[s_col[c]] : 0.0;
  __syncthreads();
  // ---- Gram of the union rows over the union free list (k_pg_form's tiling) ---------------
  __shared__ int ur[GMAXT];   // the union's row indices in LDS (a gather's row address is one LDS read away)
  for (int u = t; u < U && u < GMAXT; u += FT) ur[u] = urows_all[(int64_t)grp * umax + u];
  __syncthreads();
  const int nt = (nc + 15) >> 4, ntile = nt * (nt + 1) / 2;
  const int kp = nt * 16;
  const int gr = t >> 5, gc = t & 31;
  int col[4];
  double mc[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const int p = gc + 32 * c;
    col[c] = p < nc ? s_col[p] : -1;
    mc[c] = p < nc ? s_gm[p] : 0.0;
  }
  // two chunks' gathers in flight (v1 for the next chunk, v2 for the one after): the chunk
  // loop is bound by the gather latency, not by its MFMAs
  double v1[4], v2[4];
  auto gather = [&](double (&v)[4], int t0) {   // (unconditional loads, as k_pg_form's gather)
    const int tt = t0 + gr;
    const double* row = lr.panel + (int64_t)ur[tt < U ? tt : 0] * lr.ldp;
#pragma unroll
    for (int c = 0; c < 4; ++c) v[c] = row[col[c] >= 0 ? col[c] : 0];
  };
  auto put = [&](const double (&v)[4], double* Sb, int t0) {   // centred and masked on the way to LDS
    const int tt = t0 + gr;
#pragma unroll
    for (int c = 0; c < 4; ++c)
      if (gc + 32 * c < kp) Sb[gr * FPIT + gc + 32 * c] = (v[c] - mc[c]) * ((tt < U && col[c] >= 0) ? 1.0 : 0.0);
  };
  int tI[FTW], tJ[FTW];
#pragma unroll
  for (int j = 0; j < FTW; ++j) {
    const int q = w + FNW * j;
    int I = (int)((sqrt(8.0 * q + 1.0) - 1.0) * 0.5);
    while ((I + 1) * (I + 2) / 2 <= q) ++I;
    while (I * (I + 1) / 2 > q) --I;
    tI[j] = I;
    tJ[j] = q - I * (I + 1) / 2;
  }
  f64x4 acc[FTW];
#pragma unroll
  for (int j = 0; j < FTW; ++j) acc[j] = f64x4{0.0, 0.0, 0.0, 0.0};
  auto mma = [&](const double* Sb) {
#pragma unroll
    for (int kk = 0; kk < FKCH; kk += 4) {
      const double* r = Sb + (kk + (l >> 4)) * FPIT + (l & 15);
#pragma unroll
      for (int j = 0; j < FTW; ++j)
        if (w + FNW * j < ntile)
          acc[j] = __builtin_amdgcn_mfma_f64_16x16x4f64(r[16 * tI[j]], r[16 * tJ[j]], acc[j], 0, 0, 0);
    }
  };
  double csum = 0.0;   // thread t < nc: column sum of the centred union rows
  auto colsum = [&](const double* Sb, int t0) {
    if (t < nc)
      for (int rr = 0; rr < FKCH && t0 + rr < U; ++rr) csum += Sb[rr * FPIT + t];
  };
  double* S0 = S;
  double* S1 = S + FKCH * FPIT;
  // chunk t0 in LDS buffer sb; vr holds chunk t0 + FKCH (issued a step earlier), vi receives
  // chunk t0 + 2 FKCH: each gather has two steps of MFMAs and stores to arrive
  auto step = [&](int t0, double* sb, double* so, double (&vr)[4], double (&vi)[4]) {
    if (t0 + 2 * FKCH < U) gather(vi, t0 + 2 * FKCH);
    mma(sb);
    colsum(sb, t0);
    if (t0 + FKCH < U) put(vr, so, t0 + FKCH);
    __syncthreads();
  };
  gather(v1, 0);
  put(v1, S0, 0);
  gather(v1, FKCH);
  __syncthreads();
  for (int t0 = 0; t0 < U; t0 += 2 * FKCH) {
    step(t0, S0, S1, v1, v2);
    if (t0 + FKCH < U) step(t0 + FKCH, S1, S0, v2, v1);
  }
  double* Gs = scr + (int64_t)grp * PQ_PG_PASS_SCRATCH;
#pragma unroll
  for (int j = 0; j < FTW; ++j) {
    if (w + FNW * j < ntile) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int gi = 16 * tI[j] + (l >> 4) + 4 * r, gj = 16 * tJ[j] + (l & 15);
        Gs[(int64_t)gi * GLD + gj] = acc[j][r];
        if (tI[j] != tJ[j]) Gs[(int64_t)gj * GLD + gi] = acc[j][r];
      }
    }
  }
  for (int c = t; c < nc; c += FT) {
    Gs[GS_COL + c] = s_col[c];
    Gs[GS_MU + c] = s_gm[c];
  }
  if (t < nc) Gs[GS_CS + t] = csum;
  if (t == 0) Gs[GS_N] = nc;
  if (t < G && s_on[t]) rec[(int64_t)(d0 + t) * PGR + R_GFORM] = grp + 1;   // the date's group, + 1
}

// ---------------------------------------------------------------------------------------
// big group form: GBS workgroups per polish group with at least min_dates dates that form a
// free set of PG_KMAX + 1 .. PG_KBIG this round on an uncentred window (the tracking
// objectives: pending, not reusing K, at most GMO union rows outside the window).  Each merges
// the dates' free lists in column order (identically) and, when the union stays within KBG
// columns, computes its share of the lower 16 x 16 tiles of the union rows' Gram over it,
// X_U,F' X_U,F, into the group's pass scratch (pitch KBG); k_pg_form<PG_KBIG> then forms each
// date's P_FF = G_FF - X_o,F' X_o,F from it with its outside rows only (about U - T = 15 rows
// instead of T = 252 per date and round).  Otherwise the dates keep R_GFORM = 0 and form alone.
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(FT) void k_pg_form_grp_big(pq_lowrank lr, pq_problem pb, pq_state st, double* rec,
                                                        const int32_t* gdates, const int32_t* urows_all,
                                                        const int32_t* ucnt_all, int umax, double* scr,
                                                        int min_dates) {
  constexpr int FPB = KBG + 4;                               // LDS pitch (doubles)
  constexpr int NTB = (KBG / 16) * (KBG / 16 + 1) / 2;        // lower tiles of a full union
  constexpr int TPW = ((NTB + GBS - 1) / GBS + FNW - 1) / FNW;   // tiles per wave
  constexpr int NCB = KBG / 64;                              // gathered columns per thread and row
  static_assert(FT == 64 * FKB, "k_pg_form_grp_big: one staged row per wave");
  __shared__ __attribute__((aligned(16))) double S[2 * FKB * FPB];
  __shared__ int s_col[KBG], s_on[16], s_wcnt[FNW], s_ncol;
  const int slot = xcd_slot(blockIdx.x, gridDim.x);   // the GBS parts of a group on one XCD (its L2)
  const int grp = slot / GBS, part = slot - grp * GBS;
  const int d0 = gdates[grp], G = gdates[grp + 1] - d0, U = ucnt_all[grp];
  const int t = threadIdx.x, w = wave_id(), l = lane_id();
  const int n = pb.n, ld = pb.ld;
  if (lr.mu != nullptr) return;   // (uniform) centred windows: the small form's corrections only
  if (t < 16) {
    int on = 0;
    if (t < G) {
      const double* R = rec + (int64_t)(d0 + t) * PGR;
      const int k = (int)R[R_K];
      on = R[R_STATE] == PQ_PG_PENDING && R[R_W] == 0.0 && R[R_REUSE] == 0.0 && k > PG_KMAX && k <= PG_KBIG &&
           U - lr.tlen[d0 + t] <= GMO;
    }
    s_on[t] = on;
  }
  if (t == 0) s_ncol = 0;
  __syncthreads();
  int non = 0;
  for (int g = 0; g < G; ++g) non += s_on[g];
  if (non < min_dates) return;   // uniform
  // ---- union of the forming dates' free lists, in column order (as k_pg_form_grp) -----------
  for (int cb = 0; cb < n; cb += FT) {
    const int i = cb + t;
    bool f = false;
    {
      int fv[16];
#pragma unroll
      for (int g = 0; g < 16; ++g) {
        PGWork wg(st, d0 + (g < G ? g : 0), ld);
        fv[g] = wg.fl[i < n ? i : 0];
      }
#pragma unroll
      for (int g = 0; g < 16; ++g) f |= g < G && s_on[g] && fv[g] == 0;
      f = f && i < n;
    }
    const unsigned long long bal = __ballot(f);
    if (l == 0) s_wcnt[w] = __popcll(bal);
    __syncthreads();
    int pos = s_ncol;
    for (int ww = 0; ww < w; ++ww) pos += s_wcnt[ww];
    pos += __popcll(bal & ((1ull << l) - 1ull));
    if (f && pos < KBG) s_col[pos] = i;
    __syncthreads();
    if (t == 0)
      for (int ww = 0; ww < FNW; ++ww) s_ncol += s_wcnt[ww];
    __syncthreads();
  }
  const int nc = s_ncol;
  if (nc > KBG) return;   // uniform: the dates form alone
  __shared__ int ur[GMAXT];
  for (int u = t; u < U && u < GMAXT; u += FT) ur[u] = urows_all[(int64_t)grp * umax + u];
  __syncthreads();
  const int nt = (nc + 15) >> 4, ntile = nt * (nt + 1) / 2;
  const int kp = nt * 16;
  const int q0 = (part * ntile) / GBS, q1 = ((part + 1) * ntile) / GBS;   // this part's tiles
  const int wu = __builtin_amdgcn_readfirstlane(w);
  int tI[TPW], tJ[TPW];
  bool tv[TPW];
#pragma unroll
  for (int j = 0; j < TPW; ++j) {
    const int q = q0 + wu + FNW * j;
    tv[j] = q < q1;
    int I = (int)((sqrt(8.0 * q + 1.0) - 1.0) * 0.5);
    while ((I + 1) * (I + 2) / 2 <= q) ++I;
    while (I * (I + 1) / 2 > q) --I;
    tI[j] = I;
    tJ[j] = q - I * (I + 1) / 2;
  }
  // gather map: wave w -> staged row w of a chunk, columns l + 64 c
  int col[NCB];
#pragma unroll
  for (int c = 0; c < NCB; ++c) {
    const int p = l + 64 * c;
    col[c] = p < nc ? s_col[p] : -1;
  }
  double v[NCB];
  auto gather = [&](int t0) {   // unconditional loads from clamped addresses (as k_pg_form)
    const int tt = t0 + w;
    const double* row = lr.panel + (int64_t)ur[tt < U ? tt : 0] * lr.ldp;
#pragma unroll
    for (int c = 0; c < NCB; ++c) {
      const double x = row[col[c] >= 0 ? col[c] : 0];
      v[c] = x * ((tt < U && col[c] >= 0) ? 1.0 : 0.0);
    }
  };
  auto put = [&](double* Sb) {
#pragma unroll
    for (int c = 0; c < NCB; ++c)
      if (l + 64 * c < kp) Sb[w * FPB + l + 64 * c] = v[c];
  };
  f64x4 acc[TPW];
#pragma unroll
  for (int j = 0; j < TPW; ++j) acc[j] = f64x4{0.0, 0.0, 0.0, 0.0};
  auto mma = [&](const double* Sb) {
#pragma unroll
    for (int kk = 0; kk < FKB; kk += 4) {
      const double* r = Sb + (kk + (l >> 4)) * FPB + (l & 15);
#pragma unroll
      for (int j = 0; j < TPW; ++j)
        if (tv[j]) acc[j] = __builtin_amdgcn_mfma_f64_16x16x4f64(r[16 * tI[j]], r[16 * tJ[j]], acc[j], 0, 0, 0);
    }
  };
  double* S0 = S;
  double* S1 = S + FKB * FPB;
  gather(0);
  put(S0);
  __syncthreads();
  int buf = 0;
  for (int t0 = 0; t0 < U; t0 += FKB) {
    const bool more = t0 + FKB < U;
    if (more) gather(t0 + FKB);
    mma(buf ? S1 : S0);
    if (more) put(buf ? S0 : S1);
    __syncthreads();
    buf ^= 1;
  }
  double* Gs = scr + (int64_t)grp * PQ_PG_PASS_SCRATCH;
#pragma unroll
  for (int j = 0; j < TPW; ++j) {
    if (tv[j]) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int gi = 16 * tI[j] + (l >> 4) + 4 * r, gj = 16 * tJ[j] + (l & 15);
        Gs[GB_OFF + (int64_t)gi * KBG + gj] = acc[j][r];
        if (tI[j] != tJ[j]) Gs[GB_OFF + (int64_t)gj * KBG + gi] = acc[j][r];
      }
    }
  }
  if (part == 0) {
    for (int c = t; c < nc; c += FT) Gs[GB_COL + c] = s_col[c];
    if (t == 0) Gs[GB_N] = nc;
    if (t < G && s_on[t]) rec[(int64_t)(d0 + t) * PGR + R_GFORM] = grp + 1;   // the date's group, + 1
  }
}

// ---------------------------------------------------------------------------------------
// solve, one workgroup of NW waves per date: factor P_FF + delta I in LDS, Schur complement
// of the active rows, proximal iterative refinement.  One packed triangle per date in LDS
// bounds the dates per CU, so the waves of a date share its work: wave 0 runs the serial
// 16x16 pivot chain of each diagonal block in registers while the others wait; the panel
// tiles, the trailing MFMA tiles, the triangular-solve updates (four lanes per row), the
// residual's P_FF product (one column slice per wave) and the dot products of the active
// rows are spread over all waves.  Same arithmetic as polish_w.hip's compact mode.
// ---------------------------------------------------------------------------------------
constexpr int WMA = 8;   // active general rows handled by the solve (more: fallback)

__device__ __forceinline__ double sum16(double v) {   // over the 16 lanes of a DPP row
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double sum4(double v) {
  v += __shfl_xor(v, 1, 64);
  v += __shfl_xor(v, 2, 64);
  return v;
}

// Packed lower Cholesky of Lp (k x k) by the NW waves of the workgroup.  16-column panels:
// the 16x16 diagonal block lives in wave 0's registers in the MFMA C layout (lane l: rows
// l>>4 + 4q of column l&15, both triangles); each pivot step reads the pivot, row kk and
// column kk by cross-lane shuffles and updates the trailing block in registers; the block's
// inverse follows in the same chain and REPLACES L11 in Lp (the solves and the panel below
// use only the inverse).  The panel below is L21 = A21 L11^-T (16x16x4 MFMA tiles dealt
// round-robin over the waves).  The trailing update A22 -= L21 L21' is deferred into the
// next block's step: wave 0 updates only the next diagonal tile and goes straight on to its
// pivot chain while the other waves update the remaining tiles, so the serial chain and the
// trailing MFMA work overlap (two barriers per block).  Returns 0, or (first bad column + 1)
// -- uniform over the workgroup.
template <int NW>
__device__ __forceinline__ int b_potrf(double* Lp, int k, int* s_bad, double* prof) {
  const int t = threadIdx.x + loop_zero(), l = t & 63, w = t >> 6;
#ifdef PQ_PROFILE
  long long tp_ = wall_clock64();
#define BP_STAMP(k_)                                                                  \
  do {                                                                                \
    if (t == 0 && prof) { const long long n_ = wall_clock64(); prof[k_] += (double)(n_ - tp_); tp_ = n_; } \
  } while (0)
#else
#define BP_STAMP(k_) do { } while (0)
#endif
  const int cc = l & 15, gg = l >> 4;
  const int j16 = l & 15, kq = l >> 4;
  // tile (I, J) of the trailing block at p0 (rows p0 + 16 I.., columns p0 + 16 J..) minus the
  // product of its rows and columns in panel column block pc
  auto trail_tile = [&](int p0, int I, int J, int pc) {
    const int ri = p0 + 16 * I + j16, cj = p0 + 16 * J + j16;
    f64x4 acc = f64x4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4) {
      const int kc = pc + 4 * s4 + kq;
      const double av = ri < k ? Lp[pk(ri, kc)] : 0.0;
      const double bv = cj < k ? Lp[pk(cj, kc)] : 0.0;
      acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc, 0, 0, 0);
    }
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int gr = p0 + 16 * I + kq + 4 * rr, gc = p0 + 16 * J + j16;
      if (gr < k && gc <= gr) Lp[pk(gr, gc)] -= acc[rr];
    }
  };
  for (int p0 = 0; p0 < k; p0 += 16) {
    const int nb = min(16, k - p0);
    if (p0 > 0) {   // the previous column block's trailing update A22 -= L21 L21'
      const int nt = (k - p0 + 15) >> 4;
      int cnt = 0;
      for (int I = 0; I < nt; ++I)
        for (int J = 0; J <= I; ++J) {
          int owner = 0;   // the diagonal tile (0, 0) feeds wave 0's chain: wave 0's
          if (I > 0 && NW > 1) owner = 1 + (cnt++ % (NW - 1));
          if (owner == w) trail_tile(p0, I, J, p0 - 16);
        }
    }
    if (w == 0) {
      double A[4], Bv[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int r = gg + 4 * q;
        A[q] = (r < nb && cc < nb) ? (cc <= r ? Lp[pk(p0 + r, p0 + cc)] : Lp[pk(p0 + cc, p0 + r)])
                                   : (r == cc ? 1.0 : 0.0);
        Bv[q] = (r == cc) ? 1.0 : 0.0;
      }
      const int bad = wave_chol_inv16(A, Bv);
      if (!bad) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {   // the diagonal block now holds L11^-1
          const int r = gg + 4 * q;
          if (r < nb && cc <= r) Lp[pk(p0 + r, p0 + cc)] = Bv[q];
        }
      }
      if (l == 0) *s_bad = bad;
    }
    __syncthreads();
    if (*s_bad) return p0 + 1;
    BP_STAMP(0);
    const int q0 = p0 + 16;
    const int nt = q0 < k ? (k - q0 + 15) >> 4 : 0;
    for (int i = w; i < nt; i += NW) {   // L21 = A21 L11^-T
      const int r1 = q0 + 16 * i, ri = r1 + j16;
      f64x4 acc = f64x4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) {
        const int kc = 4 * s4 + kq;
        const double av = (ri < k && kc < nb) ? Lp[pk(ri, p0 + kc)] : 0.0;
        const double bv = (kc <= j16 && j16 < nb) ? Lp[pk(p0 + j16, p0 + kc)] : 0.0;
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc, 0, 0, 0);
      }
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int gr = r1 + kq + 4 * rr;
        if (gr < k && j16 < nb) Lp[pk(gr, p0 + j16)] = acc[rr];
      }
    }
    __syncthreads();
    BP_STAMP(1);
  }
#undef BP_STAMP
  return 0;
}

// yo <- L^-1 y (y consumed); diagonal blocks of Lp hold their inverses.  Per 16-row block:
// the 16x16 inverse times the block of y (one product per thread of a 256-thread slice, a
// 16-lane sum), then the rows below subtract their 16-column panel product, four lanes per
// row.  Entered and left with the workgroup synchronised.
template <int NW>
__device__ __forceinline__ void b_fwd(const double* Lp, int k, double* y, double* yo) {
  constexpr int T = 64 * NW;
  const int t = threadIdx.x + loop_zero();
  for (int p0 = 0; p0 < k; p0 += 16) {
    const int nb = min(16, k - p0);
    for (int e = t; e < 256; e += T) {
      const int i = e >> 4, m = e & 15;
      double v = (i < nb && m <= i) ? Lp[pk(p0 + i, p0 + m)] * y[p0 + m] : 0.0;
      v = sum16(v);
      if (m == 0 && i < nb) yo[p0 + i] = v;
    }
    __syncthreads();
    if (p0 + nb < k) {
      const int jq = t & 3;
      for (int r0 = p0 + nb; r0 < k; r0 += T / 4) {
        const int r = r0 + (t >> 2);
        double v = 0.0;
        if (r < k) {
          const double* lr_ = Lp + pk(r, p0) + 4 * jq;
#pragma unroll
          for (int jj = 0; jj < 4; ++jj) v = fma(lr_[jj], yo[p0 + 4 * jq + jj], v);
        }
        v = sum4(v);
        if (r < k && jq == 0) y[r] -= v;
      }
      __syncthreads();
    }
  }
}

// xo <- L^-T y (y consumed), blocks from the last: the transposed 16x16 inverse times the
// block of y, then the columns left of the block subtract the block rows' product.
template <int NW>
__device__ __forceinline__ void b_bwd(const double* Lp, int k, double* y, double* xo) {
  constexpr int T = 64 * NW;
  const int t = threadIdx.x + loop_zero();
  for (int B = ((k + 15) >> 4) - 1; B >= 0; --B) {
    const int p0 = 16 * B, nb = min(16, k - p0);
    for (int e = t; e < 256; e += T) {
      const int i = e >> 4, m = e & 15;
      double v = (i < nb && m >= i && m < nb) ? Lp[pk(p0 + m, p0 + i)] * y[p0 + m] : 0.0;
      v = sum16(v);
      if (m == 0 && i < nb) xo[p0 + i] = v;
    }
    __syncthreads();
    if (p0 > 0) {
      const int jq = t & 3;
      for (int c0 = 0; c0 < p0; c0 += T / 4) {
        const int c = c0 + (t >> 2);
        double v = 0.0;
        if (c < p0) {
#pragma unroll
          for (int jj = 0; jj < 4; ++jj) {
            const int j = 4 * jq + jj;
            if (j < nb) v = fma(Lp[pk(p0 + j, c)], xo[p0 + j], v);
          }
        }
        v = sum4(v);
        if (c < p0 && jq == 0) y[c] -= v;
      }
      __syncthreads();
    }
  }
}

// the solve of date b (k_pg_solve's grid-stride loop body)
template <int KS, int NW>
__device__ __forceinline__ void pg_solve_date(int b, const pq_problem& pb, const pq_state& st, double* rec,
                                              const pq_settings& s, int ldk, int klo, int inner) {
  constexpr int T = 64 * NW;
  constexpr int NP = KS * (KS + 1) / 2;
  __shared__ double Lp[NP];
  __shared__ double xF[KS], rx[KS], sc4[4 * KS];   // sc4: t1 | t2, or the residual's column-slice partials
  __shared__ double Sm[WMA * WMA], lamv[WMA], wl[WMA], rl[WMA], dAv[WMA], red[16];
  __shared__ int s_al[WMA];
  __shared__ int s_map[KS];
  __shared__ int s_flag;
  double* t1 = sc4;
  double* t2 = sc4 + KS;
  double* R = rec + (int64_t)b * PGR;
  if (R[R_STATE] != PQ_PG_PENDING || R[R_W] != 0.0) return;
  const int kb = (int)R[R_KB];   // (the bucket key: R_K may already be lowered by this kernel)
  if (kb <= klo || kb > KS) return;
  int k = kb;
  const int ma = (int)R[R_MA];
  const int t = threadIdx.x, l = t & 63, w = t >> 6;
  if (ma > WMA) {
    if (t == 0) R[R_STATE] = PQ_PG_FALLBACK;
    return;
  }
  const int n = pb.n, ld = pb.ld;
  const double* Cg = pb.Cg ? pb.Cg + (int64_t)b * pb.Cg_stride : nullptr;
  PGWork wk(st, b, ld);
  const double sc = R[R_SC];
  const double delta = s.delta * sc;
  const double* K = st.K + (int64_t)b * st.K_stride;   // P_FF (both triangles), kept for the residuals
#ifdef PQ_PROFILE
  long long t_last_ = wall_clock64();
#define WSTAMP(k_)                                                         \
  do {                                                                     \
    __syncthreads();                                                       \
    if (t == 0) { const long long n_ = wall_clock64(); R[8 + (k_)] += (double)(n_ - t_last_); t_last_ = n_; } \
  } while (0)
#else
#define WSTAMP(k_) do { } while (0)
#endif
  // the K scratch rows / columns of this round's free positions: identity, or (P_FF reused
  // from an earlier round's form) the positions in that free list
  const bool reuse = R[R_REUSE] != 0.0;
  for (int p = t; p < k; p += T) s_map[p] = reuse ? wk.posF[wk.Fl[p]] : p;
  for (int p = t; p < k; p += T) xF[p] = wk.solx[p];
  if (t < ma) {
    s_al[t] = (int)R[R_AL + t];
    lamv[t] = R[R_SOL + t];
    dAv[t] = R[R_DA + t];
  }
  const bool has_box = pb.lb != nullptr;
  const double* lb = has_box ? pb.lb + (int64_t)b * pb.box_stride : nullptr;
  const double* ub = has_box ? pb.ub + (int64_t)b * pb.box_stride : nullptr;
  __syncthreads();
  // inner primal loop: a free variable the solve leaves outside its box is fixed at that bound
  // and the reduced system (a principal submatrix of the same P_FF in K) solved again here,
  // up to `inner` times, instead of one whole round (window passes, checks, setup) per such
  // step; the round's checks then release wrongly fixed variables by their dual sign as before
  for (int it_in = 0;; ++it_in) {
  // lane ids rebuilt from an opaque zero each pass: per-lane addresses derived from them stay
  // inside the pass instead of being hoisted above the loop and held live through it
  const int t = threadIdx.x + loop_zero(), l = t & 63, w = t >> 6;
  {   // packed triangle, flat index (independent loads, 8 per thread in flight)
    const int np_ = k * (k + 1) / 2;
    int r = 0, e0 = 0;   // row of the thread's element: advance incrementally
    for (int eb = 0; eb < np_; eb += T * 8) {
      double v[8];
      int dg = 0;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int e = eb + T * j + t;
        v[j] = 0.0;
        if (e < np_) {
          while (e >= e0 + r + 1) { e0 += r + 1; ++r; }
          const int c = e - e0;
          v[j] = K[(int64_t)s_map[r] * ldk + s_map[c]];
          dg |= (r == c) << j;
        }
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int e = eb + T * j + t;
        if (e < np_) Lp[e] = v[j] + ((dg >> j) & 1 ? delta : 0.0);
      }
    }
  }
  WSTAMP(0);
  __syncthreads();
  if (b_potrf<NW>(Lp, k, &s_flag, R + 16)) {
    if (t == 0) R[R_STATE] = PQ_PG_FALLBACK;
    return;
  }
  WSTAMP(1);
  // U = L^-1 C_aF' (row a of the global U scratch), S = U'U + delta I
  for (int a = 0; a < ma; ++a) {
    const double* cr = Cg + (int64_t)s_al[a] * ld;
    for (int p = t; p < k; p += T) t1[p] = cr[wk.Fl[p]];
    __syncthreads();
    b_fwd<NW>(Lp, k, t1, t2);
    for (int p = t; p < k; p += T) wk.U[(int64_t)a * ld + p] = t2[p];
  }
  __syncthreads();
  for (int e = w; e < ma * ma; e += NW) {
    const int ii = e / ma, jj = e % ma;
    if (jj > ii) continue;
    const double* ui = wk.U + (int64_t)ii * ld;
    const double* uj = wk.U + (int64_t)jj * ld;
    double sum = 0.0;
    for (int p = l; p < k; p += 64) sum += ui[p] * uj[p];
    sum = wave_sum(sum);
    if (l == 0) Sm[ii * WMA + jj] = sum + (ii == jj ? delta : 0.0);
  }
  __syncthreads();
  if (t == 0) {   // tiny Cholesky of S (ma <= 8), one lane
    int sbad = 0;
    for (int c = 0; c < ma && !sbad; ++c) {
      double d = Sm[c * WMA + c];
      for (int m = 0; m < c; ++m) d -= Sm[c * WMA + m] * Sm[c * WMA + m];
      if (!(d > 0.0) || !isfinite(d)) { sbad = 1; break; }
      d = sqrt(d);
      Sm[c * WMA + c] = d;
      for (int r = c + 1; r < ma; ++r) {
        double v = Sm[r * WMA + c];
        for (int m = 0; m < c; ++m) v -= Sm[r * WMA + m] * Sm[c * WMA + m];
        Sm[r * WMA + c] = v / d;
      }
    }
    s_flag = sbad;
  }
  __syncthreads();
  if (s_flag) {
    if (t == 0) R[R_STATE] = PQ_PG_FALLBACK;
    return;
  }
  WSTAMP(2);
  // ---- proximal iterative refinement (polish_w.hip, compact mode) ------------------------
  const int qs = (k + NW - 1) / NW, qa = w * qs, qb = min(k, qa + qs);
  for (int itr = 0; itr < s.refine_iters; ++itr) {
    // rx = rF - P_FF x - C_aF' lam: wave w sums the column slice [qa, qb) of P_FF x (P_FF
    // symmetric in K: row p of the slice is column p, coalesced over lanes); the slices add
    // in a fixed order
    for (int p = l; p < k; p += 64) {
      double sum = 0.0;
#pragma unroll 8
      for (int qq = qa; qq < qb; ++qq) sum = fma(K[(int64_t)s_map[qq] * ldk + s_map[p]], xF[qq], sum);
      sc4[w * KS + p] = sum;
    }
    for (int a = w; a < ma; a += NW) {
      const double* cr = Cg + (int64_t)s_al[a] * ld;
      double sum = 0.0;
      for (int p = l; p < k; p += 64) sum += cr[wk.Fl[p]] * xF[p];
      sum = wave_sum(sum);
      if (l == 0) {
        const double v = dAv[a] - sum;
        rl[a] = fabs(v) <= 1e-14 * (1.0 + fabs(dAv[a]) + fabs(sum)) ? 0.0 : v;
      }
    }
    __syncthreads();
    double rm = 0.0;
    for (int p = t; p < k; p += T) {
      double sum = sc4[p];
#pragma unroll
      for (int j = 1; j < NW; ++j) sum += sc4[j * KS + p];
      double v = wk.rF[p] - sum;
      const int fp = wk.Fl[p];
      for (int a = 0; a < ma; ++a) v -= Cg[(int64_t)s_al[a] * ld + fp] * lamv[a];
      rx[p] = v;
      rm = fmax(rm, fabs(v));
    }
    if (t < ma) rm = fmax(rm, fabs(rl[t]));
    WSTAMP(3);
    if (block_max(rm, red) <= 1e-13 * sc) break;   // (its barriers also order rx / sc4)
    b_fwd<NW>(Lp, k, rx, t2);   // t2 = L^-1 rx (rx consumed)
    for (int a = w; a < ma; a += NW) {   // wl = U' t2 - rl
      const double* ua = wk.U + (int64_t)a * ld;
      double sum = 0.0;
      for (int p = l; p < k; p += 64) sum += ua[p] * t2[p];
      sum = wave_sum(sum);
      if (l == 0) wl[a] = sum - rl[a];
    }
    __syncthreads();
    if (t == 0) {   // dlam = S^-1 wl
      for (int ii = 0; ii < ma; ++ii) {
        double v = wl[ii];
        for (int jj = 0; jj < ii; ++jj) v -= Sm[ii * WMA + jj] * wl[jj];
        wl[ii] = v / Sm[ii * WMA + ii];
      }
      for (int ii = ma - 1; ii >= 0; --ii) {
        double v = wl[ii];
        for (int jj = ii + 1; jj < ma; ++jj) v -= Sm[jj * WMA + ii] * wl[jj];
        wl[ii] = v / Sm[ii * WMA + ii];
      }
    }
    __syncthreads();
    for (int p = t; p < k; p += T) {
      double v = t2[p];
      for (int a = 0; a < ma; ++a) v -= wk.U[(int64_t)a * ld + p] * wl[a];
      t1[p] = v;
    }
    __syncthreads();
    b_bwd<NW>(Lp, k, t1, t2);   // t2 = L^-T (t2 - U dlam)
    for (int p = t; p < k; p += T) xF[p] += t2[p];
    if (t < ma) lamv[t] += wl[t];
    __syncthreads();
    WSTAMP(4);
  }
  // ---- inner primal step: the free variables outside their box, fixed at the bound they
  // cross (k_pg_post's test), the others compacted in order; the reduced rhs and the active
  // rows' rhs take the fixed values (the P_FB columns are K's columns) -------------------------
  if (it_in >= inner || !has_box) break;   // uniform
  {
    int* iw = reinterpret_cast<int*>(sc4 + 2 * KS);   // 4 x KS ints in the free half of sc4
    int* s_m2 = iw;             // kept: K position
    int* s_f2 = iw + KS;        // kept: variable
    int* s_vp = iw + 2 * KS;    // violator: K position
    int* s_vi = iw + 3 * KS;    // violator: 4 variable + bound side (1 lower, 2 upper)
    double* s_vv = rx;          // violator: bound value
    if (w == 0) {
      int nk = 0, nv = 0;
      for (int p0 = 0; p0 < k; p0 += 64) {
        const int p = p0 + l;
        int f = 0, i = 0;
        double v = 0.0;
        if (p < k) {
          i = wk.Fl[p];
          const double xi = xF[p];
          if (!isinf(lb[i]) && xi < lb[i] - 1e-12 * (1.0 + fabs(lb[i]))) { f = 1; v = lb[i]; }
          else if (!isinf(ub[i]) && xi > ub[i] + 1e-12 * (1.0 + fabs(ub[i]))) { f = 2; v = ub[i]; }
        }
        const unsigned long long mv = __ballot(p < k && f != 0);
        const unsigned long long mk = __ballot(p < k && f == 0);
        const unsigned long long below = (1ull << l) - 1ull;
        if (p < k && f != 0) {
          const int j = nv + __popcll(mv & below);
          s_vp[j] = s_map[p];
          s_vi[j] = 4 * i + f;
          s_vv[j] = v;
        } else if (p < k) {
          const int j = nk + __popcll(mk & below);
          s_m2[j] = s_map[p];
          s_f2[j] = i;
          t1[j] = xF[p];
          t2[j] = wk.rF[p];
        }
        nv += __popcll(mv);
        nk += __popcll(mk);
      }
      if (l == 0) s_flag = nv;
    }
    __syncthreads();
    const int nv = s_flag;
#ifdef PQ_PROFILE
    if (t == 0) {   // inner-step counters: solves, steps taken, violators, steps over WMA rows
      R[20] += 1.0;
      R[21] += (nv > 0 && nv < k) ? 1.0 : 0.0;
      R[22] += (nv < k) ? (double)nv : 0.0;
      R[23] += (nv > 0 && nv < k && ma + nv > WMA) ? 1.0 : 0.0;
      R[24] += (double)k;
    }
#endif
    if (nv == 0 || nv == k) break;   // uniform: feasible, or nothing left free (the rounds decide)
    const int k2 = k - nv;
    for (int p = t; p < k2; p += T) {
      const int mp = s_m2[p];
      double r = t2[p];
      for (int j = 0; j < nv; ++j)
        if (s_vv[j] != 0.0) r = fma(-K[(int64_t)mp * ldk + s_vp[j]], s_vv[j], r);
      wk.rF[p] = r;
      wk.Fl[p] = s_f2[p];
      s_map[p] = mp;
      xF[p] = t1[p];
    }
    for (int j = t; j < nv; j += T) {
      const int i = s_vi[j] >> 2;
      wk.fl[i] = s_vi[j] & 3;
      wk.xb[i] = s_vv[j];
    }
    for (int a = w; a < ma; a += NW) {
      const double* cr = Cg + (int64_t)s_al[a] * ld;
      double sum = 0.0;
      for (int j = l; j < nv; j += 64) sum += cr[s_vi[j] >> 2] * s_vv[j];
      sum = wave_sum(sum);
      if (l == 0) dAv[a] -= sum;
    }
    if (t == 0) R[R_K] = k2;
    k = k2;
    __syncthreads();
  }
  }   // inner primal loop
  // ---- expand: xs = x_B off F, x_F on F; general multipliers by row ------------------------
  for (int ii = t; ii < n; ii += T) wk.xs[ii] = wk.xb[ii];
  __syncthreads();
  for (int p = t; p < k; p += T) {
    wk.xs[wk.Fl[p]] = xF[p];
    wk.solx[p] = xF[p];
  }
  if (t < 64) R[R_LAM + t] = 0.0;   // the 64 row slots
  __syncthreads();
  if (t < ma) {
    R[R_LAM + s_al[t]] = lamv[t];
    R[R_SOL + t] = lamv[t];
  }
  WSTAMP(5);
#undef WSTAMP
}

// A resident grid strides over the bucket's list of dates (k_pg_form appends them) -- with one
// workgroup per date, most of them read the record and exited, and each of those still needed
// the full LDS triangle to be dispatched, so with the other buckets filling the CUs they
// trickled in behind the dates
template <int KS, int NW>
__global__ __launch_bounds__(64 * NW) void k_pg_solve(pq_problem pb, pq_state st, double* rec, pq_settings s,
                                                      int ldk, int klo, int inner) {
  const int bk = pg_bucket(KS), cnt = (int)pg_count(rec, bk);
  for (int i = blockIdx.x; i < cnt; i += gridDim.x) {
    pg_solve_date<KS, NW>(pg_listed(rec, bk, i), pb, st, rec, s, ldk, klo, inner);
    __syncthreads();   // (LDS reused by the next date)
  }
}

// ---------------------------------------------------------------------------------------
// solve for the free sets beyond the LDS solve, PG_KMAX < k <= ldk (the tracking windows of
// configs 1/2: 160..220 free assets at n = 494), one 256-thread workgroup per date inside the
// grouped pipeline instead of handing the date to the per-date kernel (pq_polish_w_batched,
// which runs every round's window passes per date as well): P_FF from the window in the
// compact storage (form_pff: MFMA tiles, diagonal tiles in full, off-diagonal tiles
// transposed), its factor in place (wg_cholesky: 64 x 64 MFMA tiles, diagonal-block inverses
// in Dt), the Schur complement of the active rows and the proximal refinement with the
// blocked solves -- polish_w.hip's compact-mode arithmetic.  The round's grouped passes
// (exact P x, checks, scoring) then treat the date like every other.  The factor overwrites
// the lower tiles of K, so the date's next round forms again (R_FORMED = 0).
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ void pg_big_date(int b, const pq_lowrank& lr, const pq_problem& pb, const pq_state& st,
                                            double* rec, const pq_settings& s, int ldk, int kmin) {
  __shared__ __attribute__((aligned(16))) double smem[CHOL_LDS];   // exactly 80 KiB: 2 per CU
  double* R = rec + (int64_t)b * PGR;
  if (R[R_STATE] != PQ_PG_PENDING || R[R_W] != 0.0) return;
  const int k = (int)R[R_K];
  if (k <= kmin || k > ldk) return;
  const int ma = (int)R[R_MA];
  const int t = threadIdx.x, w = wave_id(), l = lane_id();
  if (ma > WMA) {
    if (t == 0) R[R_STATE] = PQ_PG_FALLBACK;
    return;
  }
  const int n = pb.n, ld = pb.ld;
  const double* Cg = pb.Cg ? pb.Cg + (int64_t)b * pb.Cg_stride : nullptr;
  PGWork wk(st, b, ld);
  const double sc = R[R_SC];
  const double delta = s.delta * sc;
  const double ps = pb.p_scale ? pb.p_scale[b] : 1.0;
  const double pd = pb.p_diag ? pb.p_diag[b] : 0.0;
  const double psw = ps * (lr.w_scale ? lr.w_scale[b] : 1.0);
  double* K = st.K + (int64_t)b * st.K_stride;
  double* Dt = st.Dt + (int64_t)b * st.Dt_stride;
  const int nbk = (k + TB - 1) / TB;
  const int kp = nbk * TB;
#ifdef PQ_PROFILE
  long long tb_last_ = wall_clock64();
#define BSTAMP(k_)                                                         \
  do {                                                                     \
    __syncthreads();                                                       \
    if (t == 0) { const long long n_ = wall_clock64(); R[25 + (k_)] += (double)(n_ - tb_last_); tb_last_ = n_; } \
  } while (0)
#else
#define BSTAMP(k_) do { } while (0)
#endif
  // P_FF (both triangles) and the reduced rhs rF = -q_F - p_scale (w_scale Xc'Xc x_B)_F come
  // from k_pg_form<PG_KBIG> on the same stream; FormW reads the diagonal 64 x 64 blocks in
  // full and the other originals from the upper half, which the factor leaves untouched
  const int info = wg_cholesky<false>(FormW{K, ldk, k, delta}, K, ldk, nbk, k, Dt, smem);
  if (t == 0) R[R_FORMED] = 0.0;   // the lower tiles now hold L: no reuse of this P_FF
  BSTAMP(0);
  if (info) {
    if (t == 0) R[R_STATE] = PQ_PG_FALLBACK;
    return;
  }
  // vectors in the (now free) factor workspace
  double* rx = smem;
  double* t1 = smem + PG_KBIG;
  double* dx = smem + 2 * PG_KBIG;
  double* sx = smem + 3 * PG_KBIG;
  double* t64 = smem + 4 * PG_KBIG;
  double* y64p = t64 + TB;
  double* part = y64p + 4 * TB;
  double* U = wk.U;   // rows a of L^-1 C_aF' (pitch ld >= kp)
  double* red = part + 4 * TB;
  double* Sm = red + 16;
  double* lamv = Sm + WMA * WMA;
  double* dAv = lamv + WMA;
  double* rl = dAv + WMA;
  double* wl = rl + WMA;
  int* s_al = reinterpret_cast<int*>(wl + WMA);
  constexpr int YC_OFF = 2048;   // the residual's per-wave column partials (PW x PG_KBIG)
  static_assert(5 * PG_KBIG + 6 * TB + 16 + WMA * WMA + 5 * WMA + WMA <= YC_OFF &&
                YC_OFF + PW * PG_KBIG <= CHOL_LDS, "k_pg_big LDS layout");
  __syncthreads();   // the factor is done with smem
  if (t < ma) {
    s_al[t] = (int)R[R_AL + t];
    lamv[t] = R[R_SOL + t];
    dAv[t] = R[R_DA + t];
  }
  __syncthreads();
  // ---- U = L^-1 C_aF', S = U'U + delta I (tiny Cholesky, one thread) -------------------------
  // With one active row (the budget: the usual case) U's forward solve is deferred into the
  // first refinement step's, as the second right-hand side of one pass over L and Dt
  const bool defer_u = ma == 1;   // (uniform)
  constexpr int CR_OFF = YC_OFF + PW * PG_KBIG, U1_OFF = CR_OFF + PG_KBIG, T2_OFF = U1_OFF + PG_KBIG,
                Y2_OFF = T2_OFF + 2 * TB;
  static_assert(Y2_OFF + 8 * TB <= CHOL_LDS, "k_pg_big LDS layout (two-right-hand-side solve)");
  auto factor_s = [&]() -> bool {   // S = U'U + delta I and its Cholesky; true: not PD (uniform)
    for (int e = w; e < ma * ma; e += PW) {
      const int ii = e / ma, jj = e % ma;
      if (jj > ii) continue;
      double sum = 0.0;
      for (int p = l; p < k; p += 64) sum += U[(int64_t)ii * ld + p] * U[(int64_t)jj * ld + p];
      sum = wave_sum(sum);
      if (l == 0) Sm[ii * WMA + jj] = sum + (ii == jj ? delta : 0.0);
    }
    __syncthreads();
    if (t == 0) {
      int sbad = 0;
      for (int c = 0; c < ma && !sbad; ++c) {
        double d = Sm[c * WMA + c];
        for (int m = 0; m < c; ++m) d -= Sm[c * WMA + m] * Sm[c * WMA + m];
        if (!(d > 0.0) || !isfinite(d)) { sbad = 1; break; }
        d = sqrt(d);
        Sm[c * WMA + c] = d;
        for (int r = c + 1; r < ma; ++r) {
          double v = Sm[r * WMA + c];
          for (int m = 0; m < c; ++m) v -= Sm[r * WMA + m] * Sm[c * WMA + m];
          Sm[r * WMA + c] = v / d;
        }
      }
      red[0] = sbad;
    }
    __syncthreads();
    return red[0] != 0.0;
  };
  if (!defer_u) {
    for (int a = 0; a < ma; ++a) {
      const double* cr = Cg + (int64_t)s_al[a] * ld;
      for (int p = t; p < kp; p += PT) rx[p] = p < k ? cr[wk.Fl[p]] : 0.0;
      __syncthreads();
      fwd_solve(K, ldk, Dt, nbk, rx, t1, t64, y64p);
      for (int p = t; p < kp; p += PT) U[(int64_t)a * ld + p] = t1[p];
      __syncthreads();
    }
    if (factor_s()) {
      if (t == 0) R[R_STATE] = PQ_PG_FALLBACK;
      return;
    }
  }
  for (int p = t; p < kp; p += PT) sx[p] = p < k ? wk.solx[p] : 0.0;
  __syncthreads();
  BSTAMP(1);
  // ---- proximal iterative refinement (polish_w.hip, compact mode) ------------------------------
  for (int itr = 0; itr < s.refine_iters; ++itr) {
    {   // rx = rF - P_FF x - C_aF' lam.  P_FF x in one coalesced pass over the stored originals
        // (the diagonal 64-blocks in full, the off-diagonal blocks in the upper half): row i's
        // entries give (P x)_i by a wave sum, and its upper off-diagonal entries also add
        // K[i][j] x_i to (P x)_j in lane registers (column 64 c + lane), combined over the waves
        // in LDS -- instead of reading the lower off-diagonal originals down the columns of the
        // upper half (64 cache lines per load: 103 of 344 us per date-round, r05G_diag_union.log)
      double* ycol = smem + YC_OFF;
      double yc[PG_KBIG / 64];
#pragma unroll
      for (int c = 0; c < PG_KBIG / 64; ++c) yc[c] = 0.0;
      // RU rows per wave in flight: all their loads unconditional from clamped addresses (a
      // load under a branch makes the compiler wait for every outstanding load at the join),
      // the entries outside the stored part zeroed by a factor after the load
      constexpr int RU = 4;
      constexpr int NCB = PG_KBIG / 64;
      for (int i0 = w; i0 < k; i0 += RU * PW) {
        double sacc[RU], xv[RU], kv[RU][NCB];
#pragma unroll
        for (int u = 0; u < RU; ++u) {
          const int i = i0 + u * PW, ic = i < k ? i : k - 1;
          xv[u] = sx[ic];
          const double* Ki = K + (int64_t)ic * ldk;
#pragma unroll
          for (int c = 0; c < NCB; ++c) {
            const int j = 64 * c + l;
            kv[u][c] = Ki[j < k ? j : ic];
          }
        }
#pragma unroll
        for (int u = 0; u < RU; ++u) {
          const int i = i0 + u * PW, bi = i >> 6;
          const bool iv = i < k;
          sacc[u] = 0.0;
#pragma unroll
          for (int c = 0; c < NCB; ++c) {
            const int j = 64 * c + l;
            const double v = kv[u][c] * ((iv && c >= bi && j < k) ? 1.0 : 0.0);
            sacc[u] = fma(v, sx[j < kp ? j : 0], sacc[u]);
            yc[c] = fma(v * (c > bi ? 1.0 : 0.0), xv[u], yc[c]);
          }
        }
#pragma unroll
        for (int u = 0; u < RU; ++u) {
          const double v = wave_sum(sacc[u]);
          if (l == 0 && i0 + u * PW < k) rx[i0 + u * PW] = v;
        }
      }
#pragma unroll
      for (int c = 0; c < PG_KBIG / 64; ++c) ycol[w * PG_KBIG + 64 * c + l] = yc[c];
      __syncthreads();
      for (int p = t; p < kp; p += PT) {
        double v = 0.0;
        if (p < k) {
          double y = rx[p];
#pragma unroll
          for (int ww = 0; ww < PW; ++ww) y += ycol[ww * PG_KBIG + p];
          v = wk.rF[p] - y;
          for (int a = 0; a < ma; ++a) v -= Cg[(int64_t)s_al[a] * ld + wk.Fl[p]] * lamv[a];
        }
        rx[p] = v;
      }
    }
    for (int a = w; a < ma; a += PW) {   // rl = dA - C_aF x
      const double* c = Cg + (int64_t)s_al[a] * ld;
      double sum = 0.0;
      for (int p = l; p < k; p += 64) sum += c[wk.Fl[p]] * sx[p];
      sum = wave_sum(sum);
      if (l == 0) {
        const double v = dAv[a] - sum;
        rl[a] = fabs(v) <= 1e-14 * (1.0 + fabs(dAv[a]) + fabs(sum)) ? 0.0 : v;
      }
    }
    __syncthreads();
    double rm = 0.0;
    for (int p = t; p < k; p += PT) rm = fmax(rm, fabs(rx[p]));
    if (t < ma) rm = fmax(rm, fabs(rl[t]));
    BSTAMP(2);
    // (with defer_u this break can come before U and S exist: the starting point then already
    // solves the regularised KKT system to 1e-13 of the problem scale and is kept as it is --
    // no step is taken, so S's Cholesky, which only guards the step, is not needed)
    if (block_max(rm, red) <= 1e-13 * sc) break;
    if (defer_u && itr == 0) {   // t1 = L^-1 rx and U = L^-1 C_aF' in one pass, then S
      double* cr2 = smem + CR_OFF;
      double* u1 = smem + U1_OFF;
      const double* cr = Cg + (int64_t)s_al[0] * ld;
      for (int p = t; p < kp; p += PT) cr2[p] = p < k ? cr[wk.Fl[p]] : 0.0;
      __syncthreads();
      fwd_solve2(K, ldk, Dt, nbk, rx, cr2, t1, u1, smem + T2_OFF, smem + Y2_OFF);
      for (int p = t; p < kp; p += PT) U[p] = u1[p];
      __syncthreads();
      if (factor_s()) {
        if (t == 0) R[R_STATE] = PQ_PG_FALLBACK;
        return;
      }
    } else {
      fwd_solve(K, ldk, Dt, nbk, rx, t1, t64, y64p);
    }
    for (int a = w; a < ma; a += PW) {   // wl = U' t1 - rl
      double sum = 0.0;
      for (int p = l; p < k; p += 64) sum += U[(int64_t)a * ld + p] * t1[p];
      sum = wave_sum(sum);
      if (l == 0) wl[a] = sum - rl[a];
    }
    __syncthreads();
    if (t == 0) {   // dlam = S^-1 wl
      for (int ii = 0; ii < ma; ++ii) {
        double v = wl[ii];
        for (int jj = 0; jj < ii; ++jj) v -= Sm[ii * WMA + jj] * wl[jj];
        wl[ii] = v / Sm[ii * WMA + ii];
      }
      for (int ii = ma - 1; ii >= 0; --ii) {
        double v = wl[ii];
        for (int jj = ii + 1; jj < ma; ++jj) v -= Sm[jj * WMA + ii] * wl[jj];
        wl[ii] = v / Sm[ii * WMA + ii];
      }
    }
    __syncthreads();
    for (int p = t; p < kp; p += PT) {   // t1 <- t1 - U dlam ; dx = L^-T t1
      double v = t1[p];
      for (int a = 0; a < ma; ++a) v -= U[(int64_t)a * ld + p] * wl[a];
      t1[p] = v;
    }
    __syncthreads();
    bwd_solve(K, ldk, Dt, nbk, t1, dx, t64, part, y64p);
    for (int p = t; p < k; p += PT) sx[p] += dx[p];
    if (t < ma) lamv[t] += wl[t];
    __syncthreads();
    BSTAMP(3);
  }
  // ---- expand: xs = x_B off F, x_F on F; general multipliers by row ------------------------
  for (int ii = t; ii < n; ii += PT) wk.xs[ii] = wk.xb[ii];
  __syncthreads();
  for (int p = t; p < k; p += PT) {
    wk.xs[wk.Fl[p]] = sx[p];
    wk.solx[p] = sx[p];
  }
  if (t < 64) R[R_LAM + t] = 0.0;
  __syncthreads();
  if (t < ma) {
    R[R_LAM + s_al[t]] = lamv[t];
    R[R_SOL + t] = lamv[t];
  }
  BSTAMP(4);
  if (t == 0) {
    R[30] += 1.0;
    R[31] += (double)k;
  }
#undef BSTAMP
}

// a resident grid striding over the large free sets' list (k_pg_form<PG_KBIG>'s)
__global__ __launch_bounds__(PT, 2) void k_pg_big(pq_lowrank lr, pq_problem pb, pq_state st, double* rec,
                                                 pq_settings s, int ldk, int kmin) {
  const int cnt = (int)pg_count(rec, PG_BIGB);
  for (int i = blockIdx.x; i < cnt; i += gridDim.x) {
    pg_big_date(pg_listed(rec, PG_BIGB, i), lr, pb, st, rec, s, ldk, kmin);
    __syncthreads();   // (LDS reused by the next date)
  }
}

// ---------------------------------------------------------------------------------------
// grouped window passes: MODE 0 -> pxb = w_scale Xc'Xc x_B (dates with x_B != 0);
// MODE 1 -> exact P x, gradient, active-set checks, final scoring of accepted dates
// ---------------------------------------------------------------------------------------
constexpr int QT = 512;
constexpr int QNW = QT / 64;
constexpr int QG = 16;     // dates per group (MFMA N)
constexpr int QU = 320;    // union rows per group

__device__ __forceinline__ double hsum32(double v) {
#pragma unroll
  for (int o = 16; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double hmax32(double v) {
#pragma unroll
  for (int o = 16; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
  return v;
}

// The two window passes of a group run split over PQ_PG_SPLIT workgroups each (the union
// rows' columns divided between them), so a late round with few pending groups is not one
// latency-bound workgroup per group:
//   k_pg_passA  (group, column slice)  partial W = X_union[:, slice] V[slice] and mu.V partials
//   k_pg_passB  (group, column slice)  W = sum of the partials (fixed order: deterministic),
//                                      Ut = window-masked W - mu.V, X~[slice] = X_union[:, slice]' Ut
//   k_pg_post   (group)                the per-date post-processing on the complete X~
constexpr int QS = 4;      // workgroups per group and pass
constexpr int QCOL = 2048; // pass A: column slices up to this long take the sparse (compacted) form

struct PassGroup {
  int grp, part, d0, G, U;
};

template <int MODE>
__device__ __forceinline__ bool pass_setup(const PassGroup& pg, const pq_lowrank& lr, const double* rec,
                                           const int32_t* uoff, int* g_on, int* g_T, int* g_off, int* s_any) {
  const int t = threadIdx.x;
  if (t < QG) {
    int on = 0;
    if (t < pg.G) {
      const double* R = rec + (int64_t)(pg.d0 + t) * PGR;
      on = R[R_STATE] == PQ_PG_PENDING && (MODE == 1 || R[R_NZB] != 0.0);
      g_T[t] = lr.tlen[pg.d0 + t];
      g_off[t] = uoff[pg.d0 + t];
    }
    g_on[t] = on;
  }
  __syncthreads();
  if (t == 0) {
    int any = 0;
    for (int g = 0; g < pg.G; ++g) any |= g_on[g];
    *s_any = any;
  }
  __syncthreads();
  return *s_any != 0;
}

__device__ __forceinline__ PassGroup pass_group(const int32_t* gdates, const int32_t* ucnt_all) {
  const int id = xcd_slot(blockIdx.x, gridDim.x);   // the slices of a group on one XCD
  PassGroup pg;
  pg.grp = id / QS;
  pg.part = id % QS;
  pg.d0 = gdates[pg.grp];
  pg.G = gdates[pg.grp + 1] - pg.d0;
  pg.U = ucnt_all[pg.grp];
  return pg;
}

// scratch per group: QS partial W images ((QU + 4) x QG) + QS x QG mu.V partials + QG sums
constexpr int64_t QSCR = (int64_t)QS * (QU + 4) * QG + QS * QG + QG;

template <int MODE>
__global__ __launch_bounds__(QT) void k_pg_passA(pq_lowrank lr, pq_problem pb, pq_state st, const double* rec,
                                                 const int32_t* gdates, const int32_t* urows_all,
                                                 const int32_t* ucnt_all, const int32_t* uoff, int umax,
                                                 double* scr) {
  __shared__ int s_urow[QU];
  __shared__ int g_on[QG], g_T[QG], g_off[QG];
  __shared__ int s_any;
  __shared__ int s_col[QCOL], s_wcnt[QNW], s_ncol;
  const PassGroup pg = pass_group(gdates, ucnt_all);
  const int U = pg.U, G = pg.G, d0 = pg.d0;
  const int t = threadIdx.x, w = wave_id(), l = lane_id();
  const int n = pb.n, ld = pb.ld;
  for (int u = t; u < QU; u += QT) s_urow[u] = u < U ? urows_all[(int64_t)pg.grp * umax + u] : 0;
  if (t == 0) s_ncol = 0;
  if (!pass_setup<MODE>(pg, lr, rec, uoff, g_on, g_T, g_off, &s_any)) return;
  const int per = ((n + QS - 1) / QS + 7) & ~7;
  const int k_lo = pg.part * per, k_hi = min(n, k_lo + per);
  double* Wp = scr + pg.grp * QSCR + (int64_t)pg.part * (QU + 4) * QG;
  double* Mp = scr + pg.grp * QSCR + (int64_t)QS * (QU + 4) * QG + pg.part * QG;
  // mu . v partial of every participating date (half-wave per date)
  const int hg = t >> 5, hl = t & 31;
  if (hg < G && g_on[hg]) {
    PGWork wk(st, d0 + hg, ld);
    const double* v = MODE == 0 ? wk.xb : wk.xs;
    const double* mu = lr.mu ? lr.mu + (int64_t)(d0 + hg) * lr.mu_stride : nullptr;
    double a = 0.0;
    if (mu)
      for (int i = k_lo + hl; i < k_hi; i += 32) a = fma(mu[i], v[i], a);
    a = hsum32(a);
    if (hl == 0) Mp[hg] = a;
  } else if (hg < QG && hl == 0) {
    Mp[hg] = 0.0;
  }
  // partial W (U x 16) = X_union[:, k_lo:k_hi] V[k_lo:k_hi]
  const int ntile = (U + 15) >> 4;
  const int kq = l >> 4, m = l & 15;
  const double* Vp = nullptr;
  if (m < G && g_on[m]) {
    PGWork wk(st, d0 + m, ld);
    Vp = MODE == 0 ? wk.xb : wk.xs;
  }
  f64x4 c[3];
  const double* arow[3];
  bool tv[3], aval[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    c[j] = f64x4{0.0, 0.0, 0.0, 0.0};
    const int u = (w + QNW * j) * 16 + m;
    tv[j] = w + QNW * j < ntile;
    aval[j] = u < U;
    arow[j] = lr.panel + (int64_t)s_urow[u < QU ? u : 0] * lr.ldp;
  }
  if (k_hi - k_lo <= QCOL) {
    // V is sparse (the new point is zero on the variables fixed at a zero bound: ~n - |F| of
    // them for long-only problems): only the slice's columns where some participating date
    // of the group is nonzero enter the product, compacted in column order (ballot + wave
    // prefix: deterministic) -- the union rows are then read at those columns only
    for (int cb = k_lo; cb < k_hi; cb += QT) {
      const int i = cb + t;
      bool nz = false;
      {   // every date's entry loaded at once (clamped, unconditional), then combined
        const int ic = i < k_hi ? i : k_lo;
        double v[QG];
#pragma unroll
        for (int g = 0; g < QG; ++g) {
          PGWork wg(st, d0 + (g < G ? g : 0), ld);
          v[g] = (MODE == 0 ? wg.xb : wg.xs)[ic];
        }
#pragma unroll
        for (int g = 0; g < QG; ++g) nz |= g < G && g_on[g] && v[g] != 0.0;
        nz = nz && i < k_hi;
      }
      const unsigned long long bal = __ballot(nz);
      if (l == 0) s_wcnt[w] = __popcll(bal);
      __syncthreads();
      int off = s_ncol;
      for (int ww = 0; ww < w; ++ww) off += s_wcnt[ww];
      if (nz) s_col[off + __popcll(bal & ((1ull << l) - 1ull))] = i;
      __syncthreads();
      if (t == 0) {
        int tot = 0;
        for (int ww = 0; ww < QNW; ++ww) tot += s_wcnt[ww];
        s_ncol += tot;
      }
      __syncthreads();
    }
    // unconditional loads from clamped addresses, V scaled to zero past the column list and
    // for dates not taking part, MFMAs on every tile (rows past U and tiles past ntile give
    // output rows the window mask of pass B drops): no branch and no select on a loaded
    // register, which made the compiler wait for every outstanding load at each step.  Four
    // column steps' loads are issued before their MFMAs
    const int ncol = s_ncol;
    const double* Vq = Vp ? Vp : lr.panel;
    for (int k0 = 0; k0 < ncol; k0 += 16) {
      double av[4][3], bv[4];
#pragma unroll
      for (int h = 0; h < 4; ++h) {
        const int kk = k0 + 4 * h + kq;
        const bool kin = kk < ncol;
        const int col = s_col[kin ? kk : 0];
        bv[h] = Vq[col] * ((Vp && kin) ? 1.0 : 0.0);
#pragma unroll
        for (int j = 0; j < 3; ++j) av[h][j] = arow[j][col];
      }
#pragma unroll
      for (int h = 0; h < 4; ++h)
#pragma unroll
        for (int j = 0; j < 3; ++j) c[j] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[h][j], bv[h], c[j], 0, 0, 0);
    }
  } else {
    const double* Vq = Vp ? Vp : lr.panel;
    for (int k0 = k_lo; k0 < k_hi; k0 += 16) {
      double2 av[2][3];
      double bx[2], by[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int kk = k0 + 8 * h + 2 * kq;
        const bool kin = kk + 1 < k_hi;   // slice ends and n are even
        const int kc = kin ? kk : k_lo;
        const double sb = (Vp && kin) ? 1.0 : 0.0;
        const double2 bl = *reinterpret_cast<const double2*>(Vq + kc);
        bx[h] = bl.x * sb;
        by[h] = bl.y * sb;
#pragma unroll
        for (int j = 0; j < 3; ++j) av[h][j] = *reinterpret_cast<const double2*>(arow[j] + kc);
      }
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          c[j] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[h][j].x, bx[h], c[j], 0, 0, 0);
          c[j] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[h][j].y, by[h], c[j], 0, 0, 0);
        }
    }
  }
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int tile = w + QNW * j;
    if (tv[j]) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int u = tile * 16 + kq + 4 * r;
        if (u < QU) Wp[u * QG + m] = c[j][r];
      }
    }
  }
}

template <int MODE>
__global__ __launch_bounds__(QT) void k_pg_passB(pq_lowrank lr, pq_problem pb, pq_state st, const double* rec,
                                                 const int32_t* gdates, const int32_t* urows_all,
                                                 const int32_t* ucnt_all, const int32_t* uoff, int umax,
                                                 double* scr) {
  __shared__ __attribute__((aligned(16))) double WU[(QU + 16) * QG];   // (rows >= ntile 16: zero)
  __shared__ int s_urow[QU];
  __shared__ int g_on[QG], g_T[QG], g_off[QG];
  __shared__ double g_mux[QG];
  __shared__ int s_any;
  const PassGroup pg = pass_group(gdates, ucnt_all);
  const int U = pg.U, G = pg.G, d0 = pg.d0;
  const int t = threadIdx.x, w = wave_id(), l = lane_id();
  const int n = pb.n, ld = pb.ld;
  for (int u = t; u < QU; u += QT) s_urow[u] = u < U ? urows_all[(int64_t)pg.grp * umax + u] : 0;
  if (!pass_setup<MODE>(pg, lr, rec, uoff, g_on, g_T, g_off, &s_any)) return;
  const double* S = scr + pg.grp * QSCR;
  const double* Mp = S + (int64_t)QS * (QU + 4) * QG;
  if (t < QG) {
    double a = 0.0;
    for (int q = 0; q < QS; ++q) a += Mp[q * QG + t];
    g_mux[t] = a;
  }
  __syncthreads();
  // Ut = sum of the partial W images (fixed order), masked to each date's own window rows
  const int ntile = (U + 15) >> 4;
  for (int e = t; e < (QU + 16) * QG; e += QT) {
    const int u = e / QG, m = e % QG;
    double v = 0.0;
    if (u < ntile * 16) {
      double a = 0.0;
      for (int q = 0; q < QS; ++q) a += S[(int64_t)q * (QU + 4) * QG + e];
      const bool inw = m < G && g_on[m] && u >= g_off[m] && u < g_off[m] + g_T[m];
      v = inw ? a - g_mux[m] : 0.0;
    }
    WU[e] = v;
  }
  __syncthreads();
  if (pg.part == 0 && t < QG) {   // sum of Ut per date (the centring term of the post)
    double a = 0.0;
    for (int u = 0; u < U; ++u) a += WU[u * QG + t];
    scr[pg.grp * QSCR + (int64_t)QS * (QU + 4) * QG + QS * QG + t] = a;
  }
  // X~ (slice x 16) = X_union[:, slice]' Ut -> raw into the date's target vector
  const int kq = l >> 4, m = l & 15;
  const int Uk = (U + 3) & ~3;
  double* dst = nullptr;
  if (m < G && g_on[m]) {
    PGWork wk(st, d0 + m, ld);
    dst = MODE == 0 ? wk.pxb : wk.g;
  }
  const int nch = (n + 31) / 32;
  const int cper = (nch + QS - 1) / QS;
  const int p_lo = pg.part * cper, p_hi = min(nch, p_lo + cper);
  for (int p = p_lo + w; p < p_hi; p += QNW) {
    const int col = p * 32 + 2 * m;
    const bool cin = col < n;
    f64x4 ce = f64x4{0.0, 0.0, 0.0, 0.0}, co = f64x4{0.0, 0.0, 0.0, 0.0};
    // unconditional loads (rows past U meet a zero Ut, columns past n are never stored), four
    // union-row steps' loads issued before their MFMAs
    const int colc = cin ? col : 0;
    for (int u0 = 0; u0 < Uk; u0 += 16) {
      double2 a[4];
#pragma unroll
      for (int h = 0; h < 4; ++h) {
        const int u = u0 + 4 * h + kq;
        a[h] = *reinterpret_cast<const double2*>(lr.panel + (int64_t)s_urow[u < U ? u : 0] * lr.ldp + colc);
      }
#pragma unroll
      for (int h = 0; h < 4; ++h) {
        const double bv = WU[(u0 + 4 * h + kq) * QG + m];   // (rows to Uk + 15: zero-filled)
        ce = __builtin_amdgcn_mfma_f64_16x16x4f64(a[h].x, bv, ce, 0, 0, 0);
        co = __builtin_amdgcn_mfma_f64_16x16x4f64(a[h].y, bv, co, 0, 0, 0);
      }
    }
    if (dst) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = p * 32 + 2 * (kq + 4 * r);
        if (i < n) dst[i] = ce[r];
        if (i + 1 < n) dst[i + 1] = co[r];
      }
    }
  }
}

// one 256-thread workgroup per pending date (a date's n-vectors spread over its threads: the
// per-date passes are load-latency bound, 4 loads per thread and vector at n = 1000 instead
// of 16 with one wave)
constexpr int PPT = 256;
// sum over j = hl, hl + PPT, ... < n of a[j] b[j], in that order: four steps' loads issued
// together (clamped, unconditional), so a long row (n = 5000: 20 steps) is 5 load round trips
// instead of 20 -- the same sum
__device__ __forceinline__ double row_dot4(const double* a, const double* b, int n, int hl) {
  double sum = 0.0;
  for (int j0 = hl; j0 < n; j0 += 4 * PPT) {
    double av[4], bv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int j = j0 + u * PPT, jc = j < n ? j : 0;
      av[u] = a[jc];
      bv[u] = b[jc];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (j0 + u * PPT < n) sum += av[u] * bv[u];
  }
  return sum;
}
template <int MODE>
__global__ __launch_bounds__(PPT) void k_pg_post(pq_lowrank lr, pq_problem pb, pq_state st, double* rec,
                                                pq_settings s, const int32_t* gdates, int ngroups,
                                                const double* scr) {
  const int b = blockIdx.x;
  double* R = rec + (int64_t)b * PGR;
  if (MODE == 0 && b == 0 && threadIdx.x < PG_NBUCKET)   // this round's solve-bucket lists start empty
    reinterpret_cast<unsigned long long*>(rec + R_CNT)[threadIdx.x] = 0ull;
  if (!(R[R_STATE] == PQ_PG_PENDING && (MODE == 1 || R[R_NZB] != 0.0))) return;
  int lo = 0, hi = ngroups;   // group of date b: gdates[grp] <= b < gdates[grp + 1]
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (gdates[mid] <= b) lo = mid; else hi = mid;
  }
  const int grp = lo, hg = b - gdates[grp];
  __shared__ double red[16];
  const int hl = threadIdx.x;
  const int n = pb.n, ld = pb.ld, mg = pb.mg;
  PGWork wk(st, b, ld);
  const double* mu = lr.mu ? lr.mu + (int64_t)b * lr.mu_stride : nullptr;
  const double su = scr[(int64_t)grp * QSCR + (int64_t)QS * (QU + 4) * QG + QS * QG + hg];
  const double wsc = lr.w_scale ? lr.w_scale[b] : 1.0;
  if (MODE == 0) {
    for (int i = hl; i < n; i += PPT) wk.pxb[i] = wsc * (wk.pxb[i] - (mu ? mu[i] * su : 0.0));
    return;
  }
  const double ps = pb.p_scale ? pb.p_scale[b] : 1.0;
  const double pd = pb.p_diag ? pb.p_diag[b] : 0.0;
  const double* q = pb.q + (int64_t)b * pb.q_stride;
  const double* Cg = pb.Cg ? pb.Cg + (int64_t)b * pb.Cg_stride : nullptr;
  const double* lg = pb.lg ? pb.lg + (int64_t)b * pb.g_stride : nullptr;
  const double* ug = pb.ug ? pb.ug + (int64_t)b * pb.g_stride : nullptr;
  const bool has_box = pb.lb != nullptr;
  const double* lb = has_box ? pb.lb + (int64_t)b * pb.box_stride : nullptr;
  const double* ub = has_box ? pb.ub + (int64_t)b * pb.box_stride : nullptr;
  const double sc = R[R_SC];
  const double dtol = s.dual_tol * sc;
  const double ptol = 1e-12;
  const double soft = s.polish_release_rel > 0.0 ? s.polish_release_rel * sc : 0.0;
  // vertex (k == 0, set up with at most one active equality row r0): its multiplier is the
  // middle of the interval in which every bound variable's multiplier has the right sign,
  //   at lb: g0_i + lam c_i >= 0,  at ub: g0_i + lam c_i <= 0   (g0 = P x + q)
  // (an empty interval leaves violations for the checks below, as any wrong active set)
  const bool vtx = R[R_K] == 0.0 && R[R_MA] == 1.0;
  const int r0 = vtx ? (int)R[R_AL] : -1;
  double lam0 = 0.0;
  if (vtx) {
    const double* c0 = Cg + (int64_t)r0 * ld;
    double lo = -INFINITY, hi = INFINITY;
    for (int i = hl; i < n; i += PPT) {
      const int f = wk.fl[i];
      const double c = c0[i];
      if (f == 0 || c == 0.0 || (has_box && lb[i] == ub[i])) continue;
      const double pxi = ps * (wsc * (wk.g[i] - (mu ? mu[i] * su : 0.0))) + pd * wk.xs[i];
      const double bnd = -(pxi + q[i]) / c;
      if ((f == 1) == (c > 0.0)) lo = fmax(lo, bnd);
      else hi = fmin(hi, bnd);
    }
    lo = block_max(lo, red);
    hi = -block_max(-hi, red);
    lam0 = (isfinite(lo) && isfinite(hi)) ? 0.5 * (lo + hi) : (isfinite(lo) ? lo : (isfinite(hi) ? hi : 0.0));
  }
  auto lamof = [&](int r) -> double { return r == r0 ? lam0 : R[R_LAM + r]; };
  // exact P x and gradient g = P x + q + Cg' lam; box checks
  int bad = 0;
  // four of the thread's elements per step, every load issued first (clamped, unconditional):
  // the stores of one element would otherwise order the next element's loads behind them
  const double lam_r0 = mg > 0 ? lamof(0) : 0.0;
  for (int i0 = hl; i0 < n; i0 += 4 * PPT) {
    double xv[4], gv[4], mv4[4], qv[4], c0[4], lbv[4], ubv[4];
    int fv[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int i = i0 + j * PPT, ic = i < n ? i : 0;
      xv[j] = wk.xs[ic];
      gv[j] = wk.g[ic];
      mv4[j] = mu ? mu[ic] : 0.0;
      qv[j] = q[ic];
      c0[j] = mg > 0 ? Cg[ic] : 0.0;
      fv[j] = wk.fl[ic];
      lbv[j] = has_box ? lb[ic] : 0.0;
      ubv[j] = has_box ? ub[ic] : 0.0;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int i = i0 + j * PPT;
      if (i >= n) continue;
      const double xi = xv[j];
      const double pxi = ps * (wsc * (gv[j] - mv4[j] * su)) + pd * xi;
      double gi = pxi + qv[j] + c0[j] * lam_r0;
      for (int r = 1; r < mg; ++r) gi += Cg[(int64_t)r * ld + i] * lamof(r);
      wk.Px[i] = pxi;
      wk.g[i] = gi;
      const int f = fv[j];
      const double lbi = lbv[j], ubi = ubv[j];
      if (f == 0 && has_box) {
        if (!isinf(lbi) && xi < lbi - ptol * (1.0 + fabs(lbi))) { wk.fl[i] = 1; bad = 1; }
        else if (!isinf(ubi) && xi > ubi + ptol * (1.0 + fabs(ubi))) { wk.fl[i] = 2; bad = 1; }
      } else if (f == 1 && lbi != ubi && -gi > dtol) { wk.fl[i] = 0; bad = 1; }
      else if (f == 2 && -gi < -dtol) { wk.fl[i] = 0; bad = 1; }
      else if (soft > 0.0 && f == 1 && lbi != ubi && -gi > dtol - soft) wk.fl[i] = 5;   // near the sign
      else if (soft > 0.0 && f == 2 && -gi < soft - dtol) wk.fl[i] = 6;                  // (resolved below)
    }
  }
  // general rows: Cg x, activity checks (lane 0 decides, as the reference kernel's lane 0)
  for (int r = 0; r < mg; ++r) {
    const double* cr = Cg + (int64_t)r * ld;
    double sum = row_dot4(cr, wk.xs, n, hl);
    sum = block_sum(sum, red);
    // a vertex whose bound variables overshoot its equality row (the round before fixed
    // several free variables at their upper bounds at once, e.g. two weights past 1 under a
    // budget of 1): no free variable can restore the row, so the variables at a bound that
    // push it past its value are released (uniform: every thread holds the sum)
    if (vtx && r == r0 && has_box && sum > ug[r] + ptol * (1.0 + fabs(ug[r]))) {
      for (int i = hl; i < n; i += PPT) {
        const int f = wk.fl[i];
        if ((f == 2 && cr[i] > 0.0) || (f == 1 && cr[i] < 0.0 && lb[i] != ub[i])) wk.fl[i] = 0;
      }
      bad = 1;
    }
    if (hl == 0) {
      if (lg[r] != ug[r]) {
        const int a = (int)R[R_ACT + r];
        const double lam = lamof(r);
        if (a == 0 && sum > ug[r] + ptol * (1.0 + fabs(ug[r]))) { R[R_ACT + r] = 2; bad = 1; }
        else if (a == 0 && sum < lg[r] - ptol * (1.0 + fabs(lg[r]))) { R[R_ACT + r] = 1; bad = 1; }
        else if (a == 2 && lam < -dtol) { R[R_ACT + r] = 0; bad = 1; }
        else if (a == 1 && lam > dtol) { R[R_ACT + r] = 0; bad = 1; }
      } else if (fabs(sum - ug[r]) > 1e-10 * (1.0 + fabs(ug[r]))) {
        bad = 1;
      }
    }
  }
  bad = block_max((double)bad, red) > 0.5;
  if (soft > 0.0)   // a rejected round also releases the near-sign variables; an accepted one keeps them
    for (int i = hl; i < n; i += PPT) {
      const int f = wk.fl[i];
      if (f >= 5) wk.fl[i] = bad ? 0 : f - 4;
    }
  if (vtx && hl == 0) {   // the next round starts from it (setup's R_SOL), or the scoring uses it
    R[R_LAM + r0] = lam0;
    R[R_SOL] = lam0;
  }
  if (bad) {
    if (hl == 0 && R[R_ROUNDS] >= s.polish_rounds) R[R_STATE] = PQ_PG_FALLBACK;
    return;
  }
  // ---- accepted: score the polished point (polish_w.hip's final block) ------------------
  double* sx = st.x + (int64_t)b * ld;
  double* sz = st.z + (int64_t)b * st.m_ld;
  double* sy = st.y + (int64_t)b * st.m_ld;
  double xpx = 0.0, qx = 0.0, pres = 0.0, dres = 0.0, gapb = 0.0;
  // (four of the thread's elements per step, every load issued first, as in the checks above;
  // the same sums in the same order)
  for (int i0 = hl; i0 < n; i0 += 4 * PPT) {
    double xv[4], pv[4], gv[4], qv[4], lbv[4], ubv[4];
    int fv[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int i = i0 + j * PPT, ic = i < n ? i : 0;
      xv[j] = wk.xs[ic];
      pv[j] = wk.Px[ic];
      gv[j] = wk.g[ic];
      qv[j] = q[ic];
      fv[j] = wk.fl[ic];
      lbv[j] = has_box ? lb[ic] : 0.0;
      ubv[j] = has_box ? ub[ic] : 0.0;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int i = i0 + j * PPT;
      if (i >= n) continue;
      const double xi = xv[j];
      double zb = 0.0;
      if (has_box) zb = fv[j] ? -gv[j] : 0.0;
      xpx += xi * pv[j];
      qx += qv[j] * xi;
      dres = fmax(dres, fabs(gv[j] + zb));
      if (has_box) {
        const double lbi = lbv[j], ubi = ubv[j];
        if (!isinf(lbi)) { pres = fmax(pres, lbi - xi); gapb += lbi * fmin(zb, 0.0); }
        if (!isinf(ubi)) { pres = fmax(pres, xi - ubi); gapb += ubi * fmax(zb, 0.0); }
        sy[st.mg_pad + i] = zb;
      }
      sx[i] = xi;
    }
  }
  for (int r = 0; r < mg; ++r) {
    const double* cr = Cg + (int64_t)r * ld;
    double sum = row_dot4(cr, wk.xs, n, hl);
    sum = block_sum(sum, red);
    const double lam = lamof(r);
    double v;
    if (lg[r] == ug[r]) v = fabs(sum - ug[r]);
    else v = fmax(isinf(ug[r]) ? 0.0 : sum - ug[r], isinf(lg[r]) ? 0.0 : lg[r] - sum);
    if (hl == 0) {
      pres = fmax(pres, v);
      gapb += (lam > 0.0 ? ug[r] : (isinf(lg[r]) ? 0.0 : lg[r])) * lam;
      sy[r] = lam;
      sz[r] = sum;
    }
  }
  xpx = block_sum(xpx, red);
  qx = block_sum(qx, red);
  gapb = block_sum(gapb, red);
  pres = block_max(pres, red);
  dres = block_max(dres, red);
  if (hl == 0) {
    double* o = st.out + (int64_t)b * PQ_OUT_FIELDS;
    o[PQ_OUT_OBJ] = 0.5 * xpx + qx;
    o[PQ_OUT_PRIM] = fmax(pres, 0.0);
    o[PQ_OUT_DUAL] = dres;
    o[PQ_OUT_GAP] = fabs(xpx + qx + gapb);
    o[PQ_OUT_RHO] = st.rho[b];
    o[PQ_OUT_NFREE] = R[R_K];
    o[PQ_OUT_ROUNDS] = R[R_ROUNDS];
    st.status[b] = PQ_SOLVED;
    R[R_STATE] = PQ_PG_DONE;
  }
}

}  // namespace pq

extern "C" int pq_polish_grouped_init(const pq_lowrank* lr, const pq_problem* pb, pq_state* st, double* rec,
                                      const pq_settings* s, void* stream) {
  PQ_CHECK_ARG(lr && pb && st && s && rec, "pq_polish_grouped_init: null argument");
  PQ_CHECK_ARG(lr->dg && lr->panel && lr->rows && lr->tlen, "pq_polish_grouped_init: window (with dg) missing");
  PQ_CHECK_ARG(pb->mg >= 0 && pb->mg <= pq::PG_MGMAX && (pb->mg == 0 || (pb->Cg && pb->lg && pb->ug)),
               "pq_polish_grouped_init: needs 0 <= mg <= %d general rows", pq::PG_MGMAX);
  PQ_CHECK_ARG(st->work && st->work_stride >= PQ_WORK_DOUBLES(pb->ld, st->mg_pad),
               "pq_polish_grouped_init: work buffer too small");
  if (pb->batch <= 0) return 0;
  hipLaunchKernelGGL(pq::k_pg_init, dim3(pb->batch), dim3(pq::PT), 0, (hipStream_t)stream, *lr, *pb, *st, rec, *s);
  PQ_CHECK_LAUNCH("pq_polish_grouped_init");
  return 0;
}

namespace pq {
// Side streams of a round's per-date solves: the free-set buckets and the wide rounds touch
// disjoint dates, so they run concurrently (fork / join events on the caller's stream)
// instead of one launch after another, each with its own tail.  Created once per device on
// first use; NULL when that fails (everything then runs on the caller's stream).  One host
// thread per device drives a round at a time (the engine's use).
struct PgSide {
  static constexpr int NS = 7;
  bool ok = false;
  hipStream_t s[NS];
  hipEvent_t fork, join[NS];
};
static PgSide* pg_side() {
  static PgSide sides[64];
  static std::mutex mu;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
  std::lock_guard<std::mutex> lock(mu);
  PgSide& p = sides[dev];
  if (!p.ok) {
    bool good = hipEventCreateWithFlags(&p.fork, hipEventDisableTiming) == hipSuccess;
    for (int i = 0; i < PgSide::NS && good; ++i)
      good = hipStreamCreateWithFlags(&p.s[i], hipStreamNonBlocking) == hipSuccess &&
             hipEventCreateWithFlags(&p.join[i], hipEventDisableTiming) == hipSuccess;
    if (!good) {
      (void)hipGetLastError();
      return nullptr;
    }
    p.ok = true;
  }
  return &p;
}

// the group form for groups with at least this many forming dates (fewer: a single window
// pass per date is cheaper than the union pass); PQ_PG_GFORM overrides, 0 = off.  Config 3
// (profiles/r03J_bench_gform*.log): 1 / 2 / 3 / 5 -> polish 4.83 / 4.86 / 4.87 / 4.91 ms
// (5.03 ms without, r03G_bench_nogform.log) -- within the run-to-run spread of each other
static int group_form_min() {
  static const int v = [] {
    const char* e = getenv("PQ_PG_GFORM");
    return e ? atoi(e) : 2;
  }();
  return v;
}

// the big group form (k_pg_form_grp_big) for groups with at least this many forming dates;
// PQ_PG_GFORM_BIG overrides, 0 = off (A/B)
static int group_form_big_min() {
  static const int v = [] {
    const char* e = getenv("PQ_PG_GFORM_BIG");
    return e ? atoi(e) : 2;
  }();
  return v;
}

// free sets beyond the LDS solve inside the pipeline (k_pg_big); PQ_PG_BIG=0 hands them to the
// per-date kernel as before (A/B)
static int pg_big() {
  static const int v = [] {
    const char* e = getenv("PQ_PG_BIG");
    return e ? atoi(e) : 1;
  }();
  return v;
}

// buckets (48, 64, 80, 96 in order) taken by the register-tile solve (polish_rt.hip) instead of
// the LDS solve: 4 (default, up to 96) or 3 (up to 80); PQ_PG_RT overrides (0 = the LDS solve
// for every bucket, A/B)
static int solve_rt() {
  static const int v = [] {
    const char* e = getenv("PQ_PG_RT");
    return e ? atoi(e) : 4;
  }();
  return v;
}

// waves per date of the solve, per free-set bucket (48, 64, 80, 96, 128): PQ_PG_SOLVE_NW
// (1, 2 or 4) overrides all buckets
static int solve_waves(int bucket) {
  static const int forced = [] {
    const char* e = getenv("PQ_PG_SOLVE_NW");
    const int v = e ? atoi(e) : 0;
    return v == 1 || v == 2 || v == 4 ? v : 0;
  }();
  static const int def[5] = {2, 2, 4, 4, 4};
  return forced ? forced : def[bucket];
}

template <int KS>
static void launch_solve_ks(int nw, int B, hipStream_t str, const pq_problem* pb, pq_state* st, double* rec,
                            const pq_settings* s, int ldk, int klo) {
  const int inner = s->polish_inner > 0 ? s->polish_inner : 0;
  if (nw == 1)
    hipLaunchKernelGGL((k_pg_solve<KS, 1>), dim3(resident_grid((const void*)k_pg_solve<KS, 1>, 64, B)), dim3(64), 0,
                       str, *pb, *st, rec, *s, ldk, klo, inner);
  else if (nw == 2)
    hipLaunchKernelGGL((k_pg_solve<KS, 2>), dim3(resident_grid((const void*)k_pg_solve<KS, 2>, 128, B)), dim3(128),
                       0, str, *pb, *st, rec, *s, ldk, klo, inner);
  else
    hipLaunchKernelGGL((k_pg_solve<KS, 4>), dim3(resident_grid((const void*)k_pg_solve<KS, 4>, 256, B)), dim3(256),
                       0, str, *pb, *st, rec, *s, ldk, klo, inner);
}
static void launch_solve(int bucket, int nw, int B, hipStream_t str, const pq_problem* pb, pq_state* st,
                         double* rec, const pq_settings* s, int ldk, int klo) {
  switch (bucket) {
    case 0: launch_solve_ks<48>(nw, B, str, pb, st, rec, s, ldk, klo); break;
    case 1: launch_solve_ks<64>(nw, B, str, pb, st, rec, s, ldk, klo); break;
    case 2: launch_solve_ks<80>(nw, B, str, pb, st, rec, s, ldk, klo); break;
    case 3: launch_solve_ks<96>(nw, B, str, pb, st, rec, s, ldk, klo); break;
    default: launch_solve_ks<128>(nw, B, str, pb, st, rec, s, ldk, klo); break;
  }
}
}  // namespace pq

extern "C" int pq_polish_grouped_round(const pq_lowrank* lr, const pq_problem* pb, pq_state* st, double* rec,
                                       int32_t ldk, const int32_t* gdates, int32_t ngroups, const int32_t* urows,
                                       const int32_t* ucnt, const int32_t* uoff, int32_t umax, const pq_settings* s,
                                       double* pass_scratch, const pq_pg_wide* wide, void* stream) {
  PQ_CHECK_ARG(lr && pb && st && s && rec && pass_scratch, "pq_polish_grouped_round: null argument");
  static_assert(pq::QSCR == pq::GB_OFF && pq::GB_END == PQ_PG_PASS_SCRATCH, "PQ_PG_PASS_SCRATCH out of date");
  PQ_CHECK_ARG(gdates && urows && ucnt && uoff && umax > 0 && umax <= pq::QU,
               "pq_polish_grouped_round: group plan missing (umax <= %d)", pq::QU);
  PQ_CHECK_ARG(pb->n % 2 == 0 && lr->ldp % 2 == 0, "pq_polish_grouped_round: needs even n and panel stride");
  PQ_CHECK_ARG(pb->mg >= 0 && pb->mg <= pq::PG_MGMAX, "pq_polish_grouped_round: mg <= %d", pq::PG_MGMAX);
  PQ_CHECK_ARG(st->K && ldk >= 64 && st->K_stride >= (int64_t)ldk * ldk,
               "pq_polish_grouped_round: K scratch (ldk x ldk per problem) too small");
  if (pb->batch <= 0 || ngroups <= 0) return 0;
  hipStream_t str = (hipStream_t)stream;
  const int B = pb->batch;
  const int kmax = ldk < pq::PG_KMAX ? ldk : pq::PG_KMAX;
  // free sets between the LDS solve and the K scratch: the grouped large-free-set solve
  const int kbig = (pq::pg_big() && ldk > kmax) ? (ldk < pq::PG_KBIG ? ldk : pq::PG_KBIG) : kmax;
  hipLaunchKernelGGL(pq::k_pg_setup, dim3(B), dim3(pq::PT), 0, str, *pb, *st, rec, kmax, wide ? 1 : 0, kbig);
  const dim3 gsplit(ngroups * pq::QS);
  hipLaunchKernelGGL(pq::k_pg_passA<0>, gsplit, dim3(pq::QT), 0, str, *lr, *pb, *st, rec, gdates, urows, ucnt, uoff,
                     umax, pass_scratch);
  hipLaunchKernelGGL(pq::k_pg_passB<0>, gsplit, dim3(pq::QT), 0, str, *lr, *pb, *st, rec, gdates, urows, ucnt, uoff,
                     umax, pass_scratch);
  hipLaunchKernelGGL(pq::k_pg_post<0>, dim3(B), dim3(pq::PPT), 0, str, *lr, *pb, *st, rec, *s, gdates, ngroups,
                     pass_scratch);
  if (pq::group_form_min() > 0)   // P_FF from one union Gram per polish group (k_pg_form_grp)
    hipLaunchKernelGGL(pq::k_pg_form_grp, dim3(ngroups), dim3(pq::FT), 0, str, *lr, *pb, *st, rec, gdates, urows,
                       ucnt, umax, pass_scratch, pq::group_form_min());
  hipLaunchKernelGGL(pq::k_pg_form<pq::PG_KMAX>, dim3(B), dim3(pq::FT), 0, str, *lr, *pb, *st, rec, ldk, gdates, ngroups, urows,
                     ucnt, uoff, umax, pass_scratch);
  // one workgroup per date, the LDS triangle sized to the free set (more dates per CU when small);
  // the buckets (and the wide rounds) on side streams, joined before the exact-P x passes
  pq::PgSide* side = pq::pg_side();
  int used = 0;
  if (side && hipEventRecord(side->fork, str) != hipSuccess) side = nullptr;
  auto on = [&](int i) -> hipStream_t {
    if (!side || hipStreamWaitEvent(side->s[i], side->fork, 0) != hipSuccess) return str;
    used |= 1 << i;
    return side->s[i];
  };
  // free sets of kmax + 1 .. kbig first (their P_FF, then the factor and solve): the longest
  // solves when there are any, and a resident grid that only reads an empty list when there are
  // none -- launched after the other buckets, its workgroups waited for their CUs to drain
  if (kbig > kmax) {
    static_assert(pq::PG_KBIG == 256, "k_pg_form<PG_KBIG> tiling");
    const hipStream_t sb = on(6);
    if (pq::group_form_big_min() > 0 && lr->mu == nullptr)   // from one union Gram per polish group
      hipLaunchKernelGGL(pq::k_pg_form_grp_big, dim3(ngroups * pq::GBS), dim3(pq::FT), 0, sb, *lr, *pb, *st, rec,
                         gdates, urows, ucnt, umax, pass_scratch, pq::group_form_big_min());
    hipLaunchKernelGGL(pq::k_pg_form<pq::PG_KBIG>, dim3(pq::resident_grid((const void*)pq::k_pg_form<pq::PG_KBIG>,
                                                                          pq::FT, B)),
                       dim3(pq::FT), 0, sb, *lr, *pb, *st, rec, ldk, gdates, ngroups, urows, ucnt, uoff, umax,
                       pass_scratch);
    hipLaunchKernelGGL(pq::k_pg_big, dim3(pq::resident_grid((const void*)pq::k_pg_big, pq::PT, B)), dim3(pq::PT), 0,
                       sb, *lr, *pb, *st, rec, *s, ldk, kmax);
  }
  // the LDS solve's buckets beyond the register solve's (largest free sets first), and the
  // register solve's buckets in one launch
  const int nrt = pq::solve_rt() <= 0 ? 0 : (pq::solve_rt() >= 4 ? 4 : 3);   // register buckets 0 .. nrt - 1
  for (int i = 4; i >= nrt; --i) {
    static const int KSB[5] = {48, 64, 80, 96, 128};
    if (i >= 2 && kmax <= KSB[i - 1]) continue;
    pq::launch_solve(i, pq::solve_waves(i), B, on(i), pb, st, rec, s, ldk, i ? KSB[i - 1] : 0);
  }
  // (side stream 1: the streams are dealt round-robin over the process's hardware queues, four
  // by default, so stream 0 shared one with the <= 128 bucket's stream 4 and the register
  // solve waited for that kernel to finish)
  if (nrt > 0 && pq_pg_solve_rt_launch(nrt + 2, B, on(1), pb, st, rec, s, ldk)) return -1;
  if (wide && pq_pg_wide_launch(lr, pb, st, rec, s, wide, on(5))) return -1;   // free sets beyond kmax
  for (int i = 0; side && i < pq::PgSide::NS; ++i)
    if ((used & (1 << i)) && (hipEventRecord(side->join[i], side->s[i]) != hipSuccess ||
                              hipStreamWaitEvent(str, side->join[i], 0) != hipSuccess)) {
      pq::set_error("pq_polish_grouped_round: joining the solve streams failed");
      return -2;
    }
  hipLaunchKernelGGL(pq::k_pg_passA<1>, gsplit, dim3(pq::QT), 0, str, *lr, *pb, *st, rec, gdates, urows, ucnt, uoff,
                     umax, pass_scratch);
  hipLaunchKernelGGL(pq::k_pg_passB<1>, gsplit, dim3(pq::QT), 0, str, *lr, *pb, *st, rec, gdates, urows, ucnt, uoff,
                     umax, pass_scratch);
  hipLaunchKernelGGL(pq::k_pg_post<1>, dim3(B), dim3(pq::PPT), 0, str, *lr, *pb, *st, rec, *s, gdates, ngroups,
                     pass_scratch);
  PQ_CHECK_LAUNCH("pq_polish_grouped_round");
  return 0;
}

// occupancy x CUs of a kernel, cached per (kernel, device); B when the query fails
int pq::resident_grid(const void* kernel, int block, int B) {
  struct Entry { const void* k; int dev, n; };
  static Entry cache[64];
  static int used = 0;
  static std::mutex mu;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return B;
  std::lock_guard<std::mutex> lock(mu);
  for (int i = 0; i < used; ++i)
    if (cache[i].k == kernel && cache[i].dev == dev) return cache[i].n < B ? cache[i].n : B;
  int per = 0, cus = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kernel, block, 0) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || per <= 0 || cus <= 0) {
    (void)hipGetLastError();
    return B;
  }
  const int n = per * cus;
  if (used < 64) cache[used++] = Entry{kernel, dev, n};
  return n < B ? n : B;
}
