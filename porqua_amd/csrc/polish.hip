// K4: active-set polish of the ADMM point + exact residuals / objective.
//
// One 256-thread workgroup per QP.  From the ADMM iterate (x, z, y) the box rows and the
// general rows (budget / group caps) are classified as active at a bound or free.  Fixed
// variables are eliminated; the reduced KKT
//      [P_FF + dI   C_aF'] [x_F]   [-q_F - P_FB x_B]
//      [C_aF       -dI   ] [lam] = [ d_a - C_aB x_B ]
// is factored with the same workgroup MFMA Cholesky as K2 (P_FF gathered through the free
// index list at first touch, never materialised), a Schur complement for the <= 64 active
// rows, and proximal iterative refinement started at the ADMM point (exact where the
// system is nonsingular, stays at the ADMM multipliers along degenerate directions, e.g.
// every weight at a bound).  Primal bound violations / wrong-sign multipliers update the
// active set for another round.  The accepted point, or the ADMM point when polishing
// fails, is scored with an exact P x mat-vec: objective 0.5 x'Px + q'x
// (src/qp_problems.py:219-221, test/tests_quadratic_program.py:72,82) and the qpsolvers
// residuals of example/compare_solver.ipynb:212-216.
#include "polish_dev.h"
#include "capi_util.h"

namespace pq {

struct PolishForm {
  const double* P;
  int64_t ld;
  const int* F;
  int k;
  double ps, dadd;
  __device__ __forceinline__ double operator()(int gi, int gj) const {
    if (gi >= k || gj >= k) return gi == gj ? 1.0 : 0.0;
    double v = ps * P[(int64_t)F[gi] * ld + F[gj]];
    if (gi == gj) v += dadd;
    return v;
  }
};

__global__ __launch_bounds__(PT) void k_polish(pq_problem pb, pq_state st, const int32_t* idx,
                                               int nidx, pq_settings s, pq_lowrank lr) {
  constexpr int LDMAX = 1024;
  __shared__ __attribute__((aligned(16))) double smem[CHOL_LDS + 2 * LDMAX + 14 * 64 + 64 + LDMAX + 256];
  double* stg = smem;                  // Cholesky stream buffers; S factor during refinement
  double* vec = smem + 4 * STAGE;      // sD region: 3 LDMAX vectors during refinement
  double* solx = smem + CHOL_LDS;      // compact solution x_F
  double* rF = solx + LDMAX;           // compact rhs of the F rows
  double* solL = rF + LDMAX;           // 64: multipliers of the active rows
  double* dA = solL + 64;              // 64: rhs of the active rows
  double* rl = dA + 64;                // 64
  double* wl = rl + 64;                // 64
  double* t64 = wl + 64;               // 64
  double* part = t64 + 64;             // 4*64 (also reduction scratch)
  double* red = part + 4 * 64;         // 64
  double* lamF = red + 64;             // 64: multipliers of all general rows (by row)
  double* y64p = lamF + 64;            // 4*64 partial sums of the diagonal-block products
  // index bookkeeping lives in LDS: these arrays are rewritten every active-set round and
  // read at wave-uniform addresses, which hipcc serves from the (non-coherent) scalar
  // cache when they sit in global memory -- stale values in round >= 2.
  int* fl = reinterpret_cast<int*>(y64p + 4 * 64);   // LDMAX: 0 free, 1 at lower, 2 at upper
  int* Fl = fl + LDMAX;                               // LDMAX: free-variable list
  int* act = Fl + LDMAX;                              // 64
  int* Al = act + 64;                                 // 64
  int* cnt = Al + 64;                                 // PT + 8

  const int b = idx ? idx[blockIdx.x] : (int)blockIdx.x;
  const int st0 = st.status[b];
  if (st0 != PQ_SOLVED && st0 != PQ_MAX_ITER) return;
  const int n = pb.n, ld = pb.ld, mg = pb.mg;
  const int t = threadIdx.x, w = wave_id(), l = lane_id();
  const double* P = pb.P + (int64_t)b * pb.P_stride;
  const double ps = pb.p_scale ? pb.p_scale[b] : 1.0;
  const double pd = pb.p_diag ? pb.p_diag[b] : 0.0;
  const double* q = pb.q + (int64_t)b * pb.q_stride;
  const double* Cg = pb.Cg ? pb.Cg + (int64_t)b * pb.Cg_stride : nullptr;
  const double* lg = pb.lg ? pb.lg + (int64_t)b * pb.g_stride : nullptr;
  const double* ug = pb.ug ? pb.ug + (int64_t)b * pb.g_stride : nullptr;
  const bool has_box = pb.lb != nullptr;
  const double* lb = has_box ? pb.lb + (int64_t)b * pb.box_stride : nullptr;
  const double* ub = has_box ? pb.ub + (int64_t)b * pb.box_stride : nullptr;
  double* K = st.K + (int64_t)b * st.K_stride;
  double* Dt = st.Dt + (int64_t)b * st.Dt_stride;
  double* sx = st.x + (int64_t)b * ld;
  double* sz = st.z + (int64_t)b * st.m_ld;
  double* sy = st.y + (int64_t)b * st.m_ld;
  // work layout (doubles): xs | xb | g | Px | U (mg_pad rows)
  double* W = st.work + (int64_t)b * st.work_stride;
  double* xs = W;
  double* xb = xs + ld;
  double* g = xb + ld;
  double* Px = g + ld;
  double* U = Px + ld;
#ifdef PQ_PROFILE
  double* prof = W + PQ_WORK_PROF(ld, st.mg_pad);
  if (t < 16) prof[t] = 0.0;
  long long t_last_ = wall_clock64();
#endif

  // ---- problem scale -> tolerances ----------------------------------------------------
  double sc = 0.0;
  for (int i = t; i < n; i += PT) sc = fmax(sc, fmax(fabs(q[i]), fabs(ps * P[(int64_t)i * ld + i] + pd)));
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

  // exact P x and gradient g = P x + q + Cg' lam of the point in xs (rows_dot_vec emit)
  auto emit_g = [&](int i, double sum) {
    const double pxi = ps * sum + pd * xs[i];
    double gi = pxi + q[i];
    for (int r = 0; r < mg; ++r) gi += Cg[(int64_t)r * ld + i] * lamF[r];
    Px[i] = pxi;
    g[i] = gi;
  };
  // P x of the point in xs: window form when given (vec / stg are free at the call sites:
  // after refinement and in the final scoring), else the dense rows of P
  auto full_px = [&]() {
    if (lr.panel) lr_px(lr, b, n, xs, vec, stg, red, emit_g);
    else rows_dot_vec(P, ld, n, n, [](int p) { return p; }, xs, emit_g);
  };

  int accepted = 0, rounds = 0, nfree = 0;
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
    {
      int p = cnt[t];
      for (int i = t * chunk; i < min(n, (t + 1) * chunk); ++i)
        if (fl[i] == 0) Fl[p++] = i;
    }
    const int k = cnt[PT];
    const int ma = cnt[PT + 1];
    nfree = k;
    const int nbk = (k + TB - 1) / TB;
    int nzb = 0;
    for (int i = t; i < ld; i += PT) {
      const double v = i < n ? (fl[i] == 1 ? lb[i] : (fl[i] == 2 ? ub[i] : 0.0)) : 0.0;
      xb[i] = v;
      nzb |= (v != 0.0);
    }
    nzb = block_or(nzb, red);
    PQ_STAMP(1);
    __builtin_amdgcn_s_dcache_inv();
    // ---- reduced rhs: rF = -q_F - ps P_FB x_B ;  d_a = rhs_a - C_aB x_B -----------------
    if (nzb && lr.panel) {   // window form (P may hold its lower triangle only): P x_B -> g
      lr_px(lr, b, n, xb, vec, stg, red, [&](int i, double sum) { g[i] = sum; });
      __syncthreads();
      for (int p = t; p < k; p += PT) rF[p] = -q[Fl[p]] - ps * g[Fl[p]];
    } else if (nzb) {   // (long-only: every fixed weight is 0 and P_FB x_B vanishes)
      rows_dot_vec(P, ld, n, k, [&](int p) { return Fl[p]; }, xb,
                   [&](int p, double sum) { rF[p] = -q[Fl[p]] - ps * sum; });
    } else {
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
    // ---- factor M = ps P_FF + (pd + delta) I ---------------------------------------------
    int info = 0;
    if (k > 0) info = wg_cholesky(PolishForm{P, ld, Fl, k, ps, pd + delta}, K, ld, nbk, k, Dt, smem);
    if (info) break;
    PQ_STAMP(3);
    double* t1 = vec;                 // LDMAX each, inside the sD region
    double* dx = vec + LDMAX;
    double* rx = vec + 2 * LDMAX;
    // ---- U = L^-1 C_aF' (columns a), S = U'U + delta I, factor S in stg ---------------
    for (int a = 0; a < ma; ++a) {
      const int r = Al[a];
      for (int p = t; p < nbk * TB; p += PT) rx[p] = p < k ? Cg[(int64_t)r * ld + Fl[p]] : 0.0;
      __syncthreads();
      fwd_solve(K, ld, Dt, nbk, rx, t1, t64, y64p);
      for (int p = t; p < nbk * TB; p += PT) U[(int64_t)a * ld + p] = t1[p];
      __syncthreads();
    }
    __builtin_amdgcn_s_dcache_inv();   // U is re-read below, partly at uniform addresses
    for (int e = t; e < TB * TB; e += PT) {
      const int i = e >> 6, j = e & 63;
      double v = (i == j) ? 1.0 : 0.0;
      if (i < ma && j < ma) {
        v = (i == j) ? delta : 0.0;
        if (j <= i) for (int p = 0; p < k; ++p) v += U[(int64_t)i * ld + p] * U[(int64_t)j * ld + p];
      }
      stg[i * DP + j] = v;
    }
    __syncthreads();
    if (tile_potrf_lds(stg, ma)) break;
    PQ_STAMP(4);
    // ---- proximal iterative refinement -------------------------------------------------
    for (int itr = 0; itr < s.refine_iters; ++itr) {
      // rx = rF - (ps P_FF + pd I) solx - C_aF' solL ;  rl = dA - C_aF solx
      for (int p = w; p < k; p += PW) {
        const int fi = Fl[p];
        double sum = 0.0;
        for (int qq = l; qq < k; qq += 64) {   // lower triangle only: P[max][min]
          const int fj = Fl[qq];
          sum += P[(int64_t)max(fi, fj) * ld + min(fi, fj)] * solx[qq];
        }
        sum = wave_sum(sum);
        if (l == 0) {
          double v = rF[p] - ps * sum - pd * solx[p];
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
      fwd_solve(K, ld, Dt, nbk, rx, t1, t64, y64p);
      // wl = U' t1 - rl ; dlam = S^-1 wl (S = Ls Ls', tiny, one thread)
      for (int a = w; a < ma; a += PW) {
        double sum = 0.0;
        for (int p = l; p < k; p += 64) sum += U[(int64_t)a * ld + p] * t1[p];
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
        for (int a = 0; a < ma; ++a) v -= U[(int64_t)a * ld + p] * wl[a];
        t1[p] = v;
      }
      __syncthreads();
      bwd_solve(K, ld, Dt, nbk, t1, dx, t64, part, y64p);
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
    __builtin_amdgcn_s_dcache_inv();   // xs was rewritten: no stale scalar-cache reads
    full_px();
    __syncthreads();
    PQ_STAMP(6);
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

static int polish_launch(const pq_lowrank* lr, const pq_problem* pb, pq_state* st, const int32_t* idx,
                         int32_t nidx, const pq_settings* s, void* stream, const char* who) {
  PQ_CHECK_ARG(pb && st && s, "%s: null argument", who);
  PQ_CHECK_ARG(pb->ld <= 1024, "%s: ld=%d exceeds the LDS-resident limit 1024", who, pb->ld);
  PQ_CHECK_ARG(pb->mg <= 64, "%s: mg must be <= 64", who);
  PQ_CHECK_ARG(st->work && st->work_stride >= PQ_WORK_DOUBLES(pb->ld, st->mg_pad),
               "%s: work buffer too small", who);
  pq_lowrank l = {};
  if (lr) {
    PQ_CHECK_ARG(lr->panel && lr->rows && lr->tlen && lr->tmax > 0 && lr->tmax <= 1024,
                 "%s: window missing or tmax > 1024", who);
    PQ_CHECK_ARG((lr->ldp & 1) == 0, "%s: the window form needs an even panel stride", who);
    l = *lr;
  }
  const int grid = idx ? nidx : pb->batch;
  if (grid <= 0) return 0;
  hipLaunchKernelGGL(pq::k_polish, dim3(grid), dim3(pq::PT), 0, (hipStream_t)stream, *pb, *st, idx, nidx, *s, l);
  PQ_CHECK_LAUNCH(who);
  return 0;
}

extern "C" int pq_polish_batched(const pq_problem* pb, pq_state* st, const int32_t* idx, int32_t nidx,
                                 const pq_settings* s, void* stream) {
  return polish_launch(nullptr, pb, st, idx, nidx, s, stream, "pq_polish_batched");
}

extern "C" int pq_polish_lr_batched(const pq_lowrank* lr, const pq_problem* pb, pq_state* st,
                                    const int32_t* idx, int32_t nidx, const pq_settings* s,
                                    void* stream) {
  PQ_CHECK_ARG(lr != nullptr, "pq_polish_lr_batched: null window description");
  return polish_launch(lr, pb, st, idx, nidx, s, stream, "pq_polish_lr_batched");
}
