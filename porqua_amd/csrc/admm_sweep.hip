// K3, risk-aversion-sweep form: the fused low-rank ADMM of k_admm_grp for groups of up to 64
// problems that share ONE window (the risk-aversion row of a rebalance date, config 5:
// P_b = 2 lam_b Sigma_d, q_b = -mu_d).
//
// k_admm_grp runs a group's iterations in one 512-thread workgroup: for config 5 that is 256
// workgroups, one per CU, each streaming the date's 252 x 5000 window twice per iteration with
// 8 waves -- latency-bound at 0.14 MFMA busy and 0.25 of HBM (profiles/r05t_config5_*).  Here
// an iteration is two launches over the whole chip:
//   k_sw_pass  one workgroup per (group, 256-asset chunk): pass 2 of iteration k
//              (x~raw = X' Ut for the chunk's assets, all 64 problems as MFMA columns), the
//              x / Px / z / y updates and residual terms of iteration k, the rhs of iteration
//              k + 1 and its pass-1 partial W_chunk = X_chunk v (MFMA again) -- the window
//              chunk is read once per iteration for all problems of the group;
//   k_sw_mid   one workgroup per problem: the convergence test of iteration k from the chunk
//              partials, W = sum of the chunk partials, u = M_b^-1 kw (the per-problem
//              capacitance inverse, lower triangle), the pass-2 operand Ut and the general
//              rows' update of iteration k + 1.
// The rhs is never stored: k_sw_pass recomputes it from x, z, y (which it reads anyway) and
// the previous general-row term, with the same expression that produced the pass-1 operand.
// Per problem-iteration HBM bytes: x, Px, z, y read + write (64 n) + q (8 n) + M^-1
// (8 k(k+1)/2) + window (8 T n / group size) + chunk partials.
//
// The iterates are those of k_admm_grp's fused form (FUSE) up to summation order: same
// stopping rule, adaptive rho (NEED_REFACTOR), min_iter / max_iter and per-call iteration
// budget.  Replaces qpsolvers.solve_problem (src/qp_problems.py:211-214) for the sweep's
// batched solve (src/optimization.py:168-174 per risk aversion).
#include "common.h"
#include "capi_util.h"

// (experiment builds only) PQ_SW_X = 1: no state stores in the updates; 4: no pass-2 MFMA;
// 5: no pass-1 MFMA
#ifndef PQ_SW_X
#define PQ_SW_X 0
#endif
#ifndef PQ_SW_RU
#define PQ_SW_RU 2
#endif
// (experiment builds only) PQ_SW_PROF: phase clocks of k_sw_pass in the spare partial slots
#ifdef PQ_SW_PROF
#define SW_STAMP(k)                        \
  do {                                     \
    if (threadIdx.x == 0) {                \
      const long long now_ = clock64();    \
      pclk[k] += (double)(now_ - tclk);    \
      tclk = now_;                         \
    }                                      \
  } while (0)
#else
#define SW_STAMP(k) do { } while (0)
#endif

namespace pq {
namespace {

constexpr int SW_T = 512;            // threads of the pass workgroup (8 waves)
constexpr int SW_G = 64;             // problems per group (4 MFMA column tiles)
constexpr int SW_K = 256;            // window rows (padded; T <= 256)
constexpr int SW_SA = 16;            // assets per sub-chunk (one MFMA row tile)
constexpr int SW_PX = SW_SA + 1;     // LDS pitch of the window slab
constexpr int SW_CH = 256;           // assets per workgroup chunk
constexpr int SW_PV = SW_G + 1;      // LDS pitch of the x~ / v slabs
constexpr int SW_MG = 4;             // general rows (register-resident)
constexpr int SW_MT = 256;           // threads of the mid workgroup
constexpr int SR_N = 80;             // per-problem scalar record (doubles)
constexpr int RP_N = 16;             // per-(chunk, problem) partial record (doubles)
// scalar record
enum {
  S_RHO = 0, S_DINV, S_RB, S_SPS, S_SU, S_ACT, S_IT, S_END, S_STAT, S_QMAX, S_PD, S_ACT0,
  S_RMV = 12,                        // 3: general-row residual terms of the next iteration
  S_CW = 16, S_RGZ = 20, S_YG = 24, S_WG = 28, S_WGP = 32, S_ZG = 36, S_CGX = 40, S_CGV = 44,
  S_RG = 48, S_LG = 52, S_UG = 56, S_CMU = 60, S_MUV = 64
};
// partial record: mode 1 (iteration) [0..5] residual maxima, [6] mu.v, [8..11] Cg.v;
// mode 0 (prologue) [0] max |q|, [1..4] Cg.mu, [6] mu.v, [8..11] Cg.v, [12..15] Cg.x
// per-problem LDS scalars of the pass kernel
constexpr int SC_N = 5 + 5 * SW_MG;
enum { C_DINV = 0, C_RB, C_SU, C_ACT, C_CW = 4, C_RGZ = 8, C_YG = 12, C_WG = 16, C_WGP = 20, C_RBI = 24 };

__device__ __forceinline__ double sw_grho(double l, double u, double rho, const pq_settings& s) {
  if (l == u) return rho * s.eq_scale;
  if (isinf(l) && isinf(u)) return s.rho_min;
  return rho;
}

// reductions over the 16 lanes of a row (xor offsets < 16 stay inside it)
__device__ __forceinline__ double qsum16(double v) {
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double qmax16(double v) {
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
  return v;
}

// ---- per-problem setup (one thread per problem slot of every group) ------------------------
__global__ __launch_bounds__(256) void k_sw_setup(pq_lowrank lr, pq_problem pb, pq_state st, pq_settings s,
                                                  const int32_t* gdates, int ngroups, double* SR,
                                                  int iters_call) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  const int grp = e / SW_G, g = e - grp * SW_G;
  if (grp >= ngroups) return;
  const int b0 = gdates[grp];
  if (g >= gdates[grp + 1] - b0) return;
  const int b = b0 + g;
  double* R = SR + (int64_t)b * SR_N;
  const int stt = st.status[b];
  const int act = (stt == PQ_UNSOLVED || stt == PQ_NEED_REFACTOR);
  const double rho = st.rho[b];
  const double rb = pb.lb ? sw_grho(pb.lb[(int64_t)b * pb.box_stride], pb.ub[(int64_t)b * pb.box_stride], rho, s)
                          : 0.0;
  const double pd = pb.p_diag ? pb.p_diag[b] : 0.0;
  const double ps = (pb.p_scale ? pb.p_scale[b] : 1.0) * (lr.w_scale ? lr.w_scale[b] : 1.0);
  R[S_RHO] = rho;
  R[S_DINV] = 1.0 / (s.sigma + pd + rb);
  R[S_RB] = rb;
  R[S_SPS] = sqrt(fmax(ps, 0.0));
  R[S_SU] = 0.0;
  R[S_ACT] = act;
  R[S_ACT0] = act;
  R[S_IT] = st.iters[b];
  R[S_END] = min(s.max_iter, st.iters[b] + iters_call);
  R[S_STAT] = stt;
  R[S_PD] = pd;
  for (int r = 0; r < 3; ++r) R[S_RMV + r] = 0.0;
  for (int r = 0; r < SW_MG; ++r) {
    double zg = 0, yg = 0, lgv = 0, ugv = 0, rg = 0;
    if (r < pb.mg) {
      zg = st.z[(int64_t)b * st.m_ld + r];
      yg = st.y[(int64_t)b * st.m_ld + r];
      lgv = pb.lg[(int64_t)b * pb.g_stride + r];
      ugv = pb.ug[(int64_t)b * pb.g_stride + r];
      rg = sw_grho(lgv, ugv, rho, s);
    }
    R[S_ZG + r] = zg;
    R[S_YG + r] = yg;
    R[S_LG + r] = lgv;
    R[S_UG + r] = ugv;
    R[S_RG + r] = rg;
    R[S_WG + r] = rg * zg - yg;
    R[S_WGP + r] = rg * zg - yg;
    R[S_CW + r] = 0.0;
    R[S_RGZ + r] = 0.0;
    R[S_CGX + r] = 0.0;
    R[S_CGV + r] = 0.0;
    R[S_CMU + r] = 0.0;
  }
}

// ---- the fused pass: [pass 2 + updates of iteration k] + rhs / pass 1 of iteration k + 1 ----
// MODE 0: the prologue (rhs of the first iteration and its pass 1 only).  One 512-thread
// workgroup per CU walks its chunk in 16-asset sub-chunks.  The window slab of a sub-chunk
// (256 rows x 16 assets) is staged in LDS, where both passes read it, and the next slab and
// the next sub-chunk's x / Px / z / y are loaded into registers while the current one
// computes (a whole sub-chunk of MFMA and update work covers the HBM latency).
//   pass 2: wave w = (column tile w >> 1, K half w & 1) -- Ut of its half in registers;
//   update: thread t = (asset t & 15, problems (t >> 4) + 32 e); residual terms and sums
//           kept per thread over the chunk, 16-lane reductions once at its end;
//   pass 1: wave w owns window-row tiles 2w, 2w + 1 and all four column tiles.
template <int MODE, int MGR>
__global__ __launch_bounds__(SW_T) void k_sw_pass(pq_lowrank lr, pq_problem pb, pq_state st, pq_settings s,
                                                  const int32_t* gdates, int nch, const double* SR,
                                                  const double* Ut, double* Wp, double* Rp, int q_shared) {
  __shared__ __attribute__((aligned(16))) double Xs[2 * SW_K * SW_PX];   // window slabs [buf][u][asset]
  __shared__ __attribute__((aligned(16))) double XV[2 * SW_SA * SW_PV];  // x~ of the two K halves; half 0 then v
  __shared__ double p_sc[SW_G * SC_N];
  __shared__ double racc_l[10 * SW_T];   // per-thread residual maxima / mu.v, [slot][e][thread]
  __shared__ int s_row[SW_K];
  __shared__ int s_any;

  const int slot = xcd_slot(blockIdx.x, gridDim.x);
  const int grp = slot / nch, ch = slot - grp * nch;
  const int b0 = gdates[grp];
  const int G = gdates[grp + 1] - b0;
  const int t = threadIdx.x;
  const int n = pb.n, ld = pb.ld, mg = pb.mg, tmax = lr.tmax;
  const int T = lr.tlen[b0];
  const double sigma = s.sigma, alpha = s.alpha;
#ifdef PQ_SW_PROF
  double pclk[4] = {0.0, 0.0, 0.0, 0.0};
  long long tclk = clock64();
#endif

  if (t < SW_G) {
    const int g = t;
    double* sc = p_sc + g * SC_N;
    if (g < G) {
      const double* R = SR + (int64_t)(b0 + g) * SR_N;
      sc[C_DINV] = R[S_DINV];
      sc[C_RB] = R[S_RB];
      sc[C_RBI] = 1.0 / R[S_RB];   // (the box projection multiplies by 1 / rho_box)
      sc[C_SU] = R[S_SU];
      sc[C_ACT] = R[S_ACT];
#pragma unroll
      for (int r = 0; r < SW_MG; ++r) {
        sc[C_CW + r] = R[S_CW + r];
        sc[C_RGZ + r] = R[S_RGZ + r];
        sc[C_YG + r] = R[S_YG + r];
        sc[C_WG + r] = R[S_WG + r];
        sc[C_WGP + r] = R[S_WGP + r];
      }
    } else {
      for (int e = 0; e < SC_N; ++e) sc[e] = 0.0;
    }
  }
  for (int u = t; u < SW_K; u += SW_T) s_row[u] = u < T ? lr.rows[(int64_t)b0 * tmax + u] : -1;
  __syncthreads();
  if (t == 0) {
    int any = 0;
    for (int g = 0; g < G; ++g) any |= p_sc[g * SC_N + C_ACT] != 0.0;
    s_any = any;
  }
  __syncthreads();
  if (!s_any) return;   // uniform: nothing left to iterate in this group

  const int w = t >> 6, l = t & 63;
  const int m16 = l & 15, k4 = l >> 4;
  const double* __restrict__ panel = lr.panel;
  const int64_t ldp = lr.ldp;
  const int c0 = ch * SW_CH;
  const int c1 = min(c0 + SW_CH, n);

  // pass-2 operand: wave w holds Ut[128 kh + 4 s + k4][16 gt + m16], s < 32
  const int kh = w & 1, gt = w >> 1;
  double ut[32];
  if constexpr (MODE == 1) {
    const double* Ug = Ut + (int64_t)grp * SW_K * SW_G;
#pragma unroll
    for (int s2 = 0; s2 < 32; ++s2) ut[s2] = Ug[(128 * kh + 4 * s2 + k4) * SW_G + 16 * gt + m16];
  }
  (void)ut;

  f64x4 wacc[2][4];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int c = 0; c < 4; ++c) wacc[a][c] = f64x4{0.0, 0.0, 0.0, 0.0};

  // slab loader: thread t -> window row t >> 1, assets 8 (t & 1) .. + 8 of the sub-chunk
  const int lrow = t >> 1, lhalf = t & 1;
  const int lr_id = s_row[lrow];
  const double* lsrc = panel + (int64_t)(lr_id < 0 ? 0 : lr_id) * ldp + 8 * lhalf;
  double sl[8];
  // unconditional loads from clamped addresses, zeroed when stored: a conditional load is an
  // exec-masked block whose else-branch zeroes the destination, a write-after-write that makes
  // the compiler wait for every outstanding load there (s_waitcnt vmcnt(0)), which would
  // expose the latency of the prefetches issued before it
  int sl_i0 = 0;
  auto slab_load = [&](int i0) {
    sl_i0 = i0;
#pragma unroll
    for (int e = 0; e < 8; ++e) sl[e] = lsrc[min(i0 + 8 * lhalf + e, n - 1) - 8 * lhalf];
  };
  auto slab_store = [&](int buf) {
    double* d = Xs + buf * (SW_K * SW_PX) + lrow * SW_PX + 8 * lhalf;
#pragma unroll
    for (int e = 0; e < 8; ++e) d[e] = (lr_id >= 0 && sl_i0 + 8 * lhalf + e < n) ? sl[e] : 0.0;
  };

  // update roles: asset i0 + (t & 15), problems g = (t >> 4) + 32 e
  const int ui = t & 15, ug = t >> 4;
  const double* mu0 = lr.mu ? lr.mu + (int64_t)b0 * lr.mu_stride : nullptr;
  const double* Cg0 = mg ? pb.Cg : nullptr;   // shared rows (host-checked Cg_stride == 0)
  constexpr int MGA = MGR > 0 ? MGR : 1;
  // prefetched one sub-chunk ahead: the element state and the asset's shared values (every
  // value the updates read from memory, so their waits never cover the next prefetch)
  double px_[2], x_[2], zb_[2], yb_[2], q_[2], mu_, lo_, up_, cg_[MGA];
  // (unconditional loads from clamped addresses, as for the slab: values of inactive or
  // out-of-range elements are loaded but never used -- the updates run under act && inb)
  auto state_load = [&](int i0) {
    const int ia = min(i0 + ui, n - 1);
    mu_ = mu0 ? mu0[ia] : 0.0;
    lo_ = pb.lb[ia];   // (shared box rows, host-checked)
    up_ = pb.ub[ia];
#pragma unroll
    for (int r = 0; r < MGA; ++r) cg_[r] = r < mg ? Cg0[(int64_t)r * ld + ia] : 0.0;
    const double qa = q_shared ? pb.q[(int64_t)b0 * pb.q_stride + ia] : 0.0;
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int g = ug + 32 * e;
      const int b = b0 + (g < G ? g : 0);
      // 32-bit element offsets (host-checked < 2^31): SGPR base + VGPR offset addressing
      const unsigned ox = (unsigned)(b * ld + ia), oz = (unsigned)(b * st.m_ld + st.mg_pad + ia);
      x_[e] = st.x[ox];
      zb_[e] = st.z[oz];
      yb_[e] = st.y[oz];
      px_[e] = MODE == 1 ? st.Px[ox] : 0.0;
      q_[e] = q_shared ? qa : pb.q[(unsigned)(b * pb.q_stride + ia)];
    }
  };

  double rcg[2][MGA], rcm[2][MGA], rcx[2][MGA];
#pragma unroll
  for (int e = 0; e < 2; ++e)
#pragma unroll
    for (int r = 0; r < MGA; ++r) rcg[e][r] = rcm[e][r] = rcx[e][r] = 0.0;
  for (int k = 0; k < 10; ++k) racc_l[k * SW_T + t] = 0.0;   // (own slots: no barrier needed)

  slab_load(c0);
  slab_store(0);
  state_load(c0);
  __syncthreads();
  SW_STAMP(3);
  int cur = 0;
  for (int i0 = c0; i0 < c1; i0 += SW_SA) {
    const bool more = i0 + SW_SA < c1;
    if (more) slab_load(i0 + SW_SA);   // lands during this sub-chunk; stored at its end
    const double* X = Xs + cur * (SW_K * SW_PX);

    if constexpr (MODE == 1) {
      // ---- pass 2: x~raw[i][g] = sum_u X[u][i] Ut[u][g] over this wave's K half ----------
      // two accumulation chains (even / odd k-steps): a dependent f64 MFMA chain issues at half rate
      f64x4 xa = f64x4{0.0, 0.0, 0.0, 0.0}, xb = f64x4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int s2 = 0; s2 < 32; s2 += 2) {
        if (PQ_SW_X == 4) break;
        xa = __builtin_amdgcn_mfma_f64_16x16x4f64(X[(128 * kh + 4 * s2 + k4) * SW_PX + m16], ut[s2], xa, 0, 0, 0);
        xb = __builtin_amdgcn_mfma_f64_16x16x4f64(X[(128 * kh + 4 * s2 + 4 + k4) * SW_PX + m16], ut[s2 + 1], xb, 0,
                                                  0, 0);
      }
      xa += xb;
      double* xv = XV + kh * (SW_SA * SW_PV);
#pragma unroll
      for (int r = 0; r < 4; ++r) xv[(k4 + 4 * r) * SW_PV + 16 * gt + m16] = xa[r];
      __syncthreads();
      SW_STAMP(0);
    }

    // ---- per-element updates (MODE 1) / first rhs (MODE 0); v = rhs / c into half 0 ---------
    {
      const int ia = i0 + ui;
      const bool inb = ia < n;
      const double mui = mu_, lo = lo_, up = up_;
      double cgi[MGA];
#pragma unroll
      for (int r = 0; r < MGA; ++r) cgi[r] = cg_[r];
      double xs[2], zs[2], ys[2], pxs[2], qs[2];
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        xs[e] = x_[e];
        zs[e] = zb_[e];
        ys[e] = yb_[e];
        pxs[e] = px_[e];
        qs[e] = q_[e];
      }
      if (more) state_load(i0 + SW_SA);   // the next sub-chunk's state, in flight from here
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int g = ug + 32 * e;
        const double* sc = p_sc + g * SC_N;
        const bool act = sc[C_ACT] != 0.0;   // (0 for g >= G)
        const int b = b0 + (g < G ? g : 0);
        double v = 0.0;
        double red[12];
#pragma unroll
        for (int k = 0; k < 12; ++k) red[k] = 0.0;
        double cgx[MGR > 0 ? MGR : 1];
#pragma unroll
        for (int r = 0; r < (MGR > 0 ? MGR : 1); ++r) cgx[r] = 0.0;
        if (act && inb) {
          const double qi = qs[e], x = xs[e], zb = zs[e], yb = ys[e];
          const double rb = sc[C_RB], dinv = sc[C_DINV];
          // this iteration's rhs (the expression that produced the pass-1 operand)
          double cgwp = 0.0;
#pragma unroll
          for (int r = 0; r < MGR; ++r) cgwp = fma(cgi[r], sc[C_WGP + r], cgwp);
          double rr0 = sigma * x - qi + cgwp;
          rr0 += rb * zb - yb;
          if constexpr (MODE == 0) {
            v = rr0 * dinv;
            red[0] = fabs(qi);
#pragma unroll
            for (int r = 0; r < MGR; ++r) {
              red[1 + r] = cgi[r] * mui;
              red[8 + r] = cgi[r] * v;
              cgx[r] = cgi[r] * x;
            }
            red[6] = mui * v;
          } else {
            const double px = pxs[e];
            const double xr = XV[ui * SW_PV + g] + XV[SW_SA * SW_PV + ui * SW_PV + g];
            double corr = xr - sc[C_SU] * mui;
#pragma unroll
            for (int r = 0; r < MGR; ++r) corr = fma(sc[C_CW + r], cgi[r], corr);
            const double xt = (rr0 - corr) * dinv;
            double pxt = rr0 - sigma * xt - rb * xt;
            double cgy = 0.0, cgw = 0.0;
#pragma unroll
            for (int r = 0; r < MGR; ++r) {
              pxt -= cgi[r] * sc[C_RGZ + r];
              cgy = fma(cgi[r], sc[C_YG + r], cgy);
              cgw = fma(cgi[r], sc[C_WG + r], cgw);
            }
            const double xn = alpha * xt + (1.0 - alpha) * x;
            const double pxn = alpha * pxt + (1.0 - alpha) * px;
            double rr = sigma * xn - qi + cgw;
            const double zh = alpha * xt + (1.0 - alpha) * zb;
            const double zn = fmin(fmax(fma(yb, sc[C_RBI], zh), lo), up);
            const double yn = yb + rb * (zh - zn);
#if PQ_SW_X != 1
            const unsigned ox = (unsigned)(b * ld + ia), oz = (unsigned)(b * st.m_ld + st.mg_pad + ia);
            st.z[oz] = zn;
            st.y[oz] = yn;
            st.x[ox] = xn;
            st.Px[ox] = pxn;
#endif
            rr += rb * zn - yn;
            red[0] = fabs(xn - zn);
            red[1] = fabs(xn);
            red[2] = fabs(zn);
            const double cy = yn + cgy;
            red[3] = fabs((pxn + qi + yn) + (cy - yn));
            red[4] = fabs(pxn);
            red[5] = fabs(cy);
            v = rr * dinv;
            red[6] = mui * v;
#pragma unroll
            for (int r = 0; r < MGR; ++r) red[8 + r] = cgi[r] * v;
          }
        }
        XV[ui * SW_PV + g] = v;   // the element this thread read (half 0), now v
        // residual terms / sums accumulate per thread over the chunk (reduced once, below):
        // the maxima and mu.v in this thread's own LDS slots, the general-row sums in registers.
        // |x|, |z| and |Px|, |C'y| only enter the test as max(|x|, |z|), max(|Px|, |C'y|, |q|)
        double* ra = racc_l + (2 * 0 + e) * SW_T + t;
        if constexpr (MODE == 1) {
          ra[0] = fmax(ra[0], red[0]);
          ra[2 * SW_T] = fmax(ra[2 * SW_T], fmax(red[1], red[2]));
          ra[4 * SW_T] = fmax(ra[4 * SW_T], red[3]);
          ra[6 * SW_T] = fmax(ra[6 * SW_T], fmax(red[4], red[5]));
          ra[8 * SW_T] += red[6];
#pragma unroll
          for (int r = 0; r < MGR; ++r) rcg[e][r] += red[8 + r];
        } else {
          ra[0] = fmax(ra[0], red[0]);
          ra[8 * SW_T] += red[6];
#pragma unroll
          for (int r = 0; r < MGR; ++r) {
            rcm[e][r] += red[1 + r];
            rcg[e][r] += red[8 + r];
            rcx[e][r] += cgx[r];
          }
        }
      }
    }
    __syncthreads();
    SW_STAMP(1);

    // ---- pass 1: W[u][g] += sum_i X[u][i] v[i][g] (window-row tiles 2w, 2w + 1) -------------
#pragma unroll
    for (int s2 = 0; s2 < SW_SA / 4; ++s2) {
      const int ii = 4 * s2 + k4;
      const double a0 = X[(32 * w + m16) * SW_PX + ii];
      const double a1 = X[(32 * w + 16 + m16) * SW_PX + ii];
      const double* vrow = XV + ii * SW_PV + m16;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const double bv = vrow[16 * c];
        if (PQ_SW_X == 5) {
          wacc[0][c][0] += a0 * bv;
          continue;
        }
        wacc[0][c] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, bv, wacc[0][c], 0, 0, 0);
        wacc[1][c] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, bv, wacc[1][c], 0, 0, 0);
      }
    }
    if (more) slab_store(cur ^ 1);
    __syncthreads();
    SW_STAMP(2);
    cur ^= 1;
  }

  // ---- chunk partials: W (problem-major rows of SW_K) and the per-problem sums --------------
  {
    double* wp = Wp + ((int64_t)(grp * nch + ch) * SW_G) * SW_K;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int r = 0; r < 4; ++r) wp[(16 * c + m16) * SW_K + 32 * w + 16 * a + k4 + 4 * r] = wacc[a][c][r];
    // the chunk's per-problem terms: 16-lane reductions of the per-thread partials, in the
    // partial-record layout (unused slots zero)
    double* rp = Rp + ((int64_t)(grp * nch + ch) * SW_G) * RP_N;
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int g = ug + 32 * e;
      double o[RP_N];
#pragma unroll
      for (int k = 0; k < RP_N; ++k) o[k] = 0.0;
      const double* ra = racc_l + e * SW_T + t;
      if constexpr (MODE == 1) {   // (slots 2 and 5 stay 0: merged into 1 and 4)
        o[0] = qmax16(ra[0]);
        o[1] = qmax16(ra[2 * SW_T]);
        o[3] = qmax16(ra[4 * SW_T]);
        o[4] = qmax16(ra[6 * SW_T]);
        o[6] = qsum16(ra[8 * SW_T]);
#pragma unroll
        for (int r = 0; r < MGR; ++r) o[8 + r] = qsum16(rcg[e][r]);
      } else {
        o[0] = qmax16(ra[0]);
        o[6] = qsum16(ra[8 * SW_T]);
#pragma unroll
        for (int r = 0; r < MGR; ++r) {
          o[1 + r] = qsum16(rcm[e][r]);
          o[8 + r] = qsum16(rcg[e][r]);
          o[12 + r] = qsum16(rcx[e][r]);
        }
      }
      if (ui == 0) {
#pragma unroll
        for (int k = 0; k < RP_N; ++k) rp[g * RP_N + k] = o[k];
      }
    }
#ifdef PQ_SW_PROF
    if (t == 0) {   // pass 2, updates, pass 1, setup (clock64 ticks) in problem 0's spare slots
      rp[7] = pclk[0];
      rp[13] = pclk[1];
      rp[14] = pclk[2];
      rp[15] = pclk[3];
    }
#endif
  }
}

// ---- per problem: convergence of iteration k, W, u = M^-1 kw, Ut, general rows of k + 1 -----
template <int MODE, int MGR>
__global__ __launch_bounds__(SW_MT) void k_sw_mid(pq_lowrank lr, pq_problem pb, pq_settings s,
                                                  const int32_t* gdates, int nch, double* SR, double* Ut,
                                                  const double* Wp, const double* Rp, const double* Minv_all,
                                                  int k_ld, int64_t M_stride, const double* pc, int64_t ldpc,
                                                  int r0, const double* cc) {
  __shared__ double kw[SW_K + 8];
  __shared__ double uv[SW_K + 8];
  __shared__ double s_dot[SW_K + 8];
  __shared__ double s_part[4 * SW_K];
  __shared__ double red[RP_N];
  __shared__ double sr[SR_N];
  __shared__ int s_cont;

  // XCD-contiguous slots: a group's problems on one XCD, so the 8-byte column writes of its Ut
  // merge in one L2 (and its chunk partials were written on the same XCD by k_sw_pass)
  const int slot = xcd_slot(blockIdx.x, gridDim.x);
  const int grp = slot / SW_G, g = slot - grp * SW_G;
  const int b0 = gdates[grp];
  if (g >= gdates[grp + 1] - b0) return;
  const int b = b0 + g;
  double* R = SR + (int64_t)b * SR_N;
  if (R[S_ACT] == 0.0) return;   // uniform
  const int t = threadIdx.x, w = t >> 6, l = t & 63;
  const int mg = pb.mg, tmax = lr.tmax, T = lr.tlen[b0];
  const int k = tmax + mg;
  static_assert(SW_MT == SW_K, "one window row per thread");

  // Every load that depends on nothing else is issued before the first barrier: the chunk
  // partials (residual terms, this thread's window row of W), this thread's row id and pc
  // entries, and the first M^-1 rows -- one HBM round trip instead of one per phase.
  const double* Mi = Minv_all + (int64_t)b * M_stride;
  constexpr int RU = PQ_SW_RU;   // rows per M^-1 load batch (two batches in flight)
  double m0[RU][4], m1[RU][4];
  // rows j = w + 4 e of this wave; lane l holds columns l + 64 q.  Blocks above the diagonal
  // block (and rows past k) load the diagonal block again (an L2 hit, no HBM bytes): every load
  // is unconditional, since a skipped load is an exec-masked branch whose zeroing of the
  // destination makes the compiler wait for all outstanding loads; the arithmetic masks c <= j
  auto rload = [&](double (&M)[RU][4], int j0) {
#pragma unroll
    for (int e = 0; e < RU; ++e) {
      const int j = j0 + 4 * e;
      const int jj = j < k ? j : 0;
      const double* rp = Mi + (int64_t)jj * k_ld + l;
#pragma unroll
      for (int q = 0; q < 4; ++q) M[e][q] = rp[64 * min(q, jj >> 6)];
    }
  };
  rload(m0, w);
  double Wj = 0.0;
  int rowj = 0;
  double pcv[MGR > 0 ? MGR : 1];
  {
    const int j = t;   // SW_MT == SW_K: one window row per thread
    {   // the chunk partials in chunk order, eight unconditional loads in flight (clamped to
        // the last chunk, added as 0 past it: the same sums)
      const double* wp = Wp + ((int64_t)grp * nch * SW_G + g) * SW_K + j;
      const int64_t cs = (int64_t)SW_G * SW_K;
      for (int c = 0; c < nch; c += 8) {
        double v[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = wp[min(c + e, nch - 1) * cs];
#pragma unroll
        for (int e = 0; e < 8; ++e) Wj += c + e < nch ? v[e] : 0.0;
      }
      if (j >= T) Wj = 0.0;
      rowj = lr.rows[(int64_t)b0 * tmax + (j < T ? j : 0)];
    }
#pragma unroll
    for (int r = 0; r < (MGR > 0 ? MGR : 1); ++r)
      pcv[r] = r < mg ? pc[(int64_t)(rowj - r0) * ldpc + r] : 0.0;   // (rows past T: times u = 0)
  }
  if (t < SR_N) sr[t] = R[t];
  if (t < RP_N) {   // four chunks' loads in flight at a time, combined in chunk order
    const bool is_max = MODE == 1 ? t < 6 : t == 0;
    const double* rp = Rp + ((int64_t)grp * nch * SW_G + g) * RP_N + t;
    const int64_t cs = (int64_t)SW_G * RP_N;
    double a = 0.0;
    for (int c = 0; c < nch; c += 8) {   // (as the chunk partials above)
      double v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = rp[min(c + e, nch - 1) * cs];
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (c + e < nch) a = is_max ? fmax(a, v[e]) : a + v[e];
    }
    red[t] = a;
  }
  __syncthreads();
  if (t == 0) {
    int cont = 1;
    if constexpr (MODE == 1) {
      const double mv0 = fmax(red[0], sr[S_RMV + 0]), mv1 = fmax(red[1], sr[S_RMV + 1]),
                   mv2 = fmax(red[2], sr[S_RMV + 2]);
      const double mv3 = red[3], mv4 = red[4], mv5 = red[5], mv6 = sr[S_QMAX];
      const double rho = sr[S_RHO];
      const int it = (int)sr[S_IT] + 1;
      int stat = PQ_UNSOLVED;
      const double eps_p = s.eps_abs + s.eps_rel * fmax(mv1, mv2);
      const double eps_d = s.eps_abs + s.eps_rel * fmax(mv4, fmax(mv5, mv6));
      double rnew = rho;
      if (it >= s.min_iter && mv0 <= eps_p && mv3 <= eps_d) {
        stat = PQ_SOLVED;
      } else if (s.adapt_interval > 0 && it % s.adapt_interval == 0) {
        const double rp = mv0 / (fmax(mv1, mv2) + 1e-30);
        const double rd = mv3 / (fmax(mv4, fmax(mv5, mv6)) + 1e-30);
        double rn = rho * sqrt(rp / (rd + 1e-30));
        rn = fmin(fmax(rn, s.rho_min), s.rho_max);
        if (rn > rho * s.adapt_tol || rn < rho / s.adapt_tol) {
          rnew = rn;
          stat = PQ_NEED_REFACTOR;
        }
      }
      if (stat == PQ_UNSOLVED && it >= s.max_iter) stat = PQ_MAX_ITER;
      cont = (stat == PQ_UNSOLVED) && it < (int)sr[S_END];
      R[S_IT] = it;
      R[S_RHO] = rnew;
      R[S_STAT] = stat;
      R[S_ACT] = cont;
      R[S_MUV] = red[6];
#pragma unroll
      for (int r = 0; r < SW_MG; ++r)
        if (r < mg) R[S_CGV + r] = sr[S_CGV + r] = red[8 + r];
    } else {
      R[S_QMAX] = red[0];
      R[S_MUV] = red[6];
#pragma unroll
      for (int r = 0; r < SW_MG; ++r)
        if (r < mg) {
          R[S_CMU + r] = sr[S_CMU + r] = red[1 + r];
          R[S_CGV + r] = sr[S_CGV + r] = red[8 + r];
          R[S_CGX + r] = sr[S_CGX + r] = red[12 + r];
        }
    }
    s_cont = cont;
  }
  __syncthreads();
  if (!s_cont) return;

  const double sps = sr[S_SPS], muv = red[6], dinv = sr[S_DINV];
  // kw = [sps (W - mu.v) over the window rows | sqrt(rho_r) Cg_r.v]
  {
    const int j = t;
    double a = 0.0;
    if (j < T) a = sps * (Wj - muv);
    else if (j >= tmax && j < k) a = sqrt(sr[S_RG + (j - tmax)]) * red[8 + (j - tmax)];
    kw[j] = a;
  }
  __syncthreads();

  // u = M^-1 kw (lower triangle, row pitch k_ld): a dot part per row (entries c <= j) and an
  // axpy part (c < j) in registers
  {
    double rv[4], acc[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int c = l + 64 * q;
      rv[q] = c < k ? kw[c] : 0.0;
      acc[q] = 0.0;
    }
    auto rblock = [&](const double (&M)[RU][4], int j0) {
      double dd[RU];
#pragma unroll
      for (int e = 0; e < RU; ++e) {
        const int j = j0 + 4 * e;
        const double a = j < k ? kw[j] : 0.0;
        double sd = 0.0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int c = l + 64 * q;
          sd = fma(c <= j ? M[e][q] : 0.0, rv[q], sd);
          acc[q] = fma(a, c < j ? M[e][q] : 0.0, acc[q]);
        }
        dd[e] = sd;
      }
#pragma unroll
      for (int e = 0; e < RU; ++e) dd[e] = wave_sum(dd[e]);
      if (l == 0) {
#pragma unroll
        for (int e = 0; e < RU; ++e) {
          const int j = j0 + 4 * e;
          if (j < k) s_dot[j] = dd[e];
        }
      }
    };
    for (int j0 = w; j0 < k; j0 += 8 * RU) {
      rload(m1, j0 + 4 * RU);
      rblock(m0, j0);
      rload(m0, j0 + 8 * RU);
      rblock(m1, j0 + 4 * RU);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) s_part[w * SW_K + l + 64 * q] = acc[q];
  }
  __syncthreads();
  {
    const int c = t;
    double u = 0.0;
    if (c < k) {
      u = s_dot[c];
#pragma unroll
      for (int ww = 0; ww < 4; ++ww) u += s_part[ww * SW_K + c];
    }
    uv[c] = u;
  }
  __syncthreads();

  // Ut column of this problem (zero outside the window rows), su, Cg x~ terms
  double su = 0.0, pcu[SW_MG] = {0.0, 0.0, 0.0, 0.0};
  {
    const int j = t;
    const double uu = j < T ? sps * uv[j] : 0.0;
    Ut[((int64_t)grp * SW_K + j) * SW_G + g] = uu;
    su = uu;
#pragma unroll
    for (int r = 0; r < MGR; ++r) pcu[r] = pcv[r] * uu;
  }
  su = wave_sum(su);
#pragma unroll
  for (int r = 0; r < MGR; ++r) pcu[r] = wave_sum(pcu[r]);
  if (l == 0) {
    s_part[w] = su;
#pragma unroll
    for (int r = 0; r < MGR; ++r) s_part[4 + 4 * r + w] = pcu[r];
  }
  __syncthreads();
  if (t == 0) {
    double sut = 0.0;
    for (int ww = 0; ww < 4; ++ww) sut += s_part[ww];
    R[S_SU] = sut;
    double cw[SW_MG] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int r = 0; r < MGR; ++r) {
      const double rg = sr[S_RG + r];
      cw[r] = r < mg ? sqrt(rg) * uv[tmax + r] : 0.0;
      R[S_CW + r] = cw[r];
    }
    double m0 = 0.0, m1 = 0.0, m2 = 0.0;
#pragma unroll
    for (int r = 0; r < MGR; ++r) {
      if (r >= mg) break;
      double a = 0.0;
      for (int ww = 0; ww < 4; ++ww) a += s_part[4 + 4 * r + ww];
      double cwr = 0.0;
      for (int r2 = 0; r2 < mg; ++r2) cwr = fma(cc[r * mg + r2], cw[r2], cwr);
      const double zt = sr[S_CGV + r] - dinv * (a - sut * sr[S_CMU + r] + cwr);
      const double rg = sr[S_RG + r], zg = sr[S_ZG + r], yg = sr[S_YG + r];
      const double zh = s.alpha * zt + (1.0 - s.alpha) * zg;
      const double zn = fmin(fmax(zh + yg / rg, sr[S_LG + r]), sr[S_UG + r]);
      const double yn = yg + rg * (zh - zn);
      const double cx = s.alpha * zt + (1.0 - s.alpha) * sr[S_CGX + r];
      m0 = fmax(m0, fabs(cx - zn));
      m1 = fmax(m1, fabs(cx));
      m2 = fmax(m2, fabs(zn));
      R[S_RGZ + r] = rg * zt;
      R[S_ZG + r] = zn;
      R[S_YG + r] = yn;
      R[S_CGX + r] = cx;
      R[S_WGP + r] = sr[S_WG + r];
      R[S_WG + r] = rg * zn - yn;
    }
    R[S_RMV + 0] = m0;
    R[S_RMV + 1] = m1;
    R[S_RMV + 2] = m2;
  }
}

// ---- any problem still iterating (one workgroup) ---------------------------------------------
__global__ __launch_bounds__(256) void k_sw_any(const int32_t* gdates, int ngroups, const double* SR, int* flag) {
  __shared__ int s_a;
  if (threadIdx.x == 0) s_a = 0;
  __syncthreads();
  const int b0 = gdates[0], b1 = gdates[ngroups];
  int a = 0;
  for (int b = b0 + threadIdx.x; b < b1; b += 256) a |= SR[(int64_t)b * SR_N + S_ACT] != 0.0;
  if (a) s_a = 1;   // benign race: every writer stores 1
  __syncthreads();
  if (threadIdx.x == 0) flag[0] = s_a;
}

// ---- write back the per-problem scalars and the general rows -----------------------------
__global__ __launch_bounds__(256) void k_sw_final(pq_problem pb, pq_state st, const int32_t* gdates, int ngroups,
                                                  const double* SR) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  const int grp = e / SW_G, g = e - grp * SW_G;
  if (grp >= ngroups) return;
  const int b0 = gdates[grp];
  if (g >= gdates[grp + 1] - b0) return;
  const int b = b0 + g;
  const double* R = SR + (int64_t)b * SR_N;
  if (R[S_ACT0] != 0.0) {
    st.iters[b] = (int)R[S_IT];
    st.status[b] = (int)R[S_STAT];
    st.rho[b] = R[S_RHO];
  }
  for (int r = 0; r < pb.mg; ++r) {
    st.z[(int64_t)b * st.m_ld + r] = R[S_ZG + r];
    st.y[(int64_t)b * st.m_ld + r] = R[S_YG + r];
  }
}

}  // namespace
}  // namespace pq

// Scratch of pq_admm_lr_sweep in doubles (per-problem records, chunk partials, Ut, a flag).
extern "C" int64_t pq_sweep_scratch_doubles(int32_t n, int32_t batch, int32_t ngroups) {
  const int64_t nch = (n + pq::SW_CH - 1) / pq::SW_CH;
  return (int64_t)batch * pq::SR_N + (int64_t)ngroups * nch * pq::SW_G * (pq::SW_K + pq::RP_N) +
         (int64_t)ngroups * pq::SW_K * pq::SW_G + 64;
}

extern "C" int pq_admm_lr_sweep(const pq_lowrank* lr, const pq_problem* pb, pq_state* st, const double* Minv,
                                int32_t k_ld, int64_t M_stride, const int32_t* gdates, int32_t ngroups,
                                const pq_settings* s, int32_t iters_this_call, const double* pc, int64_t ldpc,
                                int32_t r0, const double* cc, int32_t q_shared, double* scratch,
                                int64_t scratch_doubles, void* stream) {
  PQ_CHECK_ARG(lr && pb && st && s && Minv && gdates && scratch, "pq_admm_lr_sweep: null argument");
  PQ_CHECK_ARG(lr->panel && lr->rows && lr->tlen && lr->tmax > 0 && lr->tmax <= pq::SW_K,
               "pq_admm_lr_sweep: needs a window of at most %d rows (tmax=%d)", pq::SW_K, lr->tmax);
  PQ_CHECK_ARG(pb->mg >= 0 && pb->mg <= pq::SW_MG && (pb->mg == 0 || (pb->Cg && pb->lg && pb->ug && pc && cc)),
               "pq_admm_lr_sweep: needs 0 <= mg <= %d shared general rows with pc / cc (mg=%d)", pq::SW_MG, pb->mg);
  PQ_CHECK_ARG(pb->mg == 0 || pb->Cg_stride == 0, "pq_admm_lr_sweep: the general rows must be shared");
  PQ_CHECK_ARG(pb->lb && pb->ub && pb->box_stride == 0, "pq_admm_lr_sweep: needs shared box rows");
  PQ_CHECK_ARG((int64_t)pb->batch * (st->m_ld > pb->ld ? st->m_ld : pb->ld) < (int64_t)1 << 31 &&
                   (int64_t)pb->batch * pb->q_stride < (int64_t)1 << 31,
               "pq_admm_lr_sweep: state arrays beyond 32-bit element offsets");
  const int k = lr->tmax + pb->mg;
  PQ_CHECK_ARG(k <= k_ld && k_ld <= pq::SW_K, "pq_admm_lr_sweep: need k <= k_ld <= %d (k=%d)", pq::SW_K, k);
  PQ_CHECK_ARG(scratch_doubles >= pq_sweep_scratch_doubles(pb->n, pb->batch, ngroups),
               "pq_admm_lr_sweep: scratch too small");
  if (ngroups <= 0 || iters_this_call <= 0) return 0;
  hipStream_t str = (hipStream_t)stream;
  const int nch = (pb->n + pq::SW_CH - 1) / pq::SW_CH;
  double* SR = scratch;
  double* Wp = SR + (int64_t)pb->batch * pq::SR_N;
  double* Rp = Wp + (int64_t)ngroups * nch * pq::SW_G * pq::SW_K;
  double* Ut = Rp + (int64_t)ngroups * nch * pq::SW_G * pq::RP_N;
  int* flag = reinterpret_cast<int*>(Ut + (int64_t)ngroups * pq::SW_K * pq::SW_G);
  const int nslot = ngroups * pq::SW_G;
  PQ_CHECK_HIP(hipMemsetAsync(Ut, 0, sizeof(double) * (size_t)ngroups * pq::SW_K * pq::SW_G, str));
  hipLaunchKernelGGL(pq::k_sw_setup, dim3((nslot + 255) / 256), dim3(256), 0, str, *lr, *pb, *st, *s, gdates, ngroups,
                     SR, (int)iters_this_call);
  const bool mg1 = pb->mg <= 1;
  auto pass = [&](int mode) {
    const dim3 grid(ngroups * nch), blk(pq::SW_T);
    if (mode == 0) {
      if (mg1) hipLaunchKernelGGL((pq::k_sw_pass<0, 1>), grid, blk, 0, str, *lr, *pb, *st, *s, gdates, nch, SR, Ut, Wp, Rp, (int)q_shared);
      else hipLaunchKernelGGL((pq::k_sw_pass<0, 4>), grid, blk, 0, str, *lr, *pb, *st, *s, gdates, nch, SR, Ut, Wp, Rp, (int)q_shared);
    } else {
      if (mg1) hipLaunchKernelGGL((pq::k_sw_pass<1, 1>), grid, blk, 0, str, *lr, *pb, *st, *s, gdates, nch, SR, Ut, Wp, Rp, (int)q_shared);
      else hipLaunchKernelGGL((pq::k_sw_pass<1, 4>), grid, blk, 0, str, *lr, *pb, *st, *s, gdates, nch, SR, Ut, Wp, Rp, (int)q_shared);
    }
  };
  auto mid = [&](int mode) {
    const dim3 grid(nslot), blk(pq::SW_MT);
#define PQ_SW_MID(MD, MG)                                                                                     \
  hipLaunchKernelGGL((pq::k_sw_mid<MD, MG>), grid, blk, 0, str, *lr, *pb, *s, gdates, nch, SR, Ut, Wp, Rp, Minv, \
                     k_ld, M_stride, pc, ldpc, r0, cc)
    if (mode == 0) {
      if (mg1) PQ_SW_MID(0, 1); else PQ_SW_MID(0, 4);
    } else {
      if (mg1) PQ_SW_MID(1, 1); else PQ_SW_MID(1, 4);
    }
#undef PQ_SW_MID
  };
  pass(0);
  mid(0);
  // iterations in blocks; one flag read between blocks (the first block covers the usual
  // loose-stop run, later blocks are short)
  int done = 0, blockn = 12;
  while (done < iters_this_call) {
    const int nb = blockn < iters_this_call - done ? blockn : iters_this_call - done;
    for (int j = 0; j < nb; ++j) {
      pass(1);
      mid(1);
    }
    done += nb;
    blockn = 4;
    if (done >= iters_this_call) break;
    hipLaunchKernelGGL(pq::k_sw_any, dim3(1), dim3(256), 0, str, gdates, ngroups, SR, flag);
    int h = 0;
    PQ_CHECK_HIP(hipMemcpyAsync(&h, flag, sizeof(int), hipMemcpyDeviceToHost, str));
    PQ_CHECK_HIP(hipStreamSynchronize(str));
    if (!h) break;
  }
  hipLaunchKernelGGL(pq::k_sw_final, dim3((nslot + 255) / 256), dim3(256), 0, str, *pb, *st, gdates, ngroups, SR);
  PQ_CHECK_LAUNCH("pq_admm_lr_sweep");
  return 0;
}
