/*
 * porqua_hip.h -- C ABI of the MI355X (gfx950) engine for PorQua's backtest hot path.
 *
 * The reference (amolrpatil21/PorQua) is pure Python; each rebalance date estimates a
 * covariance / Gram matrix and hands one dense QP to the third-party `qpsolvers`.
 * This library replaces that per-date arithmetic with batched HIP kernels.  Every entry
 * point names the reference interface it stands in for.  Conventions:
 *   - all matrices FP64 row-major, device pointers owned by the caller (PyTorch-ROCm);
 *   - square per-problem matrices use a leading dimension `ld` = round_up(n, 64) with a
 *     zero-filled padding region; per-problem vectors use stride `ld` as well;
 *   - `stream` is a hipStream_t passed as void*;  return 0 on success, < 0 on an
 *     argument / HIP error (message via pq_last_error());  nothing throws across the ABI;
 *   - the library allocates nothing persistent and keeps no global mutable state besides
 *     the thread-local error string (reentrant; one device per call = the current one).
 */
#ifndef PORQUA_HIP_H
#define PORQUA_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PQ_VERSION 100

/* per-problem status codes (pq_state.status) */
#define PQ_UNSOLVED 0
#define PQ_SOLVED 1             /* ADMM converged and the polished point passed its checks */
#define PQ_SOLVED_INACCURATE 2  /* ADMM converged, polish rejected: ADMM point returned   */
#define PQ_MAX_ITER 3
#define PQ_NEED_REFACTOR 4      /* internal: adaptive rho asks for a new K^-1            */
#define PQ_PRIMAL_INFEASIBLE (-3)
#define PQ_DUAL_INFEASIBLE (-4)
#define PQ_NON_CONVEX (-5)      /* KKT Cholesky failed                                   */

/* per-problem output record (pq_state.out, PQ_OUT_FIELDS doubles each) */
#define PQ_OUT_OBJ 0        /* 0.5 x'Px + q'x (no constant; test:72,82)               */
#define PQ_OUT_PRIM 1       /* qpsolvers primal_residual()                              */
#define PQ_OUT_DUAL 2       /* qpsolvers dual_residual()                                */
#define PQ_OUT_GAP 3        /* qpsolvers duality_gap()                                  */
#define PQ_OUT_RHO 4
#define PQ_OUT_NFREE 5      /* variables strictly inside their box after polish         */
#define PQ_OUT_ROUNDS 6     /* polish active-set rounds                                 */
#define PQ_OUT_FIELDS 8

/* polish scratch per problem (doubles): xs | xb | g | Px | 4 Woodbury-mode vectors |
 * U (mg_pad rows) | flags (ld int32) | 512 spare (PQ_PROFILE phase timers at PQ_WORK_PROF) */
#define PQ_WORK_DOUBLES(ld, mg_pad) ((int64_t)(9 + (mg_pad)) * (ld) + 512)
#define PQ_WORK_PROF(ld, mg_pad) ((int64_t)(9 + (mg_pad)) * (ld))

/* A batch of dense QPs   min 0.5 x'Px + q'x  s.t.  lg <= Cg x <= ug,  lb <= x <= ub
 * (the QuadraticProgram fields P, q, G, h, A, b, lb, ub of src/qp_problems.py:34-38 with
 * A / G stacked into Cg: equality rows have lg == ug, G rows have lg = -inf).
 * Effective P = p_scale[b] * P_b + p_diag[b] * I (p_scale / p_diag may be NULL).     */
typedef struct pq_problem {
  int32_t n, ld, batch, mg;
  const double* P;   int64_t P_stride;
  const double* p_scale;
  const double* p_diag;
  const double* q;   int64_t q_stride;
  const double* Cg;  int64_t Cg_stride;   /* mg x ld per problem; stride 0 = shared   */
  const double* lg;  const double* ug;  int64_t g_stride;    /* mg; stride 0 = shared */
  const double* lb;  const double* ub;  int64_t box_stride;  /* ld; NULL = unbounded   */
} pq_problem;

/* Solver state / workspace, all device memory, indexed by problem id b < batch.       */
typedef struct pq_state {
  double* K;     int64_t K_stride;      /* ld x ld: KKT -> L -> K^-1 -> polish scratch  */
  double* Dt;    int64_t Dt_stride;     /* (ld/64) x 64 x 64 transposed diag-block inverses */
  double* x;     double* Px;            /* ld per problem                                 */
  double* z;     double* y;             /* m_ld per problem: Cg rows at [0,mg), box at [mg_pad, mg_pad+n) */
  int32_t m_ld, mg_pad;
  double* rho;                          /* per problem                                    */
  int32_t* iters; int32_t* status; int32_t* info;
  double* out;                          /* PQ_OUT_FIELDS per problem                      */
  double* work;  int64_t work_stride;   /* >= PQ_WORK_DOUBLES(ld, mg_pad) per problem      */
} pq_state;

/* rho0_rel > 0: the initial rho of problem b is rho0_rel * mean(diag(P_eff_b)) (clamped to
 * [rho_min, rho_max]) instead of rho0 -- one scale-aware value per problem.           */
typedef struct pq_settings {
  double rho0, rho0_rel, sigma, alpha, eps_abs, eps_rel, rho_min, rho_max, adapt_tol, eq_scale,
      delta, dual_tol;
  int32_t max_iter, adapt_interval, polish, polish_rounds, refine_iters;
  /* grouped polish (pq_polish_grouped_init), centred windows: a variable also starts fixed at
   * its lower bound when x - lb < polish_fix_rel * max_j (x_j - lb_j) at the ADMM point
   * (0: OSQP's rule alone) */
  double polish_fix_rel;
  /* grouped polish, LDS solve: free variables the solve leaves outside their box are fixed at
   * that bound and the reduced system solved again inside the same round, at most this many
   * times (0: one solve per round, the checks of the round's end fix them) */
  int32_t polish_inner;
  /* ADMM: the convergence test is skipped before this iteration (0: tested from the first).
   * The loose stop before the grouped polish uses it so that an early dip of the residuals
   * (ADMM's are not monotone) cannot end the iterations before the active set is predicted */
  int32_t min_iter;
  /* grouped polish: when a round's answer is rejected anyway, variables at a bound whose
   * multiplier is within polish_release_rel * (problem scale) of the wrong sign are released
   * too (0: only the wrong-sign ones) -- the next round's free set anticipates the shift, and
   * the solve's inner primal step fixes those that were right after all */
  double polish_release_rel;
} pq_settings;

/* Low-rank description of P for T < n (the backtest path): P_eff = p_scale[b] *
 * w_scale[b] * Xc'Xc + p_diag[b] * I, Xc = the T x n window of the panel
 * (rows[b][0..tlen[b])) centred by mu (mu == NULL: uncentred Gram, the LeastSquares case);
 * w_scale (NULL = 1) is 1/(T-1) when pq_problem.P holds the covariance of the same window.
 * With D = diag(sigma + p_diag + rho_box) and
 * U' = [sqrt(p_scale w_scale) Xc' | sqrt(rho_r) Cg_r'] (n x k, k = tmax + mg) the ADMM
 * system is K = D + U'U, so K^-1 = D^-1 - D^-1 U' M^-1 U D^-1 with the k x k capacitance
 * matrix M = I + U D^-1 U' (Woodbury): no n x n matrix is formed or factored.
 * dg (stride dg_stride, from pq_window_sumsq) is diag(Xc'Xc) per date: the diagonal of P
 * that pq_init_state_lr and pq_polish_w_batched need without P itself.                  */
typedef struct pq_lowrank {
  const double* panel; int64_t ldp;
  const int32_t* rows; const int32_t* tlen; int32_t tmax;
  const double* mu; int64_t mu_stride;
  const double* w_scale;
  const double* dg; int64_t dg_stride;
} pq_lowrank;

int pq_version(void);
const char* pq_last_error(void);

/* Column means of each date's window (rows[b][0..tlen[b]) of the panel) -- the first pass
 * of np.cov's two-pass algorithm behind DataFrame.cov() (src/covariance.py:65-66).      */
int pq_window_mean(const double* panel, int64_t ldp, int32_t n, const int32_t* rows,
                   const int32_t* tlen, int32_t tmax, int32_t batch, double* mu,
                   int64_t mu_stride, void* stream);

/* Column sums of squared deviations sum_t (X_ti - mu_i)^2 of each window (mu == NULL:
 * sum_t X_ti^2): diag(Xc'Xc), i.e. (T - 1) times the variances of Covariance.estimate
 * (src/covariance.py:65-66) or the Gram diagonal of LeastSquares (src/optimization.py:215).
 * Second pass of the two-pass moments over the same (L2-resident) window rows.        */
int pq_window_sumsq(const double* panel, int64_t ldp, int32_t n, const int32_t* rows,
                    const int32_t* tlen, int32_t tmax, int32_t batch, const double* mu,
                    int64_t mu_stride, double* out, int64_t out_stride, void* stream);

/* Both moments above for the dates of slide groups (engine.GroupPlan: date b's window is
 * union[uoff[b], uoff[b] + tlen[b]) of its group's union rows urows[g][0..umax), offsets
 * nondecreasing, one window length per group), in one pass: the first window summed, the
 * later ones by the rows that enter / leave (shifted sums; matches the two calls to a few
 * ulps).  Replaces pq_window_mean + pq_window_sumsq for the daily backtest
 * (src/covariance.py:65-66 per rebalance date of src/backtest.py:209-230).             */
int pq_window_moments_grouped(const double* panel, int64_t ldp, int32_t n, const int32_t* gdates,
                              int32_t ngroups, const int32_t* urows, int32_t umax,
                              const int32_t* uoff, const int32_t* tlen, double* mu,
                              int64_t mu_stride, double* dg, int64_t dg_stride, void* stream);

/* Windows with missing values (NaN): column means over the present rows (NaN when none)
 * -- the shift passed to pq_cov_pairwise_batched; geometric != 0: exp(mean log(1 + x)) - 1
 * over the present rows (MeanEstimator.estimate_geometric, src/mean_estimation.py:39-48,
 * pandas skipna).                                                                          */
int pq_window_nanmean(const double* panel, int64_t ldp, int32_t n, const int32_t* rows,
                      const int32_t* tlen, int32_t tmax, int32_t batch, double* mu, int64_t mu_stride,
                      int32_t geometric, void* stream);

/* pandas' pairwise-complete covariance, the result of DataFrame.cov() on a window with NaN
 * (src/covariance.py:65-66): entry (i, j) from the rows where both are present, with their
 * pairwise means and N_ij - 1 degrees of freedom; NaN when N_ij < 2.  Four masked FP64-MFMA
 * Grams per 64x64 tile (N = M'M, X~'M, M'X~, X~'X~; X~ shifted by `shift`, may be NULL).
 * out: batch x ld x ld, full symmetric, padding zero.                                    */
int pq_cov_pairwise_batched(const double* panel, int64_t ldp, int32_t n, const int32_t* rows,
                            const int32_t* tlen, int32_t tmax, int32_t batch, const double* shift,
                            int64_t shift_stride, double* out, int32_t ld, int64_t out_stride,
                            void* stream);

/* K1: batched windowed SYRK on FP64 MFMA.  mode 0: centred covariance with ddof=1
 * (Covariance.estimate 'pearson', src/covariance.py:40-56,65-66); mode 1: uncentred Gram
 * X'X (LeastSquares.set_objective, src/optimization.py:215).  out: batch x ld x ld.     */
int pq_cov_batched(const double* panel, int64_t ldp, int32_t n, const int32_t* rows,
                   const int32_t* tlen, int32_t tmax, int32_t batch, int32_t mode,
                   const double* mu, int64_t mu_stride, double* out, int32_t ld,
                   int64_t out_stride, void* stream);

/* K1 for overlapping windows (the same outputs as pq_cov_batched): dates are cut into
 * ngroups groups [gstart[g], gstart[g+1]); the first date of a group is a full SYRK, and
 * every later date d must hold the window of date d-1 shifted by shift[d] >= 1 rows
 * (rows[d][0..T-s) == rows[d-1][s..T), equal tlen), which is applied as a rank-2s MFMA
 * update: 2 s n^2 instead of 2 T n^2 flops per date.  The host builds the plan
 * (porqua_amd.engine.slide_plan).  lower_only != 0 writes the lower 64x64 tiles and the
 * full diagonal tiles only (LAPACK uplo = 'L' storage: half the bytes), which is all the
 * low-rank path reads.                                                                  */
int pq_cov_slide_batched(const double* panel, int64_t ldp, int32_t n, const int32_t* rows,
                         const int32_t* tlen, int32_t tmax, int32_t batch, int32_t mode,
                         const double* mu, int64_t mu_stride, double* out, int32_t ld,
                         int64_t out_stride, const int32_t* gstart, int32_t ngroups,
                         const int32_t* shift, int32_t lower_only, void* stream);

/* X'y and y'y of each window (LeastSquares q = -2 X'y, constant = y'y,
 * src/optimization.py:216-217).                                                        */
int pq_gram_xy_grouped(const double* panel, int64_t ldp, int32_t n, const double* bm, const int32_t* gdates,
                       int32_t ngroups, const int32_t* urows, int32_t umax, const int32_t* uoff,
                       const int32_t* tlen, double* xty, int64_t xty_stride, double* yty, double* dg,
                       int64_t dg_stride, void* stream);
/* (pq_gram_xy_grouped: the same for the dates of slide groups -- the layout of
 * pq_window_moments_grouped -- the first window summed, the later ones by the rows that
 * enter / leave: O(n) per date after the group's first instead of O(T n).  dg (optional):
 * diag(X'X) of every window in the same pass, the uncentred Gram diagonal of the window
 * form (src/optimization.py:215), instead of a separate pq_window_sumsq.)               */
int pq_gram_xy_batched(const double* panel, int64_t ldp, int32_t n, const double* bm,
                       const int32_t* rows, const int32_t* tlen, int32_t tmax, int32_t batch,
                       double* xty, int64_t xty_stride, double* yty, void* stream);

/* Geometric mean exp(mean(log1p X)) - 1 over each window (MeanEstimator.estimate_geometric,
 * src/mean_estimation.py:39-48).                                                       */
int pq_window_geomean(const double* panel, int64_t ldp, int32_t n, const int32_t* rows,
                      const int32_t* tlen, int32_t tmax, int32_t batch, double* mu,
                      int64_t mu_stride, void* stream);
/* The same for the dates of slide groups (the layout of pq_window_moments_grouped): the
 * first window's sum of log(1 + x) directly, the later ones by the rows that enter / leave
 * (T + 2 (G - 1) logarithms per column and group instead of G T).  Replaces
 * pq_window_geomean for the daily mean-variance backtest (src/optimization.py:157-177,
 * per rebalance date of src/backtest.py:209-230).                                        */
int pq_window_geomean_grouped(const double* panel, int64_t ldp, int32_t n, const int32_t* gdates,
                              int32_t ngroups, const int32_t* urows, int32_t umax,
                              const int32_t* uoff, const int32_t* tlen, double* mu,
                              int64_t mu_stride, void* stream);

/* Reset x, z, y, Px, iterations, status and set the initial rho (rho0, or rho0_rel times
 * the mean diagonal of P_eff) for problems idx[].                                      */
int pq_init_state(const pq_problem* pb, pq_state* st, const int32_t* idx, int32_t nidx,
                  const pq_settings* s, void* stream);

/* pq_init_state for the window form: P is not read (pb->P may be NULL); the initial rho
 * uses mean(diag P_eff) = mean(p_scale w_scale dg + p_diag).                           */
int pq_init_state_lr(const pq_lowrank* lr, const pq_problem* pb, pq_state* st, const int32_t* idx,
                     int32_t nidx, const pq_settings* s, void* stream);

/* K2: form K = P_eff + sigma I + Cg' R Cg + R_box for the current rho, factor it with a
 * batched blocked Cholesky on FP64 MFMA (info[] = first failing column + 1, the isPD test
 * of src/helper_functions.py:61-67), and if `invert` overwrite K with K^-1 (trtri+lauum):
 * invert = 1 writes the lower triangle only (what pq_admm_batched reads), invert = 2 the
 * full symmetric matrix.  With mg = 0, lb = ub = NULL and sigma = 0 this is a plain
 * batched potrf of P_eff.                                                              */
int pq_factor_batched(const pq_problem* pb, pq_state* st, const int32_t* idx, int32_t nidx,
                      const pq_settings* s, int32_t invert, void* stream);

/* K2L: pq_factor_batched for LARGE problems (the per-QP drop-in at thousands of assets:
 * QuadraticProgram.solve with a dense n x n P, src/qp_problems.py:184-216, called per date by
 * the serial Backtest.run, src/backtest.py:185-199).  Same K formation, info[] / status and
 * invert semantics, but each problem is spread over many workgroups (one 64 x 64 tile each):
 * right-looking blocked potrf (diagonal block, panel, trailing update launches per block
 * column), then trtri into `scratch` (L^-1, ld x ld per launch slot: problem idx[i] uses
 * scratch + i * scratch_stride) and lauum back into K.  scratch may be NULL when invert = 0. */
int pq_factor_large(const pq_problem* pb, pq_state* st, const int32_t* idx, int32_t nidx,
                    const pq_settings* s, int32_t invert, double* scratch, int64_t scratch_stride,
                    void* stream);

/* K3: up to `iters_this_call` OSQP-style ADMM iterations per problem idx[] (stops a
 * problem at convergence, at settings.max_iter, or when adaptive rho requests a
 * refactorisation: status PQ_NEED_REFACTOR and rho[] already updated).
 * Replaces qpsolvers.solve_problem (src/qp_problems.py:211-214).                        */
int pq_admm_batched(const pq_problem* pb, pq_state* st, const int32_t* idx, int32_t nidx,
                    const pq_settings* s, int32_t iters_this_call, void* stream);

/* Low-rank K2: capacitance matrices M_b = I + U D^-1 U' (lower 64x64 tiles, k_ld =
 * round_up(tmax + mg, 64)) for the current rho[], as an MFMA SYRK over the n assets.
 * Factor / invert them with pq_factor_batched on a pq_problem {n = k_ld, P = M}.       */
int pq_lr_capacitance(const pq_lowrank* lr, const pq_problem* pb, const pq_state* st,
                      const int32_t* idx, int32_t nidx, const pq_settings* s, double* M,
                      int32_t k_ld, int64_t M_stride, void* stream);

/* Low-rank K2, band-Gram form, for a uniform ADMM diagonal D = c I (every box row of a
 * problem has the same rho: all bounds finite with lb < ub, or all free, or all fixed --
 * the caller checks) and general rows shared by all problems (Cg_stride == 0):
 *   pq_lr_band_gram: band[r][j] = x_{r0+r} . x_{r0+r-j} for 0 <= j < W (W >= the widest
 *     window span in rows) -- an FP64 MFMA SYRK over the assets, once per panel instead
 *     of T^2 n per date -- and pc[r][g] = x_{r0+r} . Cg_g;
 *   pq_lr_capacitance_band: the same M as pq_lr_capacitance, assembled per date from the
 *     band (centring B - r1' - 1r' + s11' by the window's own mean: lr->mu must be the
 *     pq_window_mean of the same rows, or NULL), pc and cc = Cg Cg' (mg x mg).          */
int pq_lr_band_gram(const double* panel, int64_t ldp, int32_t n, int32_t r0, int32_t nrows, int32_t W,
                    double* band, int64_t ldo, const double* Cg, int32_t mg, int32_t ld_cg, double* pc,
                    int64_t ldpc, void* stream);
int pq_lr_capacitance_band(const pq_lowrank* lr, const pq_problem* pb, const pq_state* st, const int32_t* idx,
                           int32_t nidx, const pq_settings* s, const double* band, int64_t ldo, int32_t r0,
                           const double* pc, int64_t ldpc, const double* cc, double* M, int32_t k_ld,
                           int64_t M_stride, void* stream);

/* Low-rank K3: the ADMM of pq_admm_batched with x~ = K^-1 rhs applied through the window
 * (two passes over its T rows) and the lower-triangle M^-1 (Minv, k_ld x k_ld).        */
int pq_admm_lr_batched(const pq_lowrank* lr, const pq_problem* pb, pq_state* st,
                       const double* Minv, int32_t k_ld, int64_t M_stride, const int32_t* idx,
                       int32_t nidx, const pq_settings* s, int32_t iters_this_call, void* stream);

/* Low-rank K3 for groups of up to 16 consecutive dates whose windows slide over one union
 * of panel rows (engine.GroupPlan): group g holds dates [gdates[g], gdates[g+1]), its
 * union rows are urows[g * umax + u] (u < ucnt[g] <= 320) and date b's window is union
 * rows [uoff[b], uoff[b] + tlen[b]).  One workgroup per group runs the dates' iterations
 * in lock step with both window passes as FP64 MFMA GEMMs over the union; results are
 * those of pq_admm_lr_batched up to summation order.  Optional pc / cc (the tables of
 * pq_lr_band_gram: pc[r - r0][g] = x_r . Cg_g, cc = Cg Cg'; NULL = off) select the fused
 * form for a uniform ADMM diagonal (the pq_lr_capacitance_band condition) and mg <= 4:
 * Cg x~ from scalars, one pass over each date's vectors per iteration.  Needs even n and ldp, mg <= 32,
 * k_ld <= 384, work_stride >= 3 ld (work holds each date's V / rhs / x~ scratch).      */
int pq_admm_lr_grouped(const pq_lowrank* lr, const pq_problem* pb, pq_state* st, const double* Minv,
                       int32_t k_ld, int64_t M_stride, const int32_t* gdates, int32_t ngroups,
                       const int32_t* urows, const int32_t* ucnt, const int32_t* uoff, int32_t umax,
                       const pq_settings* s, int32_t iters_this_call, const double* pc, int64_t ldpc,
                       int32_t r0, const double* cc, const int32_t* cg_nzr, const double* cg_nzv,
                       int32_t nzmax, void* stream);
/* cg_nzr / cg_nzv (nzmax > 0; shared Cg with more than 4 rows): the nonzeros of each column
 * of Cg, row ids (-1 padded) and values, nzmax per column (e.g. the budget row plus one
 * sector-membership row per asset: nzmax = 2); the per-asset row sums of the updates then
 * read nzmax entries instead of mg.                                                      */

/* Risk-aversion sweep form of the fused pq_admm_lr_grouped (admm_sweep.hip): group g holds
 * problems [gdates[g], gdates[g+1]) (at most 64) that share ONE window and its centring (the
 * risk-aversion row of a date: P_b = p_scale[b] w_scale[b] Xc'Xc, own rho and M_b^-1 each).
 * An iteration is two chip-wide launches -- one workgroup per (group, 256-asset chunk) for
 * pass 2, the updates, the next rhs and its pass-1 partial (the window chunk read once for
 * all problems of the group), then one per problem for the M_b^-1 symv -- instead of one
 * workgroup per group.  Same iterates as the fused pq_admm_lr_grouped up to summation
 * order; one flag read between blocks of iterations.  Needs tmax <= 256, k_ld <= 256, shared
 * general rows mg <= 4 with pc / cc (mg > 0), shared box rows, uniform ADMM diagonal, and
 * scratch_doubles >= pq_sweep_scratch_doubles(n, batch, ngroups).  q_shared != 0: the problems
 * of a group share q too (q_b = -mu_d for every risk aversion), read from the group's first
 * problem.  Replaces
 * qpsolvers.solve_problem (src/qp_problems.py:211-214) for the sweep of
 * src/optimization.py:168-174 over risk aversions.                                       */
int pq_admm_lr_sweep(const pq_lowrank* lr, const pq_problem* pb, pq_state* st, const double* Minv,
                     int32_t k_ld, int64_t M_stride, const int32_t* gdates, int32_t ngroups,
                     const pq_settings* s, int32_t iters_this_call, const double* pc, int64_t ldpc,
                     int32_t r0, const double* cc, int32_t q_shared, double* scratch, int64_t scratch_doubles,
                     void* stream);
int64_t pq_sweep_scratch_doubles(int32_t n, int32_t batch, int32_t ngroups);

/* Group capacitance (admm_gcap.hip): the dates of each slide group (same T, same
 * c = p_scale w_scale, same p_diag, one shared rho grho[g]) share ONE capacitance matrix of
 * the union of their windows, M_U = I + W_U W_U' / d with W_U = [sqrt(c) X_U; sqrt(R) Cg]
 * (raw union rows; (U + mg) x (U + mg), general rows after the U union rows, identity
 * padding to k_ld), and each date applies its own K_b^-1 through a rank-(U - T + 1)
 * Woodbury correction (the union rows outside its window and its mean):
 *   pq_gcap_assemble   M_U per group from the band Gram (W >= the widest union span), pc, cc;
 *   (pq_factor_batched on {n = k, ld = k_ld, P = M, batch = ngroups}, invert = 2 -> Minv)
 *   pq_gcap_prepare    per date a_b = W_U mu_b, q_b = M_U^-1 a_b (aq: a | q, 2 k_ld each)
 *                      and H_b^-1 (ldh x ldh, ldh >= U - T + 1 <= 64); one workgroup per
 *                      group (idx, nidx: a subset of GROUPS, or NULL for all);
 *   pq_admm_lr_gcap    the fused grouped ADMM (pq_admm_lr_grouped with pc / cc) with the
 *                      per-date M_b^-1 symv replaced by one MFMA GEMM with M_U^-1 per
 *                      group plus the small per-date correction.  Adaptive rho is decided
 *                      per group (NEED_REFACTOR for all its running dates, grho updated).
 * Centred windows (lr->mu != NULL: MeanVariance) or uncentred (lr->mu == NULL: the
 * LeastSquares tracking of src/optimization.py:206-226, no mean column), shared general rows
 * (mg <= 4 register-resident; 4 < mg <= 24 in the column-sparse form cg_nzr / cg_nzv with
 * nzmax <= 4, as for pq_admm_lr_grouped; U + mg <= 320), uniform ADMM diagonal.
 * Replaces qpsolvers.solve_problem (src/qp_problems.py:211-214) for the batched backtest. */
typedef struct pq_gcap {
  const int32_t* gdates; int32_t ngroups;
  const int32_t* urows; const int32_t* ucnt; const int32_t* uoff; int32_t umax;
  const int32_t* gidx;          /* group of each date                                    */
  double* grho;                 /* rho of each group                                     */
  double* M; double* Minv; int32_t k_ld; int64_t M_stride;    /* per group                */
  double* aq; int64_t aq_stride;                               /* per date: a | q          */
  double* hinv; int32_t ldh;                                   /* per date: ldh x ldh      */
  int32_t gmax;                 /* dates in the largest group: 0..16 -> 16-date kernels;
                                   17..32 -> the 32-date form (one 512-thread workgroup per
                                   group; register-resident or column-sparse general rows) */
} pq_gcap;
int pq_gcap_assemble(const pq_lowrank* lr, const pq_problem* pb, const pq_gcap* gc, const pq_settings* s,
                     const double* band, int64_t ldo, int32_t r0, const double* pc, int64_t ldpc,
                     const double* cc, void* stream);
int pq_gcap_prepare(const pq_lowrank* lr, const pq_problem* pb, pq_state* st, const pq_gcap* gc,
                    const pq_settings* s, const int32_t* idx, int32_t nidx, const double* band, int64_t ldo,
                    int32_t r0, const double* pc, int64_t ldpc, void* stream);
int pq_admm_lr_gcap(const pq_lowrank* lr, const pq_problem* pb, pq_state* st, const pq_gcap* gc,
                    const pq_settings* s, int32_t iters_this_call, const double* pc, int64_t ldpc, int32_t r0,
                    const double* cc, const int32_t* cg_nzr, const double* cg_nzv, int32_t nzmax, void* stream);

/* K2, eigen form (the risk-aversion x date sweep, BASELINE configs[4]): M_b^-1 of every
 * problem b (or idx[0..nidx)) of the window path from ONE symmetric eigendecomposition per
 * date d = pdate[b] of the centred window Gram Xc_d Xc_d' = V diag(evals) V' instead of a
 * Cholesky factorisation per problem: V (k_ld x k_ld per date, row-major, V[i][k] = entry i
 * of eigenvector k, zero beyond tmax), evals (k_ld per date), What = V' Xc_d Cg' (k_ld x 4
 * per date), cc = Cg Cg' (mg x mg).  Every window has tlen == tmax, mg <= 4, uniform box rho.
 * The result (full symmetric, identity padding) is what pq_factor_batched's inverse mode
 * leaves for pq_admm_lr_batched / pq_admm_lr_grouped; a new rho is a re-form, not a
 * refactorisation.  scratch: 8 k_ld doubles per problem.  Replaces the per-(date, lambda)
 * KKT factorisation inside qpsolvers.solve_problem (src/qp_problems.py:211-214) for
 * P = 2 lambda Sigma_d (src/optimization.py:168-174).                                   */
int pq_eigcap_form(const pq_lowrank* lr, const pq_problem* pb, const pq_state* st, const pq_settings* s,
                   const int32_t* pdate, const double* V, const double* evals, const double* What,
                   const double* cc, int32_t k_ld, const int32_t* idx, int32_t nidx, double* Minv,
                   int64_t M_stride, double* scratch, void* stream);

/* K4: active-set polish of the ADMM point (reduced KKT by masked Cholesky + Schur +
 * proximal iterative refinement), then exact residuals / objective of the final point
 * into out[] (Solution.obj / primal_residual / dual_residual / duality_gap).            */
int pq_polish_batched(const pq_problem* pb, pq_state* st, const int32_t* idx, int32_t nidx,
                      const pq_settings* s, void* stream);

/* K4 with the exact P x products taken from the window form of P (lr, as for
 * pq_admm_lr_batched: two passes over the date's window rows instead of n^2 bytes of P;
 * tmax <= 1024, even ldp).  pb.P (the K1 output) is still read for P_FF.               */
int pq_polish_lr_batched(const pq_lowrank* lr, const pq_problem* pb, pq_state* st,
                         const int32_t* idx, int32_t nidx, const pq_settings* s, void* stream);

/* K4 entirely in the window form (pb->P is not read; any n): each active-set round forms
 * the reduced P_FF from the free columns of the window with FP64 MFMA tile products into
 * a compact ldk x ldk scratch (st->K, K_stride >= ldk^2; st->Dt, Dt_stride >=
 * (ldk/64) 4096), indexed by launch slot (blockIdx: the problem's position in idx[] or
 * its id when idx == NULL).  64 <= ldk <= min(ld, 1024).  A problem whose free set
 * exceeds ldk is left unchanged with out[PQ_OUT_ROUNDS] = -1 unless final_try != 0 (then
 * it is scored at its ADMM point, status PQ_SOLVED_INACCURATE).  Needs lr->dg.  A free
 * set beyond ldk is solved in Woodbury form with the T x T capacitance of the free
 * columns; with band (pq_lr_band_gram's row-band Gram of the panel, rows from r0, pitch
 * ldo; NULL = none) and every column free, that capacitance is gathered from the band
 * instead of a T x T x n product.                                                       */
int pq_polish_w_batched(const pq_lowrank* lr, const pq_problem* pb, pq_state* st, const int32_t* idx,
                        int32_t nidx, const pq_settings* s, int32_t ldk, int32_t final_try,
                        const double* band, int64_t ldo, int32_t r0, void* stream);

/* K4, grouped pipeline (polish_g.hip): the active-set polish of pq_polish_w_batched as a
 * few throughput kernels per round over every date of a window-path batch -- per-date
 * setup, an LDS-resident packed Cholesky of P_FF (free sets 1..128) with the same
 * regularised reduced KKT and refinement, and the exact P x / gradient / acceptance
 * checks as FP64 MFMA passes over the union rows of each slide group (the group plan of
 * pq_admm_lr_grouped).  rec holds PQ_PG_RECORD doubles per problem (field 3 = state:
 * PQ_PG_PENDING / DONE / FALLBACK / SKIP).  pq_polish_grouped_init classifies the ADMM
 * point; each pq_polish_grouped_round call runs one active-set round for the pending
 * problems.  Accepted problems are scored exactly as pq_polish_w_batched scores them
 * (status PQ_SOLVED, out[]); FALLBACK problems (free set outside 1..min(128, ldk), more
 * than 32 active rows, a failed factorisation, or not accepted within polish_rounds) are
 * left at their ADMM point for pq_polish_w_batched.  K scratch: ldk x ldk per problem
 * (indexed by problem id).  Needs even n and ldp, mg <= 32, umax <= 320, lr->dg.  The
 * window passes of a group run split over 4 workgroups (column slices), with
 * pass_scratch = ngroups * PQ_PG_PASS_SCRATCH doubles for their partial products.
 * Replaces, with pq_polish_w_batched, the accuracy of qpsolvers (src/qp_problems.py:211-214). */
#define PQ_PG_RECORD 384
#define PQ_PG_PASS_SCRATCH 123537  /* doubles per group: 4 x 324 x 16 + 4 x 16 + 16 (window passes)
                                      + 320 x 320 + 320 + 1 (the big group form's Gram)      */
#define PQ_PG_PENDING 0
#define PQ_PG_DONE 1
#define PQ_PG_FALLBACK 2
#define PQ_PG_SKIP 3
/* Wide rounds (polish_gw.hip, wide != NULL): a pending problem whose free set exceeds
 * min(128, ldk) with at most PQ_PG_WMB bordered rows (active general rows + variables at a
 * bound) solves its round's KKT system in n-space by a group capacitance of the polish
 * matrix K = P + d I, d = p_diag + gc->grho[g] (one value per group: built by
 * pq_gcap_assemble / pq_factor_batched / pq_gcap_prepare with mg = 0 and a unit box, so
 * that the box rho is grho), the bordered rows eliminated by a per-date Schur complement,
 * and refine_steps proximal refinement steps (early exit at convergence) whose window products are MFMA
 * passes over the union rows of the group (16 dates per pass).  pc / ldpc / r0 / cc: the
 * band setup's panel-row products with the general rows and C C'; nzr / nzv / nzmax: their
 * column-sparse form (needed when mg > 4; mg <= 24); wscr: PQ_PG_WSCR(k_ld) doubles per
 * problem, wscr_stride apart.  Replaces, with the rest of the round, the accuracy of
 * qpsolvers' answer for free sets of any size (src/qp_problems.py:211-214). */
#define PQ_PG_WMB 8
#define PQ_PG_WSCR(k_ld) (2 * PQ_PG_WMB * (int64_t)(k_ld))
typedef struct pq_pg_wide {
  const pq_gcap* gc;
  const double* pc; int64_t ldpc; int32_t r0; const double* cc;
  const int32_t* nzr; const double* nzv; int32_t nzmax;
  double* wscr; int64_t wscr_stride;
  int32_t refine_steps;         /* proximal refinement steps per wide round (>= 1)          */
} pq_pg_wide;
int pq_polish_grouped_init(const pq_lowrank* lr, const pq_problem* pb, pq_state* st, double* rec,
                           const pq_settings* s, void* stream);
int pq_polish_grouped_round(const pq_lowrank* lr, const pq_problem* pb, pq_state* st, double* rec, int32_t ldk,
                            const int32_t* gdates, int32_t ngroups, const int32_t* urows, const int32_t* ucnt,
                            const int32_t* uoff, int32_t umax, const pq_settings* s, double* pass_scratch,
                            const pq_pg_wide* wide, void* stream);

/* Strategy simulation: one holding period per rebalance date.
 * Replaces Strategy.simulate (src/portfolio.py:209-248) with floating_weights
 * (src/portfolio.py:259-296) and the end-weight part of Portfolio.turnover
 * (src/portfolio.py:111-123).  Period p floats W[p] (n weights, stride ldw) over panel rows
 * row0[p] .. row0[p] + nrows[p] - 1 (row 0 of the period is the weights themselves; NaN
 * returns count as 0) and writes its nrows[p] - 1 level returns (loan + cash + margin +
 * floated weights, pct_change) to ret[ret_off[p] ...].  fc != 0 subtracts the fixed cost
 * (1 + fc)^((ret_day[q] - ret_day[q-1]) / days_per_year) - 1 from every return q > 0 of
 * the flattened series (ret_day = calendar day of each return).  Optional outputs: wend
 * (floated end weights, rescaled to unit long / short books when rescale != 0, stride
 * ldwe) and turnover[p] = sum_j |wend[p][j] - W[p][j]|.  n <= 8192.                   */
int pq_simulate_periods(const double* panel, int64_t ldp, int32_t n, const double* W, int64_t ldw,
                        const int32_t* row0, const int32_t* nrows, int32_t nper,
                        const int64_t* ret_off, const int32_t* ret_day, double fc,
                        double days_per_year, double* ret, double* wend, int64_t ldwe,
                        double* turnover, int32_t rescale, void* stream);

/* Batched matrix-vector products with the interior-point methods' window matrices
 * (porqua_amd/ipm_l1.py, the linearised turnover / leverage problem of
 * src/qp_problems.py:40-157): trans = 0: y[b] = U[b] x[b] (U m x n, row stride ldu, batch
 * stride su; y m); trans = 1: y[b] = U[b]' x[b] (y n; m <= 8192).  HBM-bound, one read of
 * U per product.                                                                         */
int pq_gemv_batched(const double* U, int64_t ldu, int64_t su, int32_t m, int32_t n, int32_t batch,
                    int32_t trans, const double* x, int64_t sx, double* y, int64_t sy, void* stream);

/* LAD interior-point method (porqua_amd/lad.py; replaces the LP solve behind
 * LAD.model_qpsolvers, src/optimization.py:296-345): out[b] = M[b] V[b], or
 * out[b] = S[b] - M[b] V[b] when S != NULL, for M[b] n x n (row stride ldm, batch stride
 * sm) and V, S, out n x k row-major (batch strides sv, ss, so).  1 <= k <= 4 (V in LDS for n <= 1024, read through L2 beyond).
 * Applies the K2-inverted normal matrix H^-1 and H itself to the IPM right-hand sides.   */
int pq_lad_mv_batched(const double* M, int64_t ldm, int64_t sm, int32_t n, int32_t batch,
                      const double* V, int64_t sv, int32_t k, const double* S, int64_t ss,
                      double* out, int64_t so, void* stream);

/* Window-form interior-point methods (porqua_amd/ipm_lr.py; the LAD LP behind
 * LAD.model_qpsolvers, src/optimization.py:296-345, and QPs with both l1 linearisations,
 * src/qp_problems.py:40-118): the Woodbury capacitance of H = Lam + U' diag(e) U,
 *   M[b] = diag(d[b]) + diag(r[b]) U[b] diag(w[b]) U[b]' diag(r[b])   (k x k, lower tiles)
 * for U[b] k x n (row stride ldu, batch stride su), column weights w (b, n; w = 1/Lam), row
 * scales r (b, k; r = sqrt(e); NULL = 1) and diagonal d (b, k; NULL = 1).  Rows k..k_ld-1 of
 * M are identity padding (k_ld a multiple of 64), so K2 (pq_factor_batched on {n = k_ld,
 * P = M}) factors it as is.  batch <= 65535 per launch.                                   */
int pq_wgram_batched(const double* U, int64_t ldu, int64_t su, int32_t k, int32_t n, int32_t batch,
                     const double* w, int64_t sw, const double* r, int64_t sr, const double* d, int64_t sd,
                     double* M, int32_t k_ld, int64_t sm, void* stream);

/* Device bytes of the per-batch buffers a caller allocates before the solve entry points
 * (the pq_state arrays, the polish scratch and, for the window path, the capacitance
 * matrices M, M^-1 and their factor scratch), so a non-Python host can size one arena.
 * path 0 = dense (K, Dt: ld x ld per problem), 1 = window (compact polish scratch ldk x ldk,
 * ldk = min(ld, 1024, round_up(ldk, 64)); k_ld = round_up(tmax + mg, 64)).  ld =
 * round_up(n, 64), mg_pad = round_up(max(mg, 1), 8).  Returns -1 on invalid arguments.
 * Replaces nothing in the reference (qpsolvers allocates internally); SURVEY.md §8(b).   */
int64_t pq_workspace_bytes(int32_t n, int32_t batch, int32_t mg, int32_t path, int32_t tmax, int32_t ldk);


/* Batched symmetric eigensolver (two-sided block Jacobi, FP64): the eigendecomposition behind
 * nearestPD's projection (src/helper_functions.py:42-45: for symmetric B the SVD gives
 * H = Q |L| Q', so (B + H)/2 = Q max(L, 0) Q') and behind its shift loop's
 * np.linalg.eigvals (:51-56).  A (ld x ld per matrix, symmetric, overwritten: diagonalised),
 * entries beyond n ignored (zeroed); V (may be NULL) receives the eigenvectors (columns);
 * evals[b][0..ld) = diag of the diagonalised A (unsorted; 0 beyond n).  work:
 * pq_sym_eig_work_doubles(ld) doubles per matrix.  Sweeps of 64 x 64 subproblems (one
 * workgroup each, cyclic Jacobi in LDS) and MFMA tile updates, until a sweep rotates nothing
 * (at most max_sweeps; rotation threshold |a_pq| > tol sqrt|a_pp a_qq|).                  */
int64_t pq_sym_eig_work_doubles(int32_t ld);
int pq_sym_eig_batched(double* A, int32_t ld, int64_t a_stride, int32_t n, int32_t batch, double* V,
                       int64_t v_stride, double* evals, int64_t e_stride, double* work, int64_t w_stride,
                       int32_t max_sweeps, double tol, void* stream);

/* Convergence of the batch after pq_sym_eig_batched (same work buffer, same max_sweeps):
 * conv[b] = 1 when the last sweep rotated nothing in matrix b (every off-diagonal entry met
 * the tolerance), 0 when max_sweeps ran out first -- the caller must not use unconverged
 * eigenpairs as if they were the reference's (np.linalg.eigvals / SVD, :42-56).          */
int pq_sym_eig_converged(const double* work, int32_t ld, int64_t w_stride, int32_t batch, int32_t max_sweeps,
                         int32_t* conv, void* stream);

/* out = V diag(max(evals, 0)) V' (full ld x ld, columns k >= n of V ignored): the PSD
 * projection A2 of nearestPD (src/helper_functions.py:43-44) on FP64 MFMA.               */
int pq_psd_form_batched(const double* V, int64_t v_stride, const double* evals, int64_t e_stride, int32_t ld,
                        int32_t n, int32_t batch, double* out, int64_t o_stride, void* stream);

/* C = op(A) op(B) for ld x ld matrices (ta / tb != 0: transposed), FP64 MFMA tiles.      */
int pq_tile_gemm_batched(const double* A, int64_t sa, int32_t ta, const double* B, int64_t sb, int32_t tb,
                         double* C, int64_t sc, int32_t ld, int32_t batch, void* stream);

#ifdef __cplusplus
}
#endif
#endif
