// Strategy simulation over the solved weight panel.
//
// Reference: Strategy.simulate (src/portfolio.py:209-248) floats each rebalance date's
// weights to the next date (floating_weights, :259-296: row 0 = w, then a cumulative
// product of 1 + r), prepends the loan / cash / margin columns, sums them into a level and
// takes its day-on-day percentage change; Portfolio.turnover (:111-123) compares the
// floated end weights of a portfolio with its own weights.
//
// MI355X mapping: one 256-thread workgroup per holding period, each thread holding KV of
// the period's running products in registers (no LDS state), one coalesced 8 B/lane read
// of every panel row of the period and a workgroup sum per row.  The pass reads each panel
// row once per period that covers it (boundary rows twice), so it is HBM / L2 bound:
// 8 n B per period row, plus 16 n B of weights in / floated weights out per period.
#include "capi_util.h"
#include "common.h"

namespace pq {

template <int KV>
__global__ __launch_bounds__(256) void k_float_periods(
    const double* __restrict__ panel, int64_t ldp, int n, const double* __restrict__ W, int64_t ldw,
    const int32_t* __restrict__ row0, const int32_t* __restrict__ nrows, int nper,
    const int64_t* __restrict__ ret_off, const int32_t* __restrict__ ret_day, double fc,
    double days_per_year, double* __restrict__ ret, double* __restrict__ wend, int64_t ldwe,
    double* __restrict__ turnover, int rescale) {
  __shared__ double red[16];
  const int p = xcd_slot(blockIdx.x, nper);
  const int tid = threadIdx.x;
  const double* w = W + (int64_t)p * ldw;
  double c[KV], w0[KV];
  double lpos = 0.0, lneg = 0.0, s0 = 0.0;
#pragma unroll
  for (int k = 0; k < KV; ++k) {
    const int j = tid + k * 256;
    w0[k] = j < n ? w[j] : 0.0;
    c[k] = w0[k];
    if (w0[k] >= 0.0) lpos += w0[k]; else lneg += w0[k];
    s0 += w0[k];
  }
  // src/portfolio.py:226-230: margin, cash and loan are constant columns of the period
  const double L = block_sum(lpos, red);
  const double S = block_sum(lneg, red);
  const double margin = fabs(S);
  const double cash = fmax(fmin(1.0 - L, 1.0), 0.0);
  const double loan = 1.0 - (L + cash) - (S + margin);
  const double cst = loan + cash + margin;
  double lev_prev = cst + block_sum(s0, red);
  const int r0 = row0[p], nr = nrows[p];
  const int64_t off = ret_off[p];
  const double lfc = fc != 0.0 ? 1.0 + fc : 0.0;
  for (int t = 1; t < nr; ++t) {
    const double* x = panel + (int64_t)(r0 + t) * ldp;
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < KV; ++k) {
      const int j = tid + k * 256;
      if (j < n) {
        double r = x[j];
        r = r == r ? r : 0.0;          // fillna(0), src/portfolio.py:283
        c[k] *= 1.0 + r;               // xmat.cumprod(), :287
        s += c[k];
      }
    }
    const double lev = cst + block_sum(s, red);
    if (tid == 0) {
      double v = lev / lev_prev - 1.0;  // level.pct_change(1), :232
      const int64_t q = off + t - 1;
      if (lfc != 0.0 && q > 0)          // fixed cost on portf_ret[1:], :243-246
        v -= pow(lfc, (double)(ret_day[q] - ret_day[q - 1]) / days_per_year) - 1.0;
      ret[q] = v;
    }
    lev_prev = lev;
  }
  // floated end weights (rescaled as floating_weights does, :289-292) and the turnover of
  // Portfolio.turnover (:121-123): sum |w_floated - w|
  double P = 1.0, N = 1.0;
  if (rescale) {
    double sp = 0.0, sn = 0.0;
#pragma unroll
    for (int k = 0; k < KV; ++k) {
      if (c[k] >= 0.0) sp += c[k]; else sn -= c[k];
    }
    P = block_sum(sp, red);
    N = block_sum(sn, red);
  }
  double to = 0.0;
  double* we = wend ? wend + (int64_t)p * ldwe : nullptr;
#pragma unroll
  for (int k = 0; k < KV; ++k) {
    const int j = tid + k * 256;
    if (j < n) {
      double v = c[k];
      if (rescale) v = v >= 0.0 ? (P > 0.0 ? v / P : 0.0) : v / N;
      if (we) we[j] = v;
      to += fabs(v - w0[k]);
    }
  }
  to = block_sum(to, red);
  if (turnover && tid == 0) turnover[p] = to;
}

}  // namespace pq

extern "C" int pq_simulate_periods(const double* panel, int64_t ldp, int32_t n, const double* W,
                                   int64_t ldw, const int32_t* row0, const int32_t* nrows,
                                   int32_t nper, const int64_t* ret_off, const int32_t* ret_day,
                                   double fc, double days_per_year, double* ret, double* wend,
                                   int64_t ldwe, double* turnover, int32_t rescale, void* stream) {
  PQ_CHECK_ARG(panel && W && row0 && nrows && ret_off && ret, "pq_simulate_periods: null argument");
  PQ_CHECK_ARG(n > 0 && n <= 32 * 256, "pq_simulate_periods: n = %d outside 1..8192", n);
  PQ_CHECK_ARG(ldp >= n && ldw >= n && (!wend || ldwe >= n), "pq_simulate_periods: leading dimension < n");
  PQ_CHECK_ARG(fc == 0.0 || (ret_day && days_per_year > 0.0), "pq_simulate_periods: fc needs ret_day");
  if (nper <= 0) return 0;
  const int kv = (n + 255) / 256;
  hipStream_t s = (hipStream_t)stream;
#define PQ_SIM(KV)                                                                              \
  hipLaunchKernelGGL(pq::k_float_periods<KV>, dim3(nper), dim3(256), 0, s, panel, ldp, n, W, ldw, \
                     row0, nrows, nper, ret_off, ret_day, fc, days_per_year, ret, wend, ldwe,     \
                     turnover, rescale)
  if (kv <= 1) PQ_SIM(1);
  else if (kv <= 2) PQ_SIM(2);
  else if (kv <= 4) PQ_SIM(4);
  else if (kv <= 8) PQ_SIM(8);
  else if (kv <= 16) PQ_SIM(16);
  else PQ_SIM(32);
#undef PQ_SIM
  PQ_CHECK_LAUNCH("pq_simulate_periods");
  return 0;
}
