// C-ABI bookkeeping: version and per-thread error string.
#include <stdarg.h>
#include <string.h>
#include "capi_util.h"

namespace pq {
static thread_local char g_err[512] = "";
void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
}  // namespace pq

extern "C" int pq_version(void) { return PQ_VERSION; }
extern "C" const char* pq_last_error(void) { return pq::g_err; }

static inline int64_t round_up64(int64_t v, int64_t m) { return ((v + m - 1) / m) * m; }

extern "C" int64_t pq_workspace_bytes(int32_t n, int32_t batch, int32_t mg, int32_t path, int32_t tmax,
                                      int32_t ldk) {
  if (n <= 0 || batch < 0 || mg < 0 || (path != 0 && path != 1) || (path == 1 && (tmax <= 0 || ldk <= 0))) {
    pq::set_error("pq_workspace_bytes: invalid arguments");
    return -1;
  }
  const int64_t ld = round_up64(n, 64), mg_pad = round_up64(mg > 1 ? mg : 1, 8), m_ld = mg_pad + ld;
  int64_t kd = ld;
  if (path == 1) {
    kd = round_up64(ldk, 64);
    if (kd > ld) kd = ld;
    if (kd > 1024) kd = 1024;
  }
  // K + Dt | x, Px | z, y | rho | iters, status, info | out | work
  int64_t per = 8 * (kd * kd + (kd / 64) * 4096) + 8 * 2 * ld + 8 * 2 * m_ld + 8 + 3 * 4 +
                8 * PQ_OUT_FIELDS + 8 * PQ_WORK_DOUBLES(ld, mg_pad);
  if (path == 1) {
    const int64_t k_ld = round_up64((int64_t)tmax + mg, 64);
    per += 8 * (2 * k_ld * k_ld + (k_ld / 64) * 4096) + 3 * 4;   // M, M^-1, Dt | iters, status, info
  }
  return per * batch;
}
