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
