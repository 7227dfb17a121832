// Error plumbing for the C ABI: nothing throws across extern "C"; the last error message
// is kept per host thread and returned by pq_last_error().
#pragma once
#include <hip/hip_runtime.h>
#include <stdio.h>
#include "../../include/porqua_hip.h"

namespace pq {
void set_error(const char* fmt, ...);
}

#define PQ_CHECK_ARG(cond, ...)       \
  do {                                \
    if (!(cond)) {                    \
      pq::set_error(__VA_ARGS__);     \
      return -1;                      \
    }                                 \
  } while (0)

#define PQ_CHECK_LAUNCH(what)                                                   \
  do {                                                                          \
    hipError_t e_ = hipGetLastError();                                          \
    if (e_ != hipSuccess) {                                                     \
      pq::set_error("%s: HIP launch error: %s", what, hipGetErrorString(e_));   \
      return -2;                                                                \
    }                                                                           \
  } while (0)

#define PQ_CHECK_HIP(call)                                                      \
  do {                                                                          \
    hipError_t e_ = (call);                                                     \
    if (e_ != hipSuccess) {                                                     \
      pq::set_error("%s: %s", #call, hipGetErrorString(e_));                    \
      return -2;                                                                \
    }                                                                           \
  } while (0)
