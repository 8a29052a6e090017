// api_internal.h -- host-side helpers shared by the C-ABI translation units.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>

#include "../../include/ffcv_hip.h"

namespace ffcv {
void set_error(const char *fmt, ...);
int check_hip(hipError_t e, const char *what);
inline hipStream_t as_stream(void *s) { return reinterpret_cast<hipStream_t>(s); }
}  // namespace ffcv

#define FFCV_HIP_CHECK(expr)                                        \
  do {                                                              \
    hipError_t _e = (expr);                                         \
    if (_e != hipSuccess) return ffcv::check_hip(_e, #expr);        \
  } while (0)

#define FFCV_LAUNCH_CHECK(what)                                      \
  do {                                                               \
    hipError_t _e = hipGetLastError();                               \
    if (_e != hipSuccess) return ffcv::check_hip(_e, what);          \
  } while (0)
