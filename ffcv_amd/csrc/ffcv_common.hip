// ffcv_common.hip -- error state, device/stream/memory helpers and the
// reference-compatible my_memcpy (libffcv.cpp:44-46).
#include <cstdio>
#include <cstring>
#include <string>

#include "api_internal.h"

#include <algorithm>
#include <cstring>
#include <thread>
#include <vector>

namespace ffcv {
static thread_local std::string g_last_error;

void set_error(const char *fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_last_error = buf;
}

int check_hip(hipError_t e, const char *what) {
  set_error("%s: %s (%d)", what, hipGetErrorString(e), (int)e);
  return e == hipErrorOutOfMemory ? FFCV_ENOMEM : FFCV_EHIP;
}
}  // namespace ffcv

extern "C" {

int ffcv_abi_version(void) { return FFCV_HIP_ABI_VERSION; }

const char *ffcv_last_error(void) { return ffcv::g_last_error.c_str(); }

int ffcv_device_count(int *count) {
  if (!count) {
    ffcv::set_error("ffcv_device_count: count is NULL");
    return FFCV_EINVAL;
  }
  FFCV_HIP_CHECK(hipGetDeviceCount(count));
  return FFCV_OK;
}

int ffcv_set_device(int device) {
  FFCV_HIP_CHECK(hipSetDevice(device));
  return FFCV_OK;
}

int ffcv_stream_synchronize(void *stream) {
  FFCV_HIP_CHECK(hipStreamSynchronize(ffcv::as_stream(stream)));
  return FFCV_OK;
}

int ffcv_malloc(void **dptr, uint64_t bytes) {
  FFCV_HIP_CHECK(hipMalloc(dptr, bytes));
  return FFCV_OK;
}

int ffcv_free(void *dptr) {
  FFCV_HIP_CHECK(hipFree(dptr));
  return FFCV_OK;
}

int ffcv_memcpy_h2d_async(void *dst, const void *src, uint64_t bytes, void *stream) {
  FFCV_HIP_CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, ffcv::as_stream(stream)));
  return FFCV_OK;
}

int ffcv_memcpy_d2h_async(void *dst, const void *src, uint64_t bytes, void *stream) {
  FFCV_HIP_CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, ffcv::as_stream(stream)));
  return FFCV_OK;
}

// libffcv.cpp:44-46: my_memcpy(source, dst, size) -- host plumbing only.
void my_memcpy(void *source, void *dst, uint64_t size) { std::memcpy(dst, source, size); }

// libffcv.cpp:48-51: my_fread(fp, offset, destination, size) on a FILE *
// passed as an integer -- host plumbing only.
void my_fread(int64_t fp, int64_t offset, void *destination, int64_t size) {
  FILE *f = (FILE *)(intptr_t)fp;
  if (!f || size <= 0) return;
  if (fseeko(f, (off_t)offset, SEEK_SET) != 0) return;
  (void)fread(destination, 1, (size_t)size, f);
}

// Host gather of n byte ranges (e.g. a batch's compressed samples out of the
// mmap'd .beton) into one staging buffer, split over nthreads threads by
// byte count.  The PCIe path (device_cache=False) stages each batch this way
// before one hipMemcpyAsync.
int ffcv_host_gather(const uint8_t *src, const uint64_t *src_off, const uint64_t *sizes, const uint64_t *dst_off,
                     int n, uint8_t *dst, int nthreads) {
  if (n < 0 || (n > 0 && (!src || !src_off || !sizes || !dst_off || !dst))) {
    ffcv::set_error("ffcv_host_gather: invalid arguments");
    return FFCV_EINVAL;
  }
  uint64_t total = 0;
  for (int i = 0; i < n; i++) total += sizes[i];
  const int T = std::max(1, std::min(nthreads, n));
  auto work = [&](int tid) {
    // contiguous runs of samples with about total / T bytes each
    const uint64_t lo = total * tid / T, hi = total * (tid + 1) / T;
    uint64_t acc = 0;
    for (int i = 0; i < n; i++) {
      const uint64_t a = acc, b = acc + sizes[i];
      acc = b;
      if (b <= lo || a >= hi) continue;
      const uint64_t s = std::max(a, lo) - a, e = std::min(b, hi) - a;
      std::memcpy(dst + dst_off[i] + s, src + src_off[i] + s, e - s);
    }
  };
  if (T == 1) {
    work(0);
    return FFCV_OK;
  }
  std::vector<std::thread> th;
  th.reserve(T - 1);
  for (int t = 1; t < T; t++) th.emplace_back(work, t);
  work(0);
  for (auto &x : th) x.join();
  return FFCV_OK;
}

}  // extern "C"
