// ffcv_host.hip -- the reference's one-sample host entry points, same names
// and argument order as /root/reference/libffcv/libffcv.cpp, so code that
// binds them (ffcv/libffcv.py:22-48: resize_crop, imdecode; user Operations,
// transforms/utils/fast_crop.py) keeps working against libffcv_hip.so.
//
//   resize   (libffcv.cpp:33-42)  cv::resize(ROI, dst, INTER_AREA) on host
//            memory, computed on the CPU by the same single-source INTER_AREA
//            functions the kernels run (device_common.h ResizePlan ...).
//   ffcv_imdecode_device: imdecode's signature and semantics (libffcv.cpp:
//            53-112), executed by the gfx950 JPEG kernels on a per-thread
//            stream and decoder context (bytes in, pixels out with
//            hipMemcpyAsync).  imdecode itself decodes on the CPU, like the
//            reference (ffcv_cpu_jpeg.hip).
//
// The hot path never comes here: the Loader decodes whole launches on the
// device (ffcv_jpeg_rrc_fused).  These exist for drop-in compatibility.
#include <cmath>
#include <cstring>
#include <vector>

#include "api_internal.h"
#include "device_common.h"

namespace {

// One output pixel of resize() from precomputed column / row taps.
struct HostPlan {
  ResizePlan P;
  std::vector<AreaTaps> ax, ay;
  std::vector<LinTap> lx, ly;
};

void make_host_plan(HostPlan &h, int sw, int sh, int dw, int dh) {
  h.P = make_plan(sw, sh, dw, dh);
  if (h.P.kind == 2) {
    h.ax.resize(dw);
    h.ay.resize(dh);
    for (int d = 0; d < dw; d++) h.ax[d] = area_taps(sw, h.P.scale_x, d);
    for (int d = 0; d < dh; d++) h.ay[d] = area_taps(sh, h.P.scale_y, d);
  } else if (h.P.kind == 3) {
    h.lx.resize(dw);
    h.ly.resize(dh);
    for (int d = 0; d < dw; d++) h.lx[d] = lin_tap(h.P.scale_x, h.P.inv_x, sw, d);
    for (int d = 0; d < dh; d++) h.ly[d] = lin_tap(h.P.scale_y, h.P.inv_y, sh, d);
  }
}

// Per-thread device state behind imdecode (the reference keeps per-thread
// TurboJPEG handles in pthread TLS and never frees them, libffcv.cpp:19-31;
// same lifetime here).
struct HostDecoder {
  int device = -1;
  hipStream_t stream = nullptr;
  ffcv_jpeg_ctx *ctx = nullptr;
  uint32_t cap_h = 0, cap_w = 0;
  uint64_t cap_bytes = 0;
  uint8_t *d_in = nullptr;
  uint64_t in_cap = 0;
  uint8_t *d_out = nullptr;
  uint64_t out_cap = 0;
  ffcv_sample *d_smp = nullptr;
  int32_t *d_status = nullptr;
};
thread_local HostDecoder *t_dec = nullptr;

constexpr uint64_t kInPad = 256;  // zeroed slack after the stream (reader prefetch)

int grow(uint8_t **p, uint64_t *cap, uint64_t need, const char *what) {
  if (*cap >= need) return FFCV_OK;
  uint64_t n = need + need / 4;
  if (*p) (void)hipFree(*p);
  *p = nullptr;
  *cap = 0;
  hipError_t e = hipMalloc(p, n);
  if (e != hipSuccess) return ffcv::check_hip(e, what);
  *cap = n;
  return FFCV_OK;
}

int prepare(HostDecoder *d, uint32_t h, uint32_t w, uint64_t nbytes) {
  int dev = 0;
  FFCV_HIP_CHECK(hipGetDevice(&dev));
  if (d->device != dev) {  // first use on this thread (or the thread moved device)
    d->device = dev;
    d->ctx = nullptr;
    d->cap_h = d->cap_w = 0;
    d->cap_bytes = 0;
    d->d_in = d->d_out = nullptr;
    d->in_cap = d->out_cap = 0;
    FFCV_HIP_CHECK(hipStreamCreateWithFlags(&d->stream, hipStreamNonBlocking));
    FFCV_HIP_CHECK(hipMalloc(&d->d_smp, sizeof(ffcv_sample)));
    FFCV_HIP_CHECK(hipMalloc(&d->d_status, sizeof(int32_t)));
  }
  if (!d->ctx || h > d->cap_h || w > d->cap_w || nbytes > d->cap_bytes) {
    if (d->ctx) ffcv_jpeg_destroy(d->ctx);
    d->ctx = nullptr;
    d->cap_h = std::max(h, d->cap_h);
    d->cap_w = std::max(w, d->cap_w);
    d->cap_bytes = std::max(nbytes, d->cap_bytes);
    int rc = ffcv_jpeg_create(&d->ctx, 1, d->cap_h, d->cap_w, d->cap_bytes);
    if (rc) return rc;
  }
  int rc = grow(&d->d_in, &d->in_cap, nbytes + kInPad, "imdecode: input buffer");
  if (rc) return rc;
  return grow(&d->d_out, &d->out_cap, (uint64_t)h * w * 3, "imdecode: output buffer");
}

}  // namespace

extern "C" {

void resize(int64_t cresizer, int64_t source_p, int64_t sx, int64_t sy, int64_t start_row, int64_t end_row,
            int64_t start_col, int64_t end_col, int64_t dest_p, int64_t tx, int64_t ty) {
  (void)cresizer;  // unused by the reference too
  const uint8_t *src = reinterpret_cast<const uint8_t *>(source_p);
  uint8_t *dst = reinterpret_cast<uint8_t *>(dest_p);
  const int64_t sh = end_row - start_row, sw = end_col - start_col;
  if (!src || !dst || sh <= 0 || sw <= 0 || tx <= 0 || ty <= 0 || start_row < 0 || start_col < 0 ||
      end_row > sx || end_col > sy || sh > 65535 || sw > 65535 || tx > 65535 || ty > 65535) {
    ffcv::set_error("resize: invalid ROI [%lld:%lld, %lld:%lld] of %lldx%lld -> %lldx%lld",
                    (long long)start_row, (long long)end_row, (long long)start_col, (long long)end_col,
                    (long long)sx, (long long)sy, (long long)tx, (long long)ty);
    return;  // void like the reference (cv::resize would throw)
  }
  // cv::Mat(sx, sy, CV_8UC3): sx rows of sy pixels; the ROI keeps that step
  const uint64_t step = (uint64_t)sy * 3;
  RoiSrc S{src + (uint64_t)start_row * step + (uint64_t)start_col * 3, step};
  HostPlan h;
  make_host_plan(h, (int)sw, (int)sh, (int)ty, (int)tx);
  const ResizePlan &P = h.P;
  if (P.kind == 3) {
    // resize.cpp's separable form of resize_linear: HResizeLinear once per
    // source row into an int row (two rows cached, as the kernels' walk),
    // then VResizeLinear per element -- the SSE2 body's (sat_s16(h >> 4) *
    // c) >> 16 sums below vec_end, the scalar tail's rounding after it.
    const int dw = (int)ty, dh = (int)tx, n = dw * 3;
    thread_local std::vector<int> hbuf;
    hbuf.resize((size_t)2 * n);
    int *HA = hbuf.data(), *HB = HA + n;
    int ca = -1, cb = -1;
    auto hrow = [&](int r, int *H) {
      const uint8_t *rp = S.p + (uint64_t)r * S.step;
      for (int dx = 0; dx < dw; dx++) {
        const LinTap &l = h.lx[dx];
        const uint8_t *q = rp + (uint64_t)l.s * 3;
        for (int c = 0; c < 3; c++) H[dx * 3 + c] = l.border ? q[c] * 2048 : q[c] * l.c0 + q[c + 3] * l.c1;
      }
    };
    for (int dy = 0; dy < dh; dy++) {
      const LinTap &ly = h.ly[dy];
      const int ra = std::min(std::max(ly.s, 0), P.sh - 1), rb = std::min(std::max(ly.s + 1, 0), P.sh - 1);
      if (ra != ca) {
        if (ra == cb) {
          std::swap(HA, HB);
          std::swap(ca, cb);
        } else {
          hrow(ra, HA);
          ca = ra;
        }
      }
      if (rb != cb) {
        hrow(rb, HB);
        cb = rb;
      }
      uint8_t *row = dst + (uint64_t)dy * n;
      const int ve = std::min(P.vec_end, n);
      for (int e = 0; e < ve; e++) {
        const int m0 = (sat_s16i(HA[e] >> 4) * ly.c0) >> 16, m1 = (sat_s16i(HB[e] >> 4) * ly.c1) >> 16;
        row[e] = (uint8_t)sat_u8i((sat_s16i(m0 + m1) + 2) >> 2);
      }
      for (int e = ve; e < n; e++) row[e] = (uint8_t)sat_u8i((HA[e] * ly.c0 + HB[e] * ly.c1 + (1 << 21)) >> 22);
    }
    return;
  }
  for (int dy = 0; dy < (int)tx; dy++) {
    uint8_t *row = dst + (uint64_t)dy * ty * 3;
    for (int dx = 0; dx < (int)ty; dx++) {
      int v[3];
      if (P.kind == 2)
        resize_area(S, h.ax[dx], h.ay[dy], v);
      else if (P.kind == 3)
        resize_linear(P, S, dx, h.lx[dx], h.ly[dy], v);
      else
        resize_pixel(P, S, dy, dx, v);
      row[dx * 3 + 0] = (uint8_t)v[0];
      row[dx * 3 + 1] = (uint8_t)v[1];
      row[dx * 3 + 2] = (uint8_t)v[2];
    }
  }
}

int ffcv_draw_batch_host(const uint64_t *sample_ids, const uint32_t *heights, const uint32_t *widths, int batch,
                         const ffcv_draw_params *p, int32_t *crops, int32_t *cutout_yx, uint8_t *flips) {
  if (batch < 0 || !p || !sample_ids || (crops && (!heights || !widths))) {
    ffcv::set_error("ffcv_draw_batch_host: invalid arguments");
    return FFCV_EINVAL;
  }
  if (cutout_yx && p->cutout_size > 0 && (p->cutout_size > p->out_h || p->cutout_size > p->out_w)) {
    ffcv::set_error("ffcv_draw_batch_host: cutout_size %d exceeds output %dx%d", p->cutout_size, p->out_h,
                    p->out_w);
    return FFCV_EINVAL;
  }
  int err = 0;
  for (int k = 0; k < batch; k++) {
    const uint32_t H = heights ? heights[k] : 0, W = widths ? widths[k] : 0;
    for (int part = 0; part < 3; part++) err |= draw_part(part, k, sample_ids[k], H, W, *p, crops, cutout_yx, flips);
  }
  if (err) {
    ffcv::set_error("ffcv_draw_batch_host: MT19937 stream exhausted");
    return FFCV_EINVAL;
  }
  return FFCV_OK;
}

int ffcv_imdecode_device(unsigned char *input_buffer, uint64_t input_size, uint32_t source_height,
                         uint32_t source_width, unsigned char *output_buffer, uint32_t crop_height,
                         uint32_t crop_width, uint32_t offset_x, uint32_t offset_y, uint32_t scale_num,
                         uint32_t scale_denom, bool enable_crop, bool hflip) {
  (void)source_height;  // unused by the reference too (libffcv.cpp:53-112)
  (void)source_width;
  (void)offset_x;
  (void)offset_y;
  if (!input_buffer || !output_buffer || input_size == 0 || crop_height == 0 || crop_width == 0 ||
      crop_height > 65535 || crop_width > 65535) {
    ffcv::set_error("imdecode: invalid arguments");
    return -1;
  }
  if (enable_crop || hflip || scale_num != scale_denom) {
    // tjTransform lossless crop / flip and DCT scaling: never used by ffcv
    // (rgb_image.py:131,196 pass False, False, 1, 1)
    ffcv::set_error("imdecode: crop / flip / scaling transforms are not supported");
    return -1;
  }
  if (!t_dec) t_dec = new HostDecoder();
  HostDecoder *d = t_dec;
  if (prepare(d, crop_height, crop_width, input_size)) return -1;
  hipStream_t s = d->stream;
  ffcv_sample smp = {0, input_size, crop_height, crop_width, 0, 0};
  const uint64_t out_bytes = (uint64_t)crop_height * crop_width * 3;
  int32_t status = -1;
  if (hipMemcpyAsync(d->d_in, input_buffer, input_size, hipMemcpyHostToDevice, s) != hipSuccess ||
      hipMemsetAsync(d->d_in + input_size, 0, kInPad, s) != hipSuccess ||
      hipMemcpyAsync(d->d_smp, &smp, sizeof(smp), hipMemcpyHostToDevice, s) != hipSuccess) {
    ffcv::set_error("imdecode: host -> device copy failed");
    return -1;
  }
  if (ffcv_jpeg_decode_batch(d->ctx, s, d->d_in, d->d_smp, 1, d->d_out, (uint64_t)crop_width * 3,
                             d->d_status) != FFCV_OK)
    return -1;
  if (hipMemcpyAsync(output_buffer, d->d_out, out_bytes, hipMemcpyDeviceToHost, s) != hipSuccess ||
      hipMemcpyAsync(&status, d->d_status, sizeof(status), hipMemcpyDeviceToHost, s) != hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess) {
    ffcv::set_error("imdecode: device -> host copy failed");
    return -1;
  }
  if (status != FFCV_SAMPLE_OK) {
    ffcv::set_error("imdecode: JPEG decode failed (sample status %d)", status);
    return -1;
  }
  return 0;
}

}  // extern "C"
