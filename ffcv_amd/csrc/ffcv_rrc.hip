// ffcv_rrc.hip -- device random draws, raw-mode crop+INTER_AREA resize with a
// fused flip / cutout / LUT-normalize epilogue, and the standalone transforms.
//
// Reference path (raw mode): rgb_image.py:202-208 takes a
// zero-copy view of the mmap'd sample, get_random_crop draws the window and
// libffcv.cpp:33-42 cv::resize(INTER_AREA) writes the output; Cutout
// (cutout.py:36-47) and NormalizeImage (normalize.py:65) follow as separate
// passes.  Here the .beton bytes are already resident in HBM, so one launch
// reads each crop ROI once and writes the final (u8 or fp16) pixels once.
#include "api_internal.h"
#include "device_common.h"

// ------------------------------------------------------------ draws -------
__global__ void __launch_bounds__(64) draw_kernel(const uint64_t *__restrict__ ids,
                                                  const ffcv_sample *__restrict__ samples, int B,
                                                  ffcv_draw_params p, int32_t *__restrict__ crops,
                                                  int32_t *__restrict__ cut, uint8_t *__restrict__ flips,
                                                  int32_t *__restrict__ status) {
  int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= B) return;
  const uint64_t id = ids[k];
  const uint32_t H = crops ? samples[k].height : 0, W = crops ? samples[k].width : 0;
  int err = 0;
  for (int part = 0; part < 3; part++) err |= draw_part(part, k, id, H, W, p, crops, cut, flips);
  if (status) status[k] = err ? FFCV_SAMPLE_RNG : FFCV_SAMPLE_OK;
}

// ------------------------------------------------ raw crop + resize -------
struct GlobalSrc {
  const uint8_t *p;
  uint64_t step;
  FFCV_DEV int at(int y, int x, int c) const { return p[(uint64_t)y * step + (uint64_t)x * 3 + c]; }
};

template <bool FP16>
FFCV_DEV void store_px(void *out, uint64_t idx, const int v[3], const uint16_t *lut) {
  if (FP16) {
    uint16_t *o = (uint16_t *)out + idx * 3;
    o[0] = lut[v[0] * 3 + 0];
    o[1] = lut[v[1] * 3 + 1];
    o[2] = lut[v[2] * 3 + 2];
  } else {
    uint8_t *o = (uint8_t *)out + idx * 3;
    o[0] = (uint8_t)v[0];
    o[1] = (uint8_t)v[1];
    o[2] = (uint8_t)v[2];
  }
}

#define RRC_THREADS 256
#define RRC_BAND 16  // output rows per workgroup

// One workgroup per band of RRC_BAND output rows of one image.
//   Linear fast path (every crop upscaled along some axis, OpenCV's
//   "area-mode" linear with the SSE2 vertical body on every element): each
//   thread owns one output column pair and walks the band's rows, keeping
//   the two source rows' horizontal sums in registers, so the column taps
//   are computed once per thread and each source row once per column pair.
//   Otherwise (area downscale, odd widths): the per-pixel restatement.
template <bool FP16>
__global__ void __launch_bounds__(RRC_THREADS)
    rrc_raw_kernel(const uint8_t *__restrict__ base, const ffcv_sample *__restrict__ samples,
                   const int32_t *__restrict__ crops, const int32_t *__restrict__ cut,
                   const uint8_t *__restrict__ flips, ffcv_rrc_params p, uint64_t stride,
                   void *__restrict__ out) {
  __shared__ uint16_t s_lut[FP16 ? 768 : 1];
  __shared__ LinTap s_rt[RRC_BAND];
  const int k = blockIdx.y;
  const int t = threadIdx.x;
  const ffcv_sample s = samples[k];
  if (FP16) {
    for (int i = t; i < 768; i += RRC_THREADS) s_lut[i] = p.lut[i];
    __syncthreads();
  }
  if (s.mode != 1) return;
  const int oy0 = blockIdx.x * RRC_BAND, oy1 = min(p.out_h, oy0 + RRC_BAND);
  if (oy0 >= p.out_h) return;
  const int ci = crops[4 * k], cj = crops[4 * k + 1], chh = crops[4 * k + 2], cww = crops[4 * k + 3];
  GlobalSrc src{base + s.offset + ((uint64_t)ci * s.width + cj) * 3, (uint64_t)s.width * 3};
  ResizePlan P = make_plan(cww, chh, p.out_w, p.out_h);
  Epilogue ep;
  ep.out_h = p.out_h;
  ep.out_w = p.out_w;
  ep.cut_size = cut ? p.cutout_size : 0;
  ep.cut_y = cut ? cut[2 * k] : 0;
  ep.cut_x = cut ? cut[2 * k + 1] : 0;
  ep.flip = flips ? flips[k] : 0;
  ep.cut_before_flip = p.cutout_fill[3];
  ep.fill[0] = p.cutout_fill[0];
  ep.fill[1] = p.cutout_fill[1];
  ep.fill[2] = p.cutout_fill[2];
  char *o = (char *)out + stride * k;
  const int out_w = p.out_w;
  if (P.kind == 3 && P.vec_end == 3 * out_w && (out_w & 1) == 0 && out_w <= 2 * RRC_THREADS) {
    if (t < oy1 - oy0) s_rt[t] = lin_tap(P.scale_y, P.inv_y, P.sh, oy0 + t);
    __syncthreads();
    if (t >= out_w / 2) return;
    const int dx0 = 2 * t;
    const LinTap l0 = lin_tap(P.scale_x, P.inv_x, P.sw, ep.src_x(dx0));
    const LinTap l1 = lin_tap(P.scale_x, P.inv_x, P.sw, ep.src_x(dx0 + 1));
    // a border tap (src[s] * 2048) as the two-tap form with weights (2048, 0)
    const int a0w = l0.border ? 2048 : l0.c0, b0w = l0.border ? 0 : l0.c1, s0b = l0.border ? l0.s : l0.s + 1;
    const int a1w = l1.border ? 2048 : l1.c0, b1w = l1.border ? 0 : l1.c1, s1b = l1.border ? l1.s : l1.s + 1;
    auto hrow = [&](int r, int H[6]) {  // resize.cpp HResizeLinear of crop row r: sat_s16(h >> 4)
      const uint8_t *row = src.p + (uint64_t)r * src.step;
#pragma unroll
      for (int c = 0; c < 3; c++) {
        const int a0 = row[l0.s * 3 + c], b0 = row[s0b * 3 + c];
        const int a1 = row[l1.s * 3 + c], b1 = row[s1b * 3 + c];
        H[c] = sat_s16i((a0 * a0w + b0 * b0w) >> 4);
        H[3 + c] = sat_s16i((a1 * a1w + b1 * b1w) >> 4);
      }
    };
    int ca = -1, cb = -1;
    int HA[6], HB[6];
    for (int dy = oy0; dy < oy1; dy++) {
      const LinTap ly = s_rt[dy - oy0];
      const int ra = min(max(ly.s, 0), P.sh - 1), rb = min(max(ly.s + 1, 0), P.sh - 1);
      if (ra != ca) {
        if (ra == cb) {
#pragma unroll
          for (int i = 0; i < 6; i++) HA[i] = HB[i];
        } else {
          hrow(ra, HA);
        }
        ca = ra;
      }
      if (rb != cb) {
        hrow(rb, HB);
        cb = rb;
      }
      int v[6];
#pragma unroll
      for (int i = 0; i < 6; i++) {  // VResizeLinearVec_32s8u
        const int m0 = __mul24(HA[i], ly.c0) >> 16, m1 = __mul24(HB[i], ly.c1) >> 16;  // |HA| < 2^15, c <= 2048
        v[i] = sat_u8i((sat_s16i(m0 + m1) + 2) >> 2);
      }
      if (ep.in_cut(dy, dx0)) {
        v[0] = ep.fill[0];
        v[1] = ep.fill[1];
        v[2] = ep.fill[2];
      }
      if (ep.in_cut(dy, dx0 + 1)) {
        v[3] = ep.fill[0];
        v[4] = ep.fill[1];
        v[5] = ep.fill[2];
      }
      const uint64_t px = (uint64_t)dy * out_w + dx0;
      if (FP16) {  // 12-byte group, 4-byte aligned (dx0 even)
        uint32_t *o32 = (uint32_t *)((uint16_t *)o + px * 3);
        const uint32_t h0 = s_lut[v[0] * 3], h1 = s_lut[v[1] * 3 + 1], h2 = s_lut[v[2] * 3 + 2];
        const uint32_t h3 = s_lut[v[3] * 3], h4 = s_lut[v[4] * 3 + 1], h5 = s_lut[v[5] * 3 + 2];
        o32[0] = h0 | (h1 << 16);
        o32[1] = h2 | (h3 << 16);
        o32[2] = h4 | (h5 << 16);
      } else {
        uint16_t *o16 = (uint16_t *)((uint8_t *)o + px * 3);
        o16[0] = (uint16_t)(v[0] | (v[1] << 8));
        o16[1] = (uint16_t)(v[2] | (v[3] << 8));
        o16[2] = (uint16_t)(v[4] | (v[5] << 8));
      }
    }
    return;
  }
  const int npx = (oy1 - oy0) * out_w;
  for (int i = t; i < npx; i += RRC_THREADS) {
    const int dy = oy0 + i / out_w, dx = i % out_w;
    int v[3];
    if (ep.in_cut(dy, dx)) {
      v[0] = ep.fill[0];
      v[1] = ep.fill[1];
      v[2] = ep.fill[2];
    } else {
      resize_pixel(P, src, dy, ep.src_x(dx), v);
    }
    store_px<FP16>(o, (uint64_t)dy * out_w + dx, v, s_lut);
  }
}

// --------------------------------------------- simple (raw) gather -------
__global__ void __launch_bounds__(256) gather_raw_kernel(const uint8_t *__restrict__ base,
                                                         const ffcv_sample *__restrict__ samples,
                                                         uint8_t *__restrict__ out, uint64_t stride) {
  const int k = blockIdx.y;
  const ffcv_sample s = samples[k];
  if (s.mode != 1) return;
  const uint8_t *src = base + s.offset;
  uint8_t *dst = out + stride * k;
  uint64_t n = s.size;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256)
    dst[i] = src[i];
}

__global__ void __launch_bounds__(256) gather_samples_kernel(const ffcv_sample *__restrict__ table, uint64_t n,
                                                             const uint64_t *__restrict__ ids, int B,
                                                             ffcv_sample *__restrict__ out) {
  int k = blockIdx.x * 256 + threadIdx.x;
  if (k >= B) return;
  uint64_t i = ids[k];
  ffcv_sample s;
  if (i < n) {
    s = table[i];
  } else {  // out-of-range index: an empty jpg sample -> BAD_MARKER status
    s.offset = 0;
    s.size = 0;
    s.height = s.width = 1;
    s.mode = 0;
    s.reserved = 0;
  }
  out[k] = s;
}

// ------------------------------------------------------ standalone -------
__global__ void __launch_bounds__(256) cutout_kernel(uint8_t *__restrict__ img, int H, int W,
                                                     const int32_t *__restrict__ yx, int c, uint8_t f0,
                                                     uint8_t f1, uint8_t f2) {
  const int k = blockIdx.x;
  const int y0 = yx[2 * k], x0 = yx[2 * k + 1];
  uint8_t *base = img + (uint64_t)k * H * W * 3;
  for (int i = threadIdx.x; i < c * c; i += 256) {
    int y = y0 + i / c, x = x0 + i % c;
    if (y < H && x < W) {
      uint8_t *p = base + ((uint64_t)y * W + x) * 3;
      p[0] = f0;
      p[1] = f1;
      p[2] = f2;
    }
  }
}

// normalize.py:65: output = table[input * 3 + i % 3]; 12 elements (4 RGB
// pixels) per lane so loads/stores are dword-shaped.
__global__ void __launch_bounds__(256) normalize_kernel(const uint8_t *__restrict__ in, uint64_t n,
                                                        const uint16_t *__restrict__ lut,
                                                        uint16_t *__restrict__ out) {
  __shared__ uint16_t s_lut[768];
  for (int i = threadIdx.x; i < 768; i += 256) s_lut[i] = lut[i];
  __syncthreads();
  uint64_t groups = n / 12;
  for (uint64_t g = (uint64_t)blockIdx.x * 256 + threadIdx.x; g < groups; g += (uint64_t)gridDim.x * 256) {
    const uint8_t *ip = in + g * 12;
    uint16_t *op = out + g * 12;
#pragma unroll
    for (int e = 0; e < 12; e++) op[e] = s_lut[ip[e] * 3 + (e % 3)];
  }
  if (blockIdx.x == 0) {
    for (uint64_t i = groups * 12 + threadIdx.x; i < n; i += 256) out[i] = s_lut[in[i] * 3 + (i % 3)];
  }
}

__global__ void __launch_bounds__(256) flip_kernel(const uint8_t *__restrict__ in, uint8_t *__restrict__ out,
                                                   int H, int W, int cb, const uint8_t *__restrict__ flips) {
  const int k = blockIdx.y;
  const uint64_t img = (uint64_t)H * W * cb;
  const bool f = flips[k] != 0;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < img; i += (uint64_t)gridDim.x * 256) {
    uint64_t px = i / cb;
    int b = (int)(i - px * cb);
    int y = (int)(px / W), x = (int)(px - (uint64_t)y * W);
    int sx = f ? W - 1 - x : x;
    out[k * img + i] = in[k * img + ((uint64_t)y * W + sx) * cb + b];
  }
}

// ---------------------------------------------------------- C ABI -------
extern "C" {

int ffcv_draw_batch(void *stream, const uint64_t *sample_ids, const ffcv_sample *samples, int batch,
                    const ffcv_draw_params *p, int32_t *crops, int32_t *cutout_yx, uint8_t *flips,
                    int32_t *status) {
  if (batch < 0 || !p || !sample_ids || (crops && !samples)) {
    ffcv::set_error("ffcv_draw_batch: invalid arguments");
    return FFCV_EINVAL;
  }
  if (batch == 0) return FFCV_OK;
  if (p->cutout_size > 0 && (p->cutout_size > p->out_h || p->cutout_size > p->out_w)) {
    ffcv::set_error("ffcv_draw_batch: cutout_size %d exceeds output %dx%d", p->cutout_size, p->out_h,
                    p->out_w);
    return FFCV_EINVAL;
  }
  hipLaunchKernelGGL(draw_kernel, dim3((batch + 63) / 64), dim3(64), 0, ffcv::as_stream(stream),
                     sample_ids, samples, batch, *p, crops, cutout_yx, flips, status);
  FFCV_LAUNCH_CHECK("draw_kernel");
  return FFCV_OK;
}

int ffcv_rrc_raw_batch(void *stream, const uint8_t *base, const ffcv_sample *samples, int batch,
                       const int32_t *crops, const int32_t *cutout_yx, const uint8_t *flips,
                       const ffcv_rrc_params *p, void *out) {
  if (batch < 0 || !p || !base || !samples || !crops || !out || p->out_h <= 0 || p->out_w <= 0) {
    ffcv::set_error("ffcv_rrc_raw_batch: invalid arguments");
    return FFCV_EINVAL;
  }
  if (batch == 0) return FFCV_OK;
  const bool fp16 = p->lut != nullptr;
  uint64_t dense = (uint64_t)p->out_h * p->out_w * 3 * (fp16 ? 2 : 1);
  uint64_t stride = p->out_stride ? p->out_stride : dense;
  dim3 grid((p->out_h + RRC_BAND - 1) / RRC_BAND, batch);
  if (fp16)
    hipLaunchKernelGGL(rrc_raw_kernel<true>, grid, dim3(RRC_THREADS), 0, ffcv::as_stream(stream), base,
                       samples, crops, cutout_yx, flips, *p, stride, out);
  else
    hipLaunchKernelGGL(rrc_raw_kernel<false>, grid, dim3(RRC_THREADS), 0, ffcv::as_stream(stream), base,
                       samples, crops, cutout_yx, flips, *p, stride, out);
  FFCV_LAUNCH_CHECK("rrc_raw_kernel");
  return FFCV_OK;
}

int ffcv_gather_samples(void *stream, const ffcv_sample *table, uint64_t n_table, const uint64_t *ids,
                        int batch, ffcv_sample *out) {
  if (!table || !ids || !out || batch < 0) {
    ffcv::set_error("ffcv_gather_samples: invalid arguments");
    return FFCV_EINVAL;
  }
  if (batch == 0) return FFCV_OK;
  hipLaunchKernelGGL(gather_samples_kernel, dim3((batch + 255) / 256), dim3(256), 0, ffcv::as_stream(stream),
                     table, n_table, ids, batch, out);
  FFCV_LAUNCH_CHECK("gather_samples_kernel");
  return FFCV_OK;
}

int ffcv_gather_raw_batch(void *stream, const uint8_t *base, const ffcv_sample *samples, int batch,
                          uint8_t *out, uint64_t out_stride) {
  if (batch < 0 || !base || !samples || !out || !out_stride) {
    ffcv::set_error("ffcv_gather_raw_batch: invalid arguments");
    return FFCV_EINVAL;
  }
  if (batch == 0) return FFCV_OK;
  unsigned gx = (unsigned)((out_stride + 255) / 256);
  if (gx > 64) gx = 64;
  hipLaunchKernelGGL(gather_raw_kernel, dim3(gx, batch), dim3(256), 0, ffcv::as_stream(stream), base,
                     samples, out, out_stride);
  FFCV_LAUNCH_CHECK("gather_raw_kernel");
  return FFCV_OK;
}

int ffcv_cutout_batch(void *stream, uint8_t *images, int batch, int height, int width,
                      const int32_t *cutout_yx, int crop_size, const uint8_t fill[3]) {
  if (batch < 0 || !images || !cutout_yx || crop_size <= 0 || crop_size > height || crop_size > width) {
    ffcv::set_error("ffcv_cutout_batch: invalid arguments");
    return FFCV_EINVAL;
  }
  if (batch == 0) return FFCV_OK;
  hipLaunchKernelGGL(cutout_kernel, dim3(batch), dim3(256), 0, ffcv::as_stream(stream), images, height,
                     width, cutout_yx, crop_size, fill[0], fill[1], fill[2]);
  FFCV_LAUNCH_CHECK("cutout_kernel");
  return FFCV_OK;
}

int ffcv_normalize_batch(void *stream, const uint8_t *in, uint64_t n, const uint16_t *lut, uint16_t *out) {
  if (!in || !lut || !out) {
    ffcv::set_error("ffcv_normalize_batch: invalid arguments");
    return FFCV_EINVAL;
  }
  if (n == 0) return FFCV_OK;
  uint64_t groups = n / 12 + 1;
  unsigned gx = (unsigned)((groups + 255) / 256);
  if (gx > 4096) gx = 4096;
  hipLaunchKernelGGL(normalize_kernel, dim3(gx), dim3(256), 0, ffcv::as_stream(stream), in, n, lut, out);
  FFCV_LAUNCH_CHECK("normalize_kernel");
  return FFCV_OK;
}

int ffcv_flip_batch(void *stream, const uint8_t *in, uint8_t *out, int batch, int height, int width,
                    int channels_bytes, const uint8_t *flips) {
  if (batch < 0 || !in || !out || !flips || in == out || height <= 0 || width <= 0 || channels_bytes <= 0) {
    ffcv::set_error("ffcv_flip_batch: invalid arguments (in-place flip unsupported)");
    return FFCV_EINVAL;
  }
  if (batch == 0) return FFCV_OK;
  uint64_t img = (uint64_t)height * width * channels_bytes;
  unsigned gx = (unsigned)((img + 255) / 256);
  if (gx > 256) gx = 256;
  hipLaunchKernelGGL(flip_kernel, dim3(gx, batch), dim3(256), 0, ffcv::as_stream(stream), in, out, height,
                     width, channels_bytes, flips);
  FFCV_LAUNCH_CHECK("flip_kernel");
  return FFCV_OK;
}

}  // extern "C"
