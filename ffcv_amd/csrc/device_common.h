// device_common.h -- device helpers shared by the gfx950 kernels.
//
// Everything here is compiled with -ffp-contract=off: the INTER_AREA float
// accumulation and the crop draws must round exactly like the reference's
// scalar code (OpenCV 4.5.4 resize.cpp, numpy/numba RandomState).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/ffcv_hip.h"

#define FFCV_DEV __device__ __forceinline__
typedef unsigned short u16x2_t __attribute__((ext_vector_type(2)));  // v_dot2_u32_u16 operands
// The INTER_AREA restatement below is single-source: the kernels run it per
// output pixel and the host C-ABI resize() (csrc/ffcv_host.hip, the
// reference's libffcv.cpp:33-42 signature) runs the very same functions on
// the CPU.  These helpers pick the gfx950 instruction on the device pass.
#define FFCV_HD __host__ __device__ __forceinline__
// raw buffer resources: a load past num_records returns 0, a store is dropped
#define BUF_OOR 0x7ffffff0u  // an offset past every buffer's num_records
#define BUF_CFG 0x00020000   // raw buffer resource word 3 (gfx9 family)

FFCV_HD int ffcv_f2i_rn(float x) {  // round half to even, like cvRound
#if defined(__HIP_DEVICE_COMPILE__)
  return __float2int_rn(x);
#else
  return (int)nearbyintf(x);
#endif
}
FFCV_HD int ffcv_mul24(int a, int b) {  // operands < 2^23 in magnitude here
#if defined(__HIP_DEVICE_COMPILE__)
  return __mul24(a, b);
#else
  return a * b;
#endif
}
FFCV_HD uint32_t ffcv_f2u_bits(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __float_as_uint(x);
#else
  uint32_t u;
  __builtin_memcpy(&u, &x, 4);
  return u;
#endif
}
FFCV_HD float ffcv_u2f_bits(uint32_t u) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __uint_as_float(u);
#else
  float x;
  __builtin_memcpy(&x, &u, 4);
  return x;
#endif
}

// --------------------------------------------------------------------------
// MT19937 with O(1) state.
//
// The reference draws crops with numba's np.random (per-thread MT19937,
// rgb_image.py:51-58) and cutout origins with np.random.randint
// (cutout.py:38-42).  Under our seeding contract every (op, sample, epoch)
// owns a fresh generator seeded with init_genrand(seed) (numpy legacy
// RandomState.seed(int)).  A fresh generator's first 227 outputs need only
// the INITIAL state words old[n], old[n+1], old[n+397] (the twist of word n <
// 227 reads no updated word), and the initial state is a recurrence
// old[k] = 1812433253*(old[k-1]^(old[k-1]>>30)) + k.  So two cursors walking
// that recurrence (one at n, one at n+397) produce the stream with three
// registers instead of a 2.5 KB state.  Outputs 227..623 are recomputed on a
// slow path; beyond 623 the stream reports an error (a crop needs <= 44
// words, a cutout origin ~4).
// --------------------------------------------------------------------------
struct DevMT {
  uint32_t seed;
  uint32_t a0, a1;  // old[n], old[n+1]
  uint32_t b;       // old[n+397]
  int n;
  int err;
};

FFCV_HD uint32_t mt_chain(uint32_t x, uint32_t k) { return 1812433253u * (x ^ (x >> 30)) + k; }
FFCV_HD uint32_t mt_temper(uint32_t y) {
  y ^= (y >> 11);
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= (y >> 18);
  return y;
}
FFCV_HD uint32_t mt_twist1(uint32_t lo_src, uint32_t hi_next, uint32_t far) {
  uint32_t y = (lo_src & 0x80000000u) | (hi_next & 0x7fffffffu);
  return far ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
}
FFCV_HD void mt_init(DevMT &m, uint32_t seed) {
  m.seed = seed;
  m.a0 = seed;
  m.a1 = mt_chain(seed, 1);
  uint32_t x = seed;
  for (uint32_t k = 1; k <= 397; k++) x = mt_chain(x, k);
  m.b = x;
  m.n = 0;
  m.err = 0;
}
static __host__ __device__ __noinline__ uint32_t mt_old_at(uint32_t seed, int k) {
  uint32_t x = seed;
  for (int i = 1; i <= k; i++) x = mt_chain(x, (uint32_t)i);
  return x;
}
static __host__ __device__ __noinline__ uint32_t mt_new_at(uint32_t seed, int m) {
  if (m < 227) return mt_twist1(mt_old_at(seed, m), mt_old_at(seed, m + 1), mt_old_at(seed, m + 397));
  if (m < 623) return mt_twist1(mt_old_at(seed, m), mt_old_at(seed, m + 1), mt_new_at(seed, m - 227));
  return mt_twist1(mt_old_at(seed, 623), mt_new_at(seed, 0), mt_new_at(seed, 396));
}
FFCV_HD uint32_t mt_u32(DevMT &m) {
  uint32_t v;
  if (m.n < 227) {
    v = mt_twist1(m.a0, m.a1, m.b);
    m.a0 = m.a1;
    m.a1 = mt_chain(m.a1, (uint32_t)(m.n + 2));
    m.b = mt_chain(m.b, (uint32_t)(m.n + 398));
  } else if (m.n < 624) {
    v = mt_new_at(m.seed, m.n);
  } else {
    m.err = 1;
    v = 0;
  }
  m.n++;
  return mt_temper(v);
}
// genrand_res53 == numpy mt19937_next_double == numba get_next_double
FFCV_HD double mt_double(DevMT &m) {
  int32_t a = (int32_t)(mt_u32(m) >> 5);
  int32_t b = (int32_t)(mt_u32(m) >> 6);
  return (a * 67108864.0 + b) / 9007199254740992.0;
}
FFCV_HD double mt_uniform(DevMT &m, double lo, double hi) {
  double range = hi - lo;
  return lo + range * mt_double(m);
}
// legacy RandomState.randint(high): masked rejection on 32-bit draws
FFCV_HD int64_t mt_randint(DevMT &m, int64_t high) {
  uint64_t rng = (uint64_t)(high - 1);
  if (rng == 0) return 0;
  uint64_t mask = rng;
  mask |= mask >> 1;
  mask |= mask >> 2;
  mask |= mask >> 4;
  mask |= mask >> 8;
  mask |= mask >> 16;
  mask |= mask >> 32;
  uint64_t v;
  do {
    v = mt_u32(m) & mask;
  } while (v > rng && !m.err);
  return (int64_t)v;
}

FFCV_HD uint64_t splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
// Seeding contract: op ids 1 = crop, 2 = cutout, 3 = flip.
FFCV_HD uint32_t sample_seed(uint64_t loader_seed, uint64_t epoch, uint64_t sample, uint32_t op) {
  uint64_t h = splitmix64(loader_seed ^ ((uint64_t)op << 56));
  h = splitmix64(h ^ epoch);
  h = splitmix64(h ^ sample);
  return (uint32_t)h;
}

// rgb_image.py:48-72 get_random_crop (Python round() = half-to-even = rint)
FFCV_HD void random_crop(DevMT &m, uint32_t height, uint32_t width, const double *scale,
                          const double *ratio, int32_t *out) {
  uint32_t area = height * width;
  double lr0 = log(ratio[0]), lr1 = log(ratio[1]);
  for (int t = 0; t < 10; t++) {
    double target_area = (double)area * mt_uniform(m, scale[0], scale[1]);
    double aspect = exp(mt_uniform(m, lr0, lr1));
    int64_t w = (int64_t)rint(sqrt(target_area * aspect));
    int64_t h = (int64_t)rint(sqrt(target_area / aspect));
    if (0 < w && w <= (int64_t)width && 0 < h && h <= (int64_t)height) {
      int64_t i = (int64_t)mt_uniform(m, 0.0, (double)((int64_t)height - h + 1));
      int64_t j = (int64_t)mt_uniform(m, 0.0, (double)((int64_t)width - w + 1));
      out[0] = (int32_t)i;
      out[1] = (int32_t)j;
      out[2] = (int32_t)h;
      out[3] = (int32_t)w;
      return;
    }
  }
  double in_ratio = (double)width / (double)height;
  double rmin = fmin(ratio[0], ratio[1]), rmax = fmax(ratio[0], ratio[1]);
  int64_t w, h;
  if (in_ratio < rmin) {
    w = width;
    h = (int64_t)rint((double)w / rmin);
  } else if (in_ratio > rmax) {
    h = height;
    w = (int64_t)rint((double)h * rmax);
  } else {
    w = width;
    h = height;
  }
  out[0] = (int32_t)(((int64_t)height - h) / 2);
  out[1] = (int32_t)(((int64_t)width - w) / 2);
  out[2] = (int32_t)h;
  out[3] = (int32_t)w;
}

// rgb_image.py:75-81 get_center_crop
FFCV_HD void center_crop(uint32_t height, uint32_t width, double ratio, int32_t *out) {
  uint32_t s = height < width ? height : width;
  int64_t c = (int64_t)(ratio * (double)s);
  out[0] = (int32_t)(((int64_t)height - c) / 2);
  out[1] = (int32_t)(((int64_t)width - c) / 2);
  out[2] = (int32_t)c;
  out[3] = (int32_t)c;
}

// The draws of one sample under the seeding contract: part 0 =
// crop (rgb_image.py:48-81) -> crops[4k..], part 1 = cutout origin
// (cutout.py:38-42) -> cut[2k..], part 2 = flip (flip.py:35) -> flips[k].
// Returns 1 when the MT19937 stream ran out (FFCV_SAMPLE_RNG).
FFCV_HD int draw_part(int part, int k, uint64_t id, uint32_t H, uint32_t W, const ffcv_draw_params &p,
                       int32_t *crops, int32_t *cut, uint8_t *flips) {
  // Each part's stream is seeded before the per-part branches (op id = part
  // + 1): the entropy kernel draws a sample's three parts on three lanes side
  // by side, which then run the 397-step seeding chain once, together,
  // instead of once per branch (three serial chains at every workgroup start)
  DevMT m;
  mt_init(m, sample_seed(p.loader_seed, p.epoch, id, (uint32_t)part + 1));
  if (part == 0 && crops) {
    int32_t c[4];
    int err = 0;
    if (p.crop_kind == 0) {
      random_crop(m, H, W, p.scale, p.ratio, c);
      err = m.err;
    } else {
      center_crop(H, W, p.center_ratio, c);
    }
    crops[4 * k + 0] = c[0];
    crops[4 * k + 1] = c[1];
    crops[4 * k + 2] = c[2];
    crops[4 * k + 3] = c[3];
    return err;
  }
  if (part == 1 && cut && p.cutout_size > 0) {
    cut[2 * k + 0] = (int32_t)mt_randint(m, p.out_h - p.cutout_size + 1);
    cut[2 * k + 1] = (int32_t)mt_randint(m, p.out_w - p.cutout_size + 1);
    return m.err;
  }
  if (part == 2 && flips) {
    flips[k] = (uint8_t)(mt_double(m) < p.flip_prob);
  }
  return 0;
}


// --------------------------------------------------------------------------
// OpenCV 4.5.4 cv::resize(ROI, dst, dsize, 0, 0, INTER_AREA), CV_8UC3
// (libffcv.cpp:33-42), restated per OUTPUT PIXEL so one lane computes one
// pixel with exactly the reference's operation order:
//   kind 0  dsize == ssize: copy
//   kind 1  integer scales >= 1: resizeAreaFast (float sum*(1/area), rint)
//   kind 2  both scales >= 1: ResizeArea_Invoker (float taps in table order)
//   kind 3  otherwise: "area-mode" 2-tap Q11 linear (resizeGeneric_), with
//           the SSE2 vertical body for elements < vec_end, scalar tail after
// --------------------------------------------------------------------------
struct ResizePlan {
  int sw, sh, dw, dh;
  int kind;
  int isx, isy;
  int vec_end;
  double scale_x, scale_y, inv_x, inv_y;
};

FFCV_HD ResizePlan make_plan(int sw, int sh, int dw, int dh) {
  ResizePlan p;
  p.sw = sw;
  p.sh = sh;
  p.dw = dw;
  p.dh = dh;
  p.inv_x = (double)dw / sw;
  p.inv_y = (double)dh / sh;
  p.scale_x = 1. / p.inv_x;
  p.scale_y = 1. / p.inv_y;
  p.isx = (int)rint(p.scale_x);
  p.isy = (int)rint(p.scale_y);
  bool fast = fabs(p.scale_x - p.isx) < 2.220446049250313e-16 &&
              fabs(p.scale_y - p.isy) < 2.220446049250313e-16;
  if (sw == dw && sh == dh)
    p.kind = 0;
  else if (p.scale_x >= 1 && p.scale_y >= 1)
    p.kind = fast ? 1 : 2;
  else
    p.kind = 3;
  int width = dw * 3, x = 0;
  for (; x <= width - 16; x += 16) {
  }
  for (; x < width - 8; x += 8) {
  }
  p.vec_end = x;
  return p;
}

FFCV_HD int sat_u8i(int v) { return v < 0 ? 0 : (v > 255 ? 255 : v); }
FFCV_HD int sat_s16i(int v) { return v < -32768 ? -32768 : (v > 32767 ? 32767 : v); }

// computeResizeAreaTab entries for one destination index, as a contiguous
// source range [lo, hi] with a partial weight at either end (table order is
// ascending source index, which is the reference's accumulation order).
struct AreaTaps {
  int lo, hi;       // inclusive source range
  int left, right;  // partial-tap indices (or -1)
  float wl, wf, wr;
  // s == left ? wl : (s == right ? wr : wf), as register selects (a plain
  // ternary on members becomes a scratch-array lookup)
  FFCV_HD float w(int s) const {
    uint32_t r = ffcv_f2u_bits(wf);
    r = s == right ? ffcv_f2u_bits(wr) : r;
    r = s == left ? ffcv_f2u_bits(wl) : r;
    return ffcv_u2f_bits(r);
  }
};
FFCV_HD AreaTaps area_taps(int ssize, double scale, int d) {
  AreaTaps t;
  double fsx1 = d * scale;
  double fsx2 = fsx1 + scale;
  double cellWidth = fmin(scale, ssize - fsx1);
  int sx1 = (int)ceil(fsx1), sx2 = (int)floor(fsx2);
  sx2 = min(sx2, ssize - 1);
  sx1 = min(sx1, sx2);
  t.left = -1;
  t.right = -1;
  t.lo = sx1;
  t.hi = sx2 - 1;
  t.wl = t.wr = 0.f;
  if (sx1 - fsx1 > 1e-3) {
    t.left = sx1 - 1;
    t.lo = sx1 - 1;
    t.wl = (float)((sx1 - fsx1) / cellWidth);
  }
  t.wf = (float)(1.0 / cellWidth);
  if (fsx2 - sx2 > 1e-3) {
    t.right = sx2;
    t.hi = sx2;
    t.wr = (float)(fmin(fmin(fsx2 - sx2, 1.), cellWidth) / cellWidth);
  }
  return t;
}

// Linear ("area mode") coefficient for one destination index.
FFCV_HD void linear_coef(double scale, double inv, int ssize, int d, int *s_out, int16_t *c0,
                          int16_t *c1, bool *border) {
  int s = (int)floor(d * scale);
  float f = (float)((d + 1) - (s + 1) * inv);
  f = f <= 0 ? 0.f : f - (float)(int)floorf(f);
  bool b = false;
  if (s + 1 >= ssize) {
    b = true;
    if (s >= ssize - 1) {
      f = 0;
      s = ssize - 1;
    }
  }
  *s_out = s;
  *border = b;
  *c0 = (int16_t)sat_s16i(ffcv_f2i_rn((1.f - f) * 2048.f));
  *c1 = (int16_t)sat_s16i(ffcv_f2i_rn(f * 2048.f));
}

// Linear taps of one destination index (linear_coef, precomputable).
struct LinTap {
  int s;
  int c0, c1;
  int border;
};
FFCV_HD LinTap lin_tap(double scale, double inv, int ssize, int d) {
  LinTap t;
  int16_t c0, c1;
  bool b;
  linear_coef(scale, inv, ssize, d, &t.s, &c0, &c1, &b);
  t.c0 = c0;
  t.c1 = c1;
  t.border = b;
  return t;
}

// Linear taps (resize.cpp linear coefficients, LinTap) packed in 8 bytes:
// x = source index | border << 31, y = c0 | c1 << 16 (0 <= c0, c1 <= 2048).
// Written once per image (K1 for JPEG, rrc_taps_kernel for raw samples) and
// read by every band workgroup of the image.
FFCV_DEV uint2 tap_pack(const LinTap &l) {
  return make_uint2((uint32_t)l.s | ((uint32_t)l.border << 31), (uint32_t)(l.c0 & 0xffff) | ((uint32_t)l.c1 << 16));
}
FFCV_DEV LinTap tap_unpack(uint2 v) {
  LinTap l;
  l.s = (int)(v.x & 0x7fffffffu);
  l.border = (int)(v.x >> 31);
  l.c0 = (int)(int16_t)(v.y & 0xffff);
  l.c1 = (int)(int16_t)(v.y >> 16);
  return l;
}

// Source accessor: pixel (y, x) channel c of the ROI.
struct RoiSrc {
  const uint8_t *p;
  uint64_t step;  // bytes per row
  FFCV_HD int at(int y, int x, int c) const { return p[(uint64_t)y * step + (uint64_t)x * 3 + c]; }
};

// INTER_AREA general path for one output pixel from its column/row taps.
template <class Src>
FFCV_HD void resize_area(const Src &S, const AreaTaps &tx, const AreaTaps &ty, int out[3]) {
  float sum0 = 0.f, sum1 = 0.f, sum2 = 0.f;
  for (int sy = ty.lo; sy <= ty.hi; sy++) {
    float buf0 = 0.f, buf1 = 0.f, buf2 = 0.f;
    for (int sx = tx.lo; sx <= tx.hi; sx++) {
      const float a = tx.w(sx);
      buf0 = buf0 + (float)S.at(sy, sx, 0) * a;
      buf1 = buf1 + (float)S.at(sy, sx, 1) * a;
      buf2 = buf2 + (float)S.at(sy, sx, 2) * a;
    }
    const float beta = ty.w(sy);
    if (sy == ty.lo) {
      sum0 = beta * buf0;
      sum1 = beta * buf1;
      sum2 = beta * buf2;
    } else {
      sum0 = sum0 + beta * buf0;
      sum1 = sum1 + beta * buf1;
      sum2 = sum2 + beta * buf2;
    }
  }
  out[0] = sat_u8i(ffcv_f2i_rn(sum0));
  out[1] = sat_u8i(ffcv_f2i_rn(sum1));
  out[2] = sat_u8i(ffcv_f2i_rn(sum2));
}

// resize_area on an LDS-staged source (S.pix(y, x): the byte address of pixel
// (y, x), RGB): the same arithmetic, each tap pixel's three bytes from two
// ALIGNED 4-byte LDS reads joined by v_alignbyte.  Byte reads of adjacent
// channels are merged by the compiler into 2-byte reads at odd addresses, and
// misaligned LDS reads made the raw kernel's area walk 4-5x slower (round 5).
// Reads up to 5 bytes past the last pixel: the caller keeps them inside LDS.
template <class Src>
FFCV_DEV void resize_area_lds(const Src &S, const AreaTaps &tx, const AreaTaps &ty, int out[3]) {
  float sum0 = 0.f, sum1 = 0.f, sum2 = 0.f;
  for (int sy = ty.lo; sy <= ty.hi; sy++) {
    float buf0 = 0.f, buf1 = 0.f, buf2 = 0.f;
    for (int sx = tx.lo; sx <= tx.hi; sx++) {
      const float a = tx.w(sx);
      const uint8_t *q = S.pix(sy, sx);
      const uint32_t *qa = (const uint32_t *)__builtin_align_down(q, 4);
      const uint32_t v = __builtin_amdgcn_alignbyte(qa[1], qa[0], (uint32_t)(q - (const uint8_t *)qa));
      buf0 = buf0 + (float)(v & 0xffu) * a;
      buf1 = buf1 + (float)((v >> 8) & 0xffu) * a;
      buf2 = buf2 + (float)((v >> 16) & 0xffu) * a;
    }
    const float beta = ty.w(sy);
    if (sy == ty.lo) {
      sum0 = beta * buf0;
      sum1 = beta * buf1;
      sum2 = beta * buf2;
    } else {
      sum0 = sum0 + beta * buf0;
      sum1 = sum1 + beta * buf1;
      sum2 = sum2 + beta * buf2;
    }
  }
  out[0] = sat_u8i(ffcv_f2i_rn(sum0));
  out[1] = sat_u8i(ffcv_f2i_rn(sum1));
  out[2] = sat_u8i(ffcv_f2i_rn(sum2));
}

// Area-mode linear (Q11) path for one output pixel; dx is the destination
// column (the SSE2-body / scalar-tail split depends on it).
template <class Src>
FFCV_HD void resize_linear(const ResizePlan &P, const Src &S, int dx, const LinTap &lx, const LinTap &ly,
                            int out[3]) {
  const int sx = lx.s, sy = ly.s;
  const int r0 = sy < 0 ? 0 : (sy >= P.sh ? P.sh - 1 : sy);
  const int r1 = sy + 1 < 0 ? 0 : (sy + 1 >= P.sh ? P.sh - 1 : sy + 1);
#pragma unroll
  for (int c = 0; c < 3; c++) {
    int h0, h1;
    if (lx.border) {
      h0 = S.at(r0, sx, c) * 2048;
      h1 = S.at(r1, sx, c) * 2048;
    } else {
      h0 = S.at(r0, sx, c) * lx.c0 + S.at(r0, sx + 1, c) * lx.c1;
      h1 = S.at(r1, sx, c) * lx.c0 + S.at(r1, sx + 1, c) * lx.c1;
    }
    const int e = dx * 3 + c;
    if (e < P.vec_end) {
      int s0 = sat_s16i(h0 >> 4), s1 = sat_s16i(h1 >> 4);
      int m0 = ffcv_mul24(s0, ly.c0) >> 16, m1 = ffcv_mul24(s1, ly.c1) >> 16;
      int t = sat_s16i(m0 + m1);
      out[c] = sat_u8i((t + 2) >> 2);
    } else {
      out[c] = sat_u8i((h0 * ly.c0 + h1 * ly.c1 + (1 << 21)) >> 22);
    }
  }
}

// Compute the 3 channels of output pixel (dy, dx).
template <class Src>
FFCV_HD void resize_pixel(const ResizePlan &P, const Src &S, int dy, int dx, int out[3]) {
  if (P.kind == 0) {
    for (int c = 0; c < 3; c++) out[c] = S.at(dy, dx, c);
    return;
  }
  if (P.kind == 1) {
    int sy0 = dy * P.isy, sx0 = dx * P.isx;
    float sc = 1.f / (float)(P.isx * P.isy);
    for (int c = 0; c < 3; c++) {
      int sum = 0;
      for (int yy = 0; yy < P.isy; yy++)
        for (int xx = 0; xx < P.isx; xx++) sum += S.at(sy0 + yy, sx0 + xx, c);
      out[c] = sat_u8i(ffcv_f2i_rn((float)sum * sc));
    }
    return;
  }
  if (P.kind == 2) {
    resize_area(S, area_taps(P.sw, P.scale_x, dx), area_taps(P.sh, P.scale_y, dy), out);
    return;
  }
  resize_linear(P, S, dx, lin_tap(P.scale_x, P.inv_x, P.sw, dx), lin_tap(P.scale_y, P.inv_y, P.sh, dy), out);
}

// Source rows of the crop that output rows [oy0, oy1) read.
FFCV_HD void band_rows(const ResizePlan &P, int oy0, int oy1, int *r0, int *r1) {
  if (P.kind == 0) {
    *r0 = oy0;
    *r1 = oy1 - 1;
  } else if (P.kind == 1) {
    *r0 = oy0 * P.isy;
    *r1 = oy1 * P.isy - 1;
  } else if (P.kind == 2) {
    AreaTaps a = area_taps(P.sh, P.scale_y, oy0);
    AreaTaps b = area_taps(P.sh, P.scale_y, oy1 - 1);
    *r0 = a.lo;
    *r1 = b.hi;
  } else {
    int s0 = (int)floor(oy0 * P.scale_y), s1 = (int)floor((oy1 - 1) * P.scale_y) + 1;
    *r0 = s0;
    *r1 = s1;
  }
  *r0 = min(max(*r0, 0), P.sh - 1);
  *r1 = min(max(*r1, 0), P.sh - 1);
}

// Epilogue: flip (flip.py:35-40), cutout (cutout.py:44), LUT (normalize.py:65).
// Returns the source x to resize for output column dx, and whether the
// output pixel is inside the cutout square.
struct Epilogue {
  int out_h, out_w;
  int cut_size;
  int cut_y, cut_x;
  int flip;
  int cut_before_flip;
  uint8_t fill[3];
  FFCV_DEV int src_x(int dx) const { return flip ? out_w - 1 - dx : dx; }
  FFCV_DEV bool in_cut(int dy, int dx) const {
    if (cut_size <= 0) return false;
    // cutout coordinates live in the frame where cutout ran
    int x = (flip && cut_before_flip) ? out_w - 1 - dx : dx;
    return dy >= cut_y && dy < cut_y + cut_size && x >= cut_x && x < cut_x + cut_size;
  }
};
