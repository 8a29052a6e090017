/*
 * ffcv_oracle.c -- CPU restatement of the reference decode-and-augment path.
 *
 * TEST INFRASTRUCTURE ONLY: used by tests/ (parity checker), by
 * __graft_entry__.smoke() (checker) and by bench.py's cpu_baseline leg.
 * The product path (ffcv_amd/) never loads it.
 *
 * Compile with -ffp-contract=off: the INTER_AREA float path and the crop draws
 * must round exactly like the reference's scalar code.
 *
 * Pinning (see DESIGN.md "Oracle"):
 *   - JPEG: bit-exact against libjpeg-turbo 3.1.4 (Pillow-bundled) driven with
 *     the reference's TurboJPEG settings through oracle/ljt_harness.c, and
 *     (islow) against Pillow's own decode.
 *   - crops / cutout / LUT / order: golden vectors produced by the reference's
 *     own Python (tests/golden/make_golden.py, stub harness).
 *   - INTER_AREA: OpenCV is not vendored and not installed; restated from
 *     OpenCV 4.5.4 imgproc/resize.cpp and pinned by the reference's constant-
 *     image invariant (tests/test_rrc.py:63) and identity/integer-scale cases.
 */
#include "ffcv_oracle.h"

#include <fenv.h>
#include <float.h>
#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ======================================================================= */
/* RNG: numpy legacy RandomState (== numba np.random per-thread MT19937)    */
/* ======================================================================= */

/* numpy/random/src/mt19937/mt19937.c mt19937_seed (init_genrand). */
void orc_mt_seed(orc_mt *s, uint32_t seed) {
  for (int pos = 0; pos < 624; pos++) {
    s->key[pos] = seed;
    seed = 1812433253u * (seed ^ (seed >> 30)) + (uint32_t)pos + 1u;
  }
  s->pos = 624;
}

static void mt_twist(orc_mt *s) {
  uint32_t *k = s->key;
  int i;
  uint32_t y;
  for (i = 0; i < 624 - 397; i++) {
    y = (k[i] & 0x80000000u) | (k[i + 1] & 0x7fffffffu);
    k[i] = k[i + 397] ^ (y >> 1) ^ (-(y & 1u) & 0x9908b0dfu);
  }
  for (; i < 623; i++) {
    y = (k[i] & 0x80000000u) | (k[i + 1] & 0x7fffffffu);
    k[i] = k[i + (397 - 624)] ^ (y >> 1) ^ (-(y & 1u) & 0x9908b0dfu);
  }
  y = (k[623] & 0x80000000u) | (k[0] & 0x7fffffffu);
  k[623] = k[396] ^ (y >> 1) ^ (-(y & 1u) & 0x9908b0dfu);
  s->pos = 0;
}

uint32_t orc_mt_u32(orc_mt *s) {
  if (s->pos == 624) mt_twist(s);
  uint32_t y = s->key[s->pos++];
  y ^= (y >> 11);
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= (y >> 18);
  return y;
}

/* genrand_res53 (numpy mt19937_next_double; numba get_next_double). */
double orc_mt_double(orc_mt *s) {
  int32_t a = (int32_t)(orc_mt_u32(s) >> 5), b = (int32_t)(orc_mt_u32(s) >> 6);
  return (a * 67108864.0 + b) / 9007199254740992.0;
}

/* RandomState.uniform(low, high) = low + (high-low)*next_double. */
double orc_uniform(orc_mt *s, double lo, double hi) {
  double range = hi - lo;
  return lo + range * orc_mt_double(s);
}

/* RandomState.randint(high): legacy masked rejection on 32-bit draws
 * (numpy distributions.c random_bounded_uint64_fill, use_masked). */
int64_t orc_randint(orc_mt *s, int64_t high) {
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
  while ((v = (orc_mt_u32(s) & mask)) > rng) {
  }
  return (int64_t)v;
}

uint64_t orc_splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

/* Seeding contract: one MT19937 per (stochastic op, sample, epoch). */
uint32_t orc_sample_seed(uint64_t loader_seed, uint64_t epoch, uint64_t sample,
                         uint32_t op_id) {
  uint64_t h = orc_splitmix64(loader_seed ^ ((uint64_t)op_id << 56));
  h = orc_splitmix64(h ^ epoch);
  h = orc_splitmix64(h ^ sample);
  return (uint32_t)(h & 0xffffffffu);
}

static double py_round(double x) { /* Python round(): half to even */
  return nearbyint(x);           /* default FE_TONEAREST */
}

/* ffcv/fields/rgb_image.py:48-72 get_random_crop */
void orc_random_crop(orc_mt *s, uint32_t height, uint32_t width,
                     const double scale[2], const double ratio[2],
                     int32_t out[4]) {
  uint32_t area = height * width;
  double log_r0 = log(ratio[0]), log_r1 = log(ratio[1]);
  for (int t = 0; t < 10; t++) {
    double target_area = (double)area * orc_uniform(s, scale[0], scale[1]);
    double aspect_ratio = exp(orc_uniform(s, log_r0, log_r1));
    int64_t w = (int64_t)py_round(sqrt(target_area * aspect_ratio));
    int64_t h = (int64_t)py_round(sqrt(target_area / aspect_ratio));
    if (0 < w && w <= (int64_t)width && 0 < h && h <= (int64_t)height) {
      int64_t i = (int64_t)orc_uniform(s, 0.0, (double)((int64_t)height - h + 1));
      int64_t j = (int64_t)orc_uniform(s, 0.0, (double)((int64_t)width - w + 1));
      out[0] = (int32_t)i;
      out[1] = (int32_t)j;
      out[2] = (int32_t)h;
      out[3] = (int32_t)w;
      return;
    }
  }
  double in_ratio = (double)width / (double)height;
  double rmin = ratio[0] < ratio[1] ? ratio[0] : ratio[1];
  double rmax = ratio[0] < ratio[1] ? ratio[1] : ratio[0];
  int64_t w, h;
  if (in_ratio < rmin) {
    w = width;
    h = (int64_t)py_round((double)w / rmin);
  } else if (in_ratio > rmax) {
    h = height;
    w = (int64_t)py_round((double)h * rmax);
  } else {
    w = width;
    h = height;
  }
  out[0] = (int32_t)(((int64_t)height - h) / 2);
  out[1] = (int32_t)(((int64_t)width - w) / 2);
  out[2] = (int32_t)h;
  out[3] = (int32_t)w;
}

/* ffcv/fields/rgb_image.py:75-81 get_center_crop */
void orc_center_crop(uint32_t height, uint32_t width, double ratio,
                     int32_t out[4]) {
  uint32_t s = height < width ? height : width;
  int64_t c = (int64_t)(ratio * (double)s);
  out[0] = (int32_t)(((int64_t)height - c) / 2);
  out[1] = (int32_t)(((int64_t)width - c) / 2);
  out[2] = (int32_t)c;
  out[3] = (int32_t)c;
}

/* ======================================================================= */
/* OpenCV 4.5.4 resize INTER_AREA (imgproc/src/resize.cpp), CV_8UC3        */
/* ======================================================================= */

static inline int cv_round_f(float v) { return (int)nearbyintf(v); }
static inline int cv_floor_d(double v) { return (int)floor(v); }
static inline int cv_ceil_d(double v) { return (int)ceil(v); }
static inline int cv_floor_f(float v) { return (int)floorf(v); }
static inline uint8_t sat_u8(int v) { return (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v); }
static inline int16_t sat_s16(int v) {
  return (int16_t)(v < -32768 ? -32768 : v > 32767 ? 32767 : v);
}
static inline int16_t sat_s16_f(float v) { return sat_s16(cv_round_f(v)); }

typedef struct {
  int di, si;
  float alpha;
} dec_alpha;

/* computeResizeAreaTab */
static int area_tab(int ssize, int dsize, int cn, double scale, dec_alpha *tab) {
  int k = 0;
  for (int dx = 0; dx < dsize; dx++) {
    double fsx1 = dx * scale;
    double fsx2 = fsx1 + scale;
    double cellWidth = scale < (ssize - fsx1) ? scale : (ssize - fsx1);
    int sx1 = cv_ceil_d(fsx1), sx2 = cv_floor_d(fsx2);
    sx2 = sx2 < ssize - 1 ? sx2 : ssize - 1;
    sx1 = sx1 < sx2 ? sx1 : sx2;
    if (sx1 - fsx1 > 1e-3) {
      tab[k].di = dx * cn;
      tab[k].si = (sx1 - 1) * cn;
      tab[k++].alpha = (float)((sx1 - fsx1) / cellWidth);
    }
    for (int sx = sx1; sx < sx2; sx++) {
      tab[k].di = dx * cn;
      tab[k].si = sx * cn;
      tab[k++].alpha = (float)(1.0 / cellWidth);
    }
    if (fsx2 - sx2 > 1e-3) {
      double m = fsx2 - sx2;
      m = m < 1.0 ? m : 1.0;
      m = m < cellWidth ? m : cellWidth;
      tab[k].di = dx * cn;
      tab[k].si = sx2 * cn;
      tab[k++].alpha = (float)(m / cellWidth);
    }
  }
  return k;
}

/* resizeAreaFast_Invoker (integer scale, cn==3 => no SIMD fast mode). */
static void resize_area_fast(const uint8_t *src, size_t sstep, int sw, int sh,
                             uint8_t *dst, size_t dstep, int dw, int dh, int isx,
                             int isy) {
  const int cn = 3;
  int area = isx * isy;
  float scale = 1.f / (float)area;
  int dwidth1 = (sw / isx) * cn;
  int dwidth = dw * cn, swidth = sw * cn;
  for (int dy = 0; dy < dh; dy++) {
    uint8_t *D = dst + dstep * (size_t)dy;
    int sy0 = dy * isy;
    int w = sy0 + isy <= sh ? dwidth1 : 0;
    if (sy0 >= sh) {
      for (int dx = 0; dx < dwidth; dx++) D[dx] = 0;
      continue;
    }
    int dx = 0;
    for (; dx < w; dx++) {
      int sx0 = isx * dx; /* xofs[dx] = isx*j + k with j=dx-k ... equals isx*(dx/cn)*cn + dx%cn */
      sx0 = isx * (dx / cn) * cn + dx % cn;
      const uint8_t *S = src + sstep * (size_t)sy0 + sx0;
      int sum = 0;
      int k = 0;
      /* ofs[k] = sy*sstep + sx*cn, k = sy*isx + sx, summed in that order */
      for (; k <= area - 4; k += 4) {
        int o0 = (k / isx) * (int)sstep + (k % isx) * cn;
        int o1 = ((k + 1) / isx) * (int)sstep + ((k + 1) % isx) * cn;
        int o2 = ((k + 2) / isx) * (int)sstep + ((k + 2) % isx) * cn;
        int o3 = ((k + 3) / isx) * (int)sstep + ((k + 3) % isx) * cn;
        sum += S[o0] + S[o1] + S[o2] + S[o3];
      }
      for (; k < area; k++) sum += S[(k / isx) * (int)sstep + (k % isx) * cn];
      D[dx] = sat_u8(cv_round_f((float)sum * scale));
    }
    for (; dx < dwidth; dx++) {
      int sum = 0, count = 0;
      int sx0 = isx * (dx / cn) * cn + dx % cn;
      if (sx0 >= swidth) D[dx] = 0;
      for (int sy = 0; sy < isy; sy++) {
        if (sy0 + sy >= sh) break;
        const uint8_t *S = src + sstep * (size_t)(sy0 + sy) + sx0;
        for (int sx = 0; sx < isx * cn; sx += cn) {
          if (sx0 + sx >= swidth) break;
          sum += S[sx];
          count++;
        }
      }
      D[dx] = sat_u8(cv_round_f((float)sum / (float)count));
    }
  }
}

/* ResizeArea_Invoker (true area, float accumulation in table order). */
static void resize_area_general(const uint8_t *src, size_t sstep, int sw, int sh,
                                uint8_t *dst, size_t dstep, int dw, int dh,
                                double scale_x, double scale_y) {
  const int cn = 3;
  dec_alpha *xtab = (dec_alpha *)malloc(sizeof(dec_alpha) * (size_t)(sw * 2 + 2));
  dec_alpha *ytab = (dec_alpha *)malloc(sizeof(dec_alpha) * (size_t)(sh * 2 + 2));
  int xtab_size = area_tab(sw, dw, cn, scale_x, xtab);
  int ytab_size = area_tab(sh, dh, 1, scale_y, ytab);
  int dwidth = dw * cn;
  float *buf = (float *)malloc(sizeof(float) * (size_t)dwidth * 2);
  float *sum = buf + dwidth;
  for (int dx = 0; dx < dwidth; dx++) sum[dx] = 0.f;
  int prev_dy = ytab[0].di;
  for (int j = 0; j < ytab_size; j++) {
    float beta = ytab[j].alpha;
    int dy = ytab[j].di;
    int sy = ytab[j].si;
    const uint8_t *S = src + sstep * (size_t)sy;
    for (int dx = 0; dx < dwidth; dx++) buf[dx] = 0.f;
    for (int k = 0; k < xtab_size; k++) {
      int sxn = xtab[k].si, dxn = xtab[k].di;
      float alpha = xtab[k].alpha;
      float t0 = buf[dxn] + (float)S[sxn] * alpha;
      float t1 = buf[dxn + 1] + (float)S[sxn + 1] * alpha;
      float t2 = buf[dxn + 2] + (float)S[sxn + 2] * alpha;
      buf[dxn] = t0;
      buf[dxn + 1] = t1;
      buf[dxn + 2] = t2;
    }
    if (dy != prev_dy) {
      uint8_t *D = dst + dstep * (size_t)prev_dy;
      for (int dx = 0; dx < dwidth; dx++) {
        D[dx] = sat_u8(cv_round_f(sum[dx]));
        sum[dx] = beta * buf[dx];
      }
      prev_dy = dy;
    } else {
      for (int dx = 0; dx < dwidth; dx++) sum[dx] += beta * buf[dx];
    }
  }
  uint8_t *D = dst + dstep * (size_t)prev_dy;
  for (int dx = 0; dx < dwidth; dx++) D[dx] = sat_u8(cv_round_f(sum[dx]));
  free(buf);
  free(xtab);
  free(ytab);
}

/* "area-mode" linear (ksize 2), fixed point Q11; resizeGeneric_ with
 * HResizeLinear<uchar,int,short,2048> and VResizeLinear<...,FixedPtCast<22>>
 * whose SSE2 vector body (VResizeLinearVec_32s8u, 16 lanes) covers the first
 * elements and a scalar tail the rest. */
static void resize_area_linear(const uint8_t *src, size_t sstep, int sw, int sh,
                               uint8_t *dst, size_t dstep, int dw, int dh,
                               double inv_scale_x, double inv_scale_y,
                               double scale_x, double scale_y) {
  const int cn = 3;
  int width = dw * cn;
  int *xofs = (int *)malloc(sizeof(int) * (size_t)width);
  int16_t *ialpha = (int16_t *)malloc(sizeof(int16_t) * (size_t)width * 2);
  int *yofs = (int *)malloc(sizeof(int) * (size_t)dh);
  int16_t *ibeta = (int16_t *)malloc(sizeof(int16_t) * (size_t)dh * 2);
  int xmax = dw;
  for (int dx = 0; dx < dw; dx++) {
    int sx = cv_floor_d(dx * scale_x);
    float fx = (float)((dx + 1) - (sx + 1) * inv_scale_x);
    fx = fx <= 0 ? 0.f : fx - (float)cv_floor_f(fx);
    if (sx + 1 >= sw) {
      xmax = xmax < dx ? xmax : dx;
      if (sx >= sw - 1) {
        fx = 0;
        sx = sw - 1;
      }
    }
    for (int k = 0; k < cn; k++) xofs[dx * cn + k] = sx * cn + k;
    float c0 = 1.f - fx, c1 = fx;
    int16_t a0 = sat_s16_f(c0 * 2048.f), a1 = sat_s16_f(c1 * 2048.f);
    for (int k = 0; k < cn; k++) {
      ialpha[(dx * cn + k) * 2] = a0;
      ialpha[(dx * cn + k) * 2 + 1] = a1;
    }
  }
  for (int dy = 0; dy < dh; dy++) {
    int sy = cv_floor_d(dy * scale_y);
    float fy = (float)((dy + 1) - (sy + 1) * inv_scale_y);
    fy = fy <= 0 ? 0.f : fy - (float)cv_floor_f(fy);
    yofs[dy] = sy;
    ibeta[dy * 2] = sat_s16_f((1.f - fy) * 2048.f);
    ibeta[dy * 2 + 1] = sat_s16_f(fy * 2048.f);
  }
  int xmax_e = xmax * cn;
  int *rows0 = (int *)malloc(sizeof(int) * (size_t)width);
  int *rows1 = (int *)malloc(sizeof(int) * (size_t)width);
  /* number of elements handled by the SSE2 vector path */
  int vec_end = 0;
  {
    int x = 0;
    for (; x <= width - 16; x += 16) {
    }
    for (; x < width - 8; x += 8) {
    }
    vec_end = x;
  }
  for (int dy = 0; dy < dh; dy++) {
    for (int k = 0; k < 2; k++) {
      int sy = yofs[dy] + k;
      sy = sy < 0 ? 0 : (sy >= sh ? sh - 1 : sy);
      const uint8_t *S = src + sstep * (size_t)sy;
      int *D = k ? rows1 : rows0;
      int dx = 0;
      for (; dx < xmax_e; dx++) {
        int sx = xofs[dx];
        D[dx] = S[sx] * ialpha[dx * 2] + S[sx + cn] * ialpha[dx * 2 + 1];
      }
      for (; dx < width; dx++) D[dx] = S[xofs[dx]] * 2048;
    }
    int b0 = ibeta[dy * 2], b1 = ibeta[dy * 2 + 1];
    uint8_t *D = dst + dstep * (size_t)dy;
    for (int x = 0; x < width; x++) {
      if (x < vec_end) {
        /* v_pack(S>>4) saturating to s16, v_mul_hi, saturating add,
         * v_rshr_pack_u<2> */
        int s0 = sat_s16(rows0[x] >> 4), s1 = sat_s16(rows1[x] >> 4);
        int m0 = (s0 * b0) >> 16, m1 = (s1 * b1) >> 16;
        int t = sat_s16(m0 + m1);
        D[x] = sat_u8((t + 2) >> 2);
      } else {
        D[x] = sat_u8((rows0[x] * b0 + rows1[x] * b1 + (1 << 21)) >> 22);
      }
    }
  }
  free(rows0);
  free(rows1);
  free(xofs);
  free(ialpha);
  free(yofs);
  free(ibeta);
}

void orc_resize_area_u8c3(const uint8_t *src, size_t src_step, int sw, int sh,
                          uint8_t *dst, size_t dst_step, int dw, int dh) {
  if (sw == dw && sh == dh) { /* cv::resize: dsize == ssize -> copyTo */
    for (int y = 0; y < sh; y++) memcpy(dst + dst_step * (size_t)y, src + src_step * (size_t)y, (size_t)sw * 3);
    return;
  }
  double inv_scale_x = (double)dw / sw, inv_scale_y = (double)dh / sh;
  double scale_x = 1. / inv_scale_x, scale_y = 1. / inv_scale_y;
  int iscale_x = (int)nearbyint(scale_x), iscale_y = (int)nearbyint(scale_y);
  int is_area_fast = fabs(scale_x - iscale_x) < DBL_EPSILON &&
                     fabs(scale_y - iscale_y) < DBL_EPSILON;
  if (scale_x >= 1 && scale_y >= 1) {
    if (is_area_fast)
      resize_area_fast(src, src_step, sw, sh, dst, dst_step, dw, dh, iscale_x,
                       iscale_y);
    else
      resize_area_general(src, src_step, sw, sh, dst, dst_step, dw, dh, scale_x,
                          scale_y);
    return;
  }
  resize_area_linear(src, src_step, sw, sh, dst, dst_step, dw, dh, inv_scale_x,
                     inv_scale_y, scale_x, scale_y);
}

/* libffcv.cpp:33-42: cv::Mat(sx, sy, CV_8UC3) ROI rows [r0,r1) cols [c0,c1)
 * resized into a (tx, ty) CV_8UC3 destination. */
void orc_resize_crop(const uint8_t *src, int64_t sx, int64_t sy, int64_t r0,
                     int64_t r1, int64_t c0, int64_t c1, uint8_t *dst,
                     int64_t tx, int64_t ty) {
  (void)sx;
  size_t step = (size_t)sy * 3;
  orc_resize_area_u8c3(src + (size_t)r0 * step + (size_t)c0 * 3, step,
                       (int)(c1 - c0), (int)(r1 - r0), dst, (size_t)ty * 3,
                       (int)ty, (int)tx);
}

/* ======================================================================= */
/* JPEG baseline decode restating libjpeg-turbo (jdhuff.c, jidctfst.c,      */
/* jidctint.c, jdsample.c, jdcolor.c, jdmaster.c range limit)               */
/* ======================================================================= */

static const int natural_order[64 + 16] = {
    0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
    12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
    35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
    58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63,
    63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63};

typedef struct {
  int present;
  uint8_t bits[17];
  uint8_t vals[256];
  int32_t mincode[17], maxcode[18], valptr[17];
  int bad; /* jdhuff.c jpeg_make_d_derived_tbl would reject it */
} huff_t;

typedef struct {
  orc_jpeg_info info;
  uint16_t qt[4][64]; /* natural order */
  int qt_present[4];
  huff_t dc[4], ac[4];
  int color_rgb; /* 3-comp stream already RGB (Adobe transform 0 / 'RGB' ids) */
  int comp_id[4];
  int saw_jfif, saw_adobe, adobe_transform;
  int scan_ncomp;
  int scan_comp[4];
} jdec_t;

/* jdhuff.c jpeg_make_d_derived_tbl: canonical codes; a length whose codes
 * reach 2^l (over-subscribed or all-ones code) and, for DC tables, a symbol
 * above 15 are JERR_BAD_HUFF_TABLE (checked for the tables a scan uses). */
static void huff_build(huff_t *h, int is_dc) {
  int code = 0, k = 0;
  h->bad = 0;
  for (int l = 1; l <= 16; l++) {
    if (h->bits[l]) {
      h->valptr[l] = k;
      h->mincode[l] = code;
      code += h->bits[l];
      k += h->bits[l];
      h->maxcode[l] = code - 1;
    } else {
      h->maxcode[l] = -1;
    }
    if (code >= (1 << l)) h->bad = 1;
    code <<= 1;
  }
  h->maxcode[17] = 0x7fffffff;
  if (is_dc)
    for (int i = 0; i < k; i++)
      if (h->vals[i] > 15) h->bad = 1;
}

static int rd16(const uint8_t *p) { return (p[0] << 8) | p[1]; }

static int jpeg_parse(const uint8_t *buf, size_t n, jdec_t *d) {
  memset(d, 0, sizeof(*d));
  orc_jpeg_info *in = &d->info;
  if (n < 4 || buf[0] != 0xFF || buf[1] != 0xD8) return -1;
  size_t p = 2;
  int have_sof = 0;
  while (p + 4 <= n) {
    if (buf[p] != 0xFF) return -2;
    while (p < n && buf[p] == 0xFF) p++;
    if (p >= n) return -2;
    int m = buf[p++];
    if (m == 0xD8 || (m >= 0xD0 && m <= 0xD7) || m == 0x01) continue;
    if (m == 0xD9) return -3; /* EOI before SOS */
    if (p + 2 > n) return -2;
    int len = rd16(buf + p);
    if (len < 2 || p + (size_t)len > n) return -2;
    const uint8_t *s = buf + p + 2;
    int sl = len - 2;
    if (m == 0xDB) { /* DQT */
      int o = 0;
      while (o < sl) {
        int pq = s[o] >> 4, tq = s[o] & 15;
        o++;
        if (tq > 3) return -4;
        for (int i = 0; i < 64; i++) {
          int v = pq ? rd16(s + o + 2 * i) : s[o + i];
          d->qt[tq][natural_order[i]] = (uint16_t)v;
        }
        o += pq ? 128 : 64;
        d->qt_present[tq] = 1;
      }
    } else if (m == 0xC4) { /* DHT */
      int o = 0;
      while (o < sl) {
        int tc = s[o] >> 4, th = s[o] & 15;
        o++;
        if (th > 3 || tc > 1) return -5;
        huff_t *h = tc ? &d->ac[th] : &d->dc[th];
        int total = 0;
        h->bits[0] = 0;
        for (int l = 1; l <= 16; l++) {
          h->bits[l] = s[o + l - 1];
          total += h->bits[l];
        }
        o += 16;
        if (total > 256) return -5;
        memcpy(h->vals, s + o, (size_t)total);
        o += total;
        h->present = 1;
        huff_build(h, tc == 0);
      }
    } else if (m == 0xC0 || m == 0xC1) { /* baseline / extended sequential */
      if (s[0] != 8) return -6;
      in->sof = m;
      in->height = rd16(s + 1);
      in->width = rd16(s + 3);
      in->ncomp = s[5];
      if (in->ncomp != 1 && in->ncomp != 3) return -7;
      in->hmax = in->vmax = 1;
      for (int c = 0; c < in->ncomp; c++) {
        d->comp_id[c] = s[6 + 3 * c];
        in->h[c] = s[7 + 3 * c] >> 4;
        in->v[c] = s[7 + 3 * c] & 15;
        in->tq[c] = s[8 + 3 * c];
        if (in->h[c] < 1 || in->h[c] > 4 || in->v[c] < 1 || in->v[c] > 4) return -8;
        if (in->h[c] > in->hmax) in->hmax = in->h[c];
        if (in->v[c] > in->vmax) in->vmax = in->v[c];
      }
      have_sof = 1;
    } else if (m >= 0xC2 && m <= 0xCF && m != 0xC4 && m != 0xC8 && m != 0xCC) {
      return -9; /* progressive / lossless / arithmetic: not on this path */
    } else if (m == 0xDD) {
      in->restart_interval = rd16(s);
    } else if (m == 0xE0) {
      if (sl >= 5 && !memcmp(s, "JFIF", 5)) d->saw_jfif = 1;
    } else if (m == 0xEE) {
      if (sl >= 12 && !memcmp(s, "Adobe", 5)) {
        d->saw_adobe = 1;
        d->adobe_transform = s[11];
      }
    } else if (m == 0xDA) { /* SOS */
      if (!have_sof) return -10;
      int ns = s[0];
      if (ns != in->ncomp) return -11; /* multi-scan sequential: unsupported */
      d->scan_ncomp = ns;
      for (int i = 0; i < ns; i++) {
        int cid = s[1 + 2 * i], tables = s[2 + 2 * i];
        int c = -1;
        for (int k = 0; k < in->ncomp; k++)
          if (d->comp_id[k] == cid) c = k;
        if (c < 0) return -12;
        d->scan_comp[i] = c;
        in->td[c] = tables >> 4;
        in->ta[c] = tables & 15;
      }
      in->scan_off = p + (size_t)len;
      /* entropy-coded segment ends at the first marker that is not RSTn */
      size_t q = in->scan_off;
      while (q + 1 < n) {
        if (buf[q] == 0xFF && buf[q + 1] != 0x00 &&
            !(buf[q + 1] >= 0xD0 && buf[q + 1] <= 0xD7))
          break;
        q++;
      }
      in->scan_end = q + 1 < n ? q : n;
      /* default_decompress_parms colour-space rule (jdapimin.c) */
      if (in->ncomp == 3) {
        if (d->saw_jfif)
          d->color_rgb = 0;
        else if (d->saw_adobe)
          d->color_rgb = d->adobe_transform == 0;
        else
          d->color_rgb = d->comp_id[0] == 82 && d->comp_id[1] == 71 && d->comp_id[2] == 66;
      }
      for (int c = 0; c < in->ncomp; c++) {
        if (!d->qt_present[in->tq[c]]) return -13;
        if (!d->dc[in->td[c]].present || !d->ac[in->ta[c]].present) return -14;
        if (d->dc[in->td[c]].bad || d->ac[in->ta[c]].bad) return -5;
      }
      return 0;
    }
    p += (size_t)len;
  }
  return -15;
}

int orc_jpeg_header(const uint8_t *buf, size_t n, orc_jpeg_info *info) {
  jdec_t d;
  int rc = jpeg_parse(buf, n, &d);
  if (rc == 0) *info = d.info;
  return rc;
}

/* bit reader over the entropy-coded segment (destuffing; zeros past end) */
typedef struct {
  const uint8_t *p, *end;
  uint64_t acc;
  int nbits;
  int hit_marker;
} bitrd;

static void br_fill(bitrd *b) {
  while (b->nbits <= 56) {
    int byte = 0;
    if (!b->hit_marker && b->p < b->end) {
      byte = *b->p;
      if (byte == 0xFF) {
        int nxt = b->p + 1 < b->end ? b->p[1] : 0xD9;
        if (nxt == 0x00) {
          b->p += 2;
        } else {
          b->hit_marker = 1;
          byte = 0;
        }
      } else {
        b->p++;
      }
    }
    b->acc |= (uint64_t)byte << (56 - b->nbits);
    b->nbits += 8;
  }
}
static int br_get(bitrd *b, int n) {
  if (n == 0) return 0;
  if (b->nbits < n) br_fill(b);
  int v = (int)(b->acc >> (64 - n));
  b->acc <<= n;
  b->nbits -= n;
  return v;
}
static int huff_decode(bitrd *b, const huff_t *h) {
  int code = br_get(b, 1);
  int l = 1;
  while (code > h->maxcode[l]) {
    code = (code << 1) | br_get(b, 1);
    if (++l > 16) return 0; /* corrupt: libjpeg returns 0 */
  }
  return h->vals[(h->valptr[l] + code - h->mincode[l]) & 0xff];
}
static int huff_extend(int x, int s) {
  return x < (1 << (s - 1)) ? x + (int)(((unsigned)-1) << s) + 1 : x;
}

typedef struct {
  int bw[4], bh[4];       /* plane size in blocks (MCU padded) */
  int cw[4], ch[4];       /* downsampled component size in samples */
  int mcux, mcuy;
  int16_t *coef[4];       /* [bh][bw][64] */
} coefimg_t;

static int decode_coefficients(const uint8_t *buf, jdec_t *d, coefimg_t *ci) {
  orc_jpeg_info *in = &d->info;
  memset(ci, 0, sizeof(*ci));
  ci->mcux = (in->width + 8 * in->hmax - 1) / (8 * in->hmax);
  ci->mcuy = (in->height + 8 * in->vmax - 1) / (8 * in->vmax);
  for (int c = 0; c < in->ncomp; c++) {
    ci->cw[c] = (in->width * in->h[c] + in->hmax - 1) / in->hmax;
    ci->ch[c] = (in->height * in->v[c] + in->vmax - 1) / in->vmax;
    ci->bw[c] = ci->mcux * in->h[c];
    ci->bh[c] = ci->mcuy * in->v[c];
    ci->coef[c] = (int16_t *)calloc((size_t)ci->bw[c] * ci->bh[c] * 64, sizeof(int16_t));
  }
  bitrd b = {buf + in->scan_off, buf + in->scan_end, 0, 0, 0};
  int pred[4] = {0, 0, 0, 0};
  int ri = in->restart_interval;
  int mcus_left = ri;
  /* block visiting order */
  int nmcu;
  int single = in->ncomp == 1;
  int sbw = 0, sbh = 0;
  if (single) {
    sbw = (ci->cw[0] + 7) / 8;
    sbh = (ci->ch[0] + 7) / 8;
    nmcu = sbw * sbh;
  } else {
    nmcu = ci->mcux * ci->mcuy;
  }
  for (int m = 0; m < nmcu; m++) {
    if (ri) {
      if (mcus_left == 0) {
        /* process_restart: discard bits to byte boundary, skip RSTn */
        b.acc = 0;
        b.nbits = 0;
        if (b.hit_marker) {
          /* the marker is the RST: skip it */
          const uint8_t *q = b.p;
          while (q < b.end && *q == 0xFF) q++;
          if (q < b.end && *q >= 0xD0 && *q <= 0xD7) {
            b.p = q + 1;
            b.hit_marker = 0;
          }
        } else {
          const uint8_t *q = b.p;
          while (q < b.end && *q == 0xFF) q++;
          if (q < b.end && *q >= 0xD0 && *q <= 0xD7) b.p = q + 1;
        }
        pred[0] = pred[1] = pred[2] = pred[3] = 0;
        mcus_left = ri;
      }
      mcus_left--;
    }
    int nblk = 0;
    int bc[10], bx[10], by[10];
    if (single) {
      bc[0] = 0;
      bx[0] = m % sbw;
      by[0] = m / sbw;
      nblk = 1;
    } else {
      int mx = m % ci->mcux, my = m / ci->mcux;
      for (int si = 0; si < d->scan_ncomp; si++) {
        int c = d->scan_comp[si];
        for (int yy = 0; yy < in->v[c]; yy++)
          for (int xx = 0; xx < in->h[c]; xx++) {
            bc[nblk] = c;
            bx[nblk] = mx * in->h[c] + xx;
            by[nblk] = my * in->v[c] + yy;
            nblk++;
          }
      }
    }
    for (int k = 0; k < nblk; k++) {
      int c = bc[k];
      int16_t *blk = ci->coef[c] + ((size_t)by[k] * ci->bw[c] + bx[k]) * 64;
      const huff_t *hd = &d->dc[in->td[c]], *ha = &d->ac[in->ta[c]];
      int s = huff_decode(&b, hd);
      if (s) {
        int r = br_get(&b, s);
        s = huff_extend(r, s);
      }
      pred[c] += s;
      blk[0] = (int16_t)pred[c];
      for (int z = 1; z < 64; z++) {
        int rs = huff_decode(&b, ha);
        int r = rs >> 4;
        s = rs & 15;
        if (s) {
          z += r;
          int v = br_get(&b, s);
          blk[natural_order[z]] = (int16_t)huff_extend(v, s);
        } else {
          if (r != 15) break;
          z += 15;
        }
      }
    }
  }
  return 0;
}

/* jdmaster.c prepare_range_limit_table; post-IDCT view is +CENTERJSAMPLE */
static uint8_t g_idct_rl[1024];
static uint8_t g_simple_rl[256 * 3]; /* index -256 .. 511 */
static pthread_once_t g_rl_once = PTHREAD_ONCE_INIT;
static void init_rl(void) {
  uint8_t table[5 * 256 + 128];
  uint8_t *t = table + 256;
  memset(table, 0, 256);
  for (int i = 0; i <= 255; i++) t[i] = (uint8_t)i;
  uint8_t *t2 = t + 128;
  for (int i = 128; i < 512; i++) t2[i] = 255;
  memset(t2 + 512, 0, 512 - 128);
  memcpy(t2 + 1024 - 128, t, 128);
  for (int v = 0; v < 1024; v++) g_idct_rl[v] = t2[v];
  for (int i = -256; i < 512; i++) g_simple_rl[i + 256] = i < 0 ? 0 : (i > 255 ? 255 : (uint8_t)i);
}

static const int aanscales[64] = {
    16384, 22725, 21407, 19266, 16384, 12873, 8867,  4520,  22725, 31521, 29692,
    26722, 22725, 17855, 12299, 6270,  21407, 29692, 27969, 25172, 21407, 16819,
    11585, 5906,  19266, 26722, 25172, 22654, 19266, 15137, 10426, 5315,  16384,
    22725, 21407, 19266, 16384, 12873, 8867,  4520,  12873, 17855, 16819, 15137,
    12873, 10114, 6967,  3552,  8867,  12299, 11585, 10426, 8867,  6967,  4799,
    2446,  4520,  6270,  5906,  5315,  4520,  3552,  2446,  1247};

/* jidctfst.c jpeg_idct_ifast (8-bit, CONST_BITS 8, PASS1_BITS 2, truncating
 * DESCALE), dequantising with jddctmgr.c's ifast multiplier table. */
static void idct_ifast(const int16_t *in, const int16_t *qm, uint8_t *out,
                       int stride) {
#define FMUL(v, c) ((int)(((int)(v) * (c)) >> 8))
  int ws[64];
  for (int c = 0; c < 8; c++) {
    const int16_t *ip = in + c;
    const int16_t *q = qm + c;
    int *w = ws + c;
    if (!ip[8] && !ip[16] && !ip[24] && !ip[32] && !ip[40] && !ip[48] && !ip[56]) {
      int dc = ip[0] * q[0];
      for (int r = 0; r < 8; r++) w[8 * r] = dc;
      continue;
    }
    int tmp0 = ip[0] * q[0], tmp1 = ip[16] * q[16], tmp2 = ip[32] * q[32], tmp3 = ip[48] * q[48];
    int tmp10 = tmp0 + tmp2, tmp11 = tmp0 - tmp2;
    int tmp13 = tmp1 + tmp3, tmp12 = FMUL(tmp1 - tmp3, 362) - tmp13;
    tmp0 = tmp10 + tmp13;
    tmp3 = tmp10 - tmp13;
    tmp1 = tmp11 + tmp12;
    tmp2 = tmp11 - tmp12;
    int tmp4 = ip[8] * q[8], tmp5 = ip[24] * q[24], tmp6 = ip[40] * q[40], tmp7 = ip[56] * q[56];
    int z13 = tmp6 + tmp5, z10 = tmp6 - tmp5, z11 = tmp4 + tmp7, z12 = tmp4 - tmp7;
    tmp7 = z11 + z13;
    tmp11 = FMUL(z11 - z13, 362);
    int z5 = FMUL(z10 + z12, 473);
    tmp10 = FMUL(z12, 277) - z5;
    tmp12 = FMUL(z10, -669) + z5;
    tmp6 = tmp12 - tmp7;
    tmp5 = tmp11 - tmp6;
    tmp4 = tmp10 + tmp5;
    w[0] = tmp0 + tmp7;
    w[56] = tmp0 - tmp7;
    w[8] = tmp1 + tmp6;
    w[48] = tmp1 - tmp6;
    w[16] = tmp2 + tmp5;
    w[40] = tmp2 - tmp5;
    w[32] = tmp3 + tmp4;
    w[24] = tmp3 - tmp4;
  }
  for (int r = 0; r < 8; r++) {
    const int *w = ws + 8 * r;
    uint8_t *o = out + (size_t)r * stride;
    if (!w[1] && !w[2] && !w[3] && !w[4] && !w[5] && !w[6] && !w[7]) {
      uint8_t dc = g_idct_rl[(w[0] >> 5) & 1023];
      for (int k = 0; k < 8; k++) o[k] = dc;
      continue;
    }
    int tmp10 = w[0] + w[4], tmp11 = w[0] - w[4];
    int tmp13 = w[2] + w[6], tmp12 = FMUL(w[2] - w[6], 362) - tmp13;
    int tmp0 = tmp10 + tmp13, tmp3 = tmp10 - tmp13, tmp1 = tmp11 + tmp12, tmp2 = tmp11 - tmp12;
    int z13 = w[5] + w[3], z10 = w[5] - w[3], z11 = w[1] + w[7], z12 = w[1] - w[7];
    int tmp7 = z11 + z13;
    tmp11 = FMUL(z11 - z13, 362);
    int z5 = FMUL(z10 + z12, 473);
    tmp10 = FMUL(z12, 277) - z5;
    tmp12 = FMUL(z10, -669) + z5;
    int tmp6 = tmp12 - tmp7, tmp5 = tmp11 - tmp6, tmp4 = tmp10 + tmp5;
    o[0] = g_idct_rl[((tmp0 + tmp7) >> 5) & 1023];
    o[7] = g_idct_rl[((tmp0 - tmp7) >> 5) & 1023];
    o[1] = g_idct_rl[((tmp1 + tmp6) >> 5) & 1023];
    o[6] = g_idct_rl[((tmp1 - tmp6) >> 5) & 1023];
    o[2] = g_idct_rl[((tmp2 + tmp5) >> 5) & 1023];
    o[5] = g_idct_rl[((tmp2 - tmp5) >> 5) & 1023];
    o[4] = g_idct_rl[((tmp3 + tmp4) >> 5) & 1023];
    o[3] = g_idct_rl[((tmp3 - tmp4) >> 5) & 1023];
  }
#undef FMUL
}

/* jidctint.c jpeg_idct_islow (CONST_BITS 13, PASS1_BITS 2, rounding DESCALE) */
static void idct_islow(const int16_t *in, const uint16_t *q, uint8_t *out,
                       int stride) {
#define DS(x, n) ((int)(((x) + ((int64_t)1 << ((n)-1))) >> (n)))
  int ws[64];
  for (int c = 0; c < 8; c++) {
    const int16_t *ip = in + c;
    const uint16_t *qq = q + c;
    int *w = ws + c;
    if (!ip[8] && !ip[16] && !ip[24] && !ip[32] && !ip[40] && !ip[48] && !ip[56]) {
      int dc = (ip[0] * qq[0]) * 4;
      for (int r = 0; r < 8; r++) w[8 * r] = dc;
      continue;
    }
    int64_t z2 = ip[16] * qq[16], z3 = ip[48] * qq[48];
    int64_t z1 = (z2 + z3) * 4433;
    int64_t tmp2 = z1 + z3 * -15137, tmp3 = z1 + z2 * 6270;
    z2 = ip[0] * qq[0];
    z3 = ip[32] * qq[32];
    int64_t tmp0 = (z2 + z3) * 8192, tmp1 = (z2 - z3) * 8192;
    int64_t tmp10 = tmp0 + tmp3, tmp13 = tmp0 - tmp3, tmp11 = tmp1 + tmp2, tmp12 = tmp1 - tmp2;
    tmp0 = ip[56] * qq[56];
    tmp1 = ip[40] * qq[40];
    tmp2 = ip[24] * qq[24];
    tmp3 = ip[8] * qq[8];
    z1 = tmp0 + tmp3;
    z2 = tmp1 + tmp2;
    z3 = tmp0 + tmp2;
    int64_t z4 = tmp1 + tmp3;
    int64_t z5 = (z3 + z4) * 9633;
    tmp0 *= 2446;
    tmp1 *= 16819;
    tmp2 *= 25172;
    tmp3 *= 12299;
    z1 *= -7373;
    z2 *= -20995;
    z3 *= -16069;
    z4 *= -3196;
    z3 += z5;
    z4 += z5;
    tmp0 += z1 + z3;
    tmp1 += z2 + z4;
    tmp2 += z2 + z3;
    tmp3 += z1 + z4;
    w[0] = DS(tmp10 + tmp3, 11);
    w[56] = DS(tmp10 - tmp3, 11);
    w[8] = DS(tmp11 + tmp2, 11);
    w[48] = DS(tmp11 - tmp2, 11);
    w[16] = DS(tmp12 + tmp1, 11);
    w[40] = DS(tmp12 - tmp1, 11);
    w[24] = DS(tmp13 + tmp0, 11);
    w[32] = DS(tmp13 - tmp0, 11);
  }
  for (int r = 0; r < 8; r++) {
    const int *w = ws + 8 * r;
    uint8_t *o = out + (size_t)r * stride;
    if (!w[1] && !w[2] && !w[3] && !w[4] && !w[5] && !w[6] && !w[7]) {
      uint8_t dc = g_idct_rl[DS((int64_t)w[0], 5) & 1023];
      for (int k = 0; k < 8; k++) o[k] = dc;
      continue;
    }
    int64_t z2 = w[2], z3 = w[6];
    int64_t z1 = (z2 + z3) * 4433;
    int64_t tmp2 = z1 + z3 * -15137, tmp3 = z1 + z2 * 6270;
    int64_t tmp0 = ((int64_t)w[0] + w[4]) * 8192, tmp1 = ((int64_t)w[0] - w[4]) * 8192;
    int64_t tmp10 = tmp0 + tmp3, tmp13 = tmp0 - tmp3, tmp11 = tmp1 + tmp2, tmp12 = tmp1 - tmp2;
    tmp0 = w[7];
    tmp1 = w[5];
    tmp2 = w[3];
    tmp3 = w[1];
    z1 = tmp0 + tmp3;
    z2 = tmp1 + tmp2;
    z3 = tmp0 + tmp2;
    int64_t z4 = tmp1 + tmp3;
    int64_t z5 = (z3 + z4) * 9633;
    tmp0 *= 2446;
    tmp1 *= 16819;
    tmp2 *= 25172;
    tmp3 *= 12299;
    z1 *= -7373;
    z2 *= -20995;
    z3 *= -16069;
    z4 *= -3196;
    z3 += z5;
    z4 += z5;
    tmp0 += z1 + z3;
    tmp1 += z2 + z4;
    tmp2 += z2 + z3;
    tmp3 += z1 + z4;
    o[0] = g_idct_rl[DS(tmp10 + tmp3, 18) & 1023];
    o[7] = g_idct_rl[DS(tmp10 - tmp3, 18) & 1023];
    o[1] = g_idct_rl[DS(tmp11 + tmp2, 18) & 1023];
    o[6] = g_idct_rl[DS(tmp11 - tmp2, 18) & 1023];
    o[2] = g_idct_rl[DS(tmp12 + tmp1, 18) & 1023];
    o[5] = g_idct_rl[DS(tmp12 - tmp1, 18) & 1023];
    o[3] = g_idct_rl[DS(tmp13 + tmp0, 18) & 1023];
    o[4] = g_idct_rl[DS(tmp13 - tmp0, 18) & 1023];
  }
#undef DS
}

/* sample fetch with libjpeg context-row semantics (edge rows replicate) */
static inline int px(const uint8_t *p, int stride, int ch, int y, int x) {
  y = y < 0 ? 0 : (y >= ch ? ch - 1 : y);
  return p[(size_t)y * stride + x];
}

/* jdsample.c upsample of one component to full resolution sample (y, x). */
static int upsample_at(const uint8_t *p, int stride, int cw, int ch, int he,
                       int ve, int y, int x) {
  if (he == 1 && ve == 1) return p[(size_t)y * stride + x];
  if (he == 2 && ve == 1) {
    int col = x >> 1;
    if (cw <= 2) return p[(size_t)y * stride + col]; /* h2v1_upsample */
    int cur = p[(size_t)y * stride + col] * 3;
    if (x & 1) {
      int nxt = col + 1 < cw ? p[(size_t)y * stride + col + 1] : -1;
      if (nxt < 0) return p[(size_t)y * stride + col]; /* last column */
      return (cur + nxt + 2) >> 2;
    } else {
      if (col == 0) return p[(size_t)y * stride];
      return (cur + p[(size_t)y * stride + col - 1] + 1) >> 2;
    }
  }
  if (he == 1 && ve == 2) { /* h1v2_fancy_upsample */
    int row = y >> 1;
    int other = (y & 1) ? row + 1 : row - 1;
    int sum = px(p, stride, ch, row, x) * 3 + px(p, stride, ch, other, x);
    return (sum + ((y & 1) ? 2 : 1)) >> 2;
  }
  if (he == 2 && ve == 2) {
    int row = y >> 1, col = x >> 1;
    if (cw <= 2) return p[(size_t)row * stride + col]; /* h2v2_upsample */
    int other = (y & 1) ? row + 1 : row - 1;
#define CS(cc) (px(p, stride, ch, row, (cc)) * 3 + px(p, stride, ch, other, (cc)))
    int thiss = CS(col);
    if (x & 1) {
      int nxt = col + 1 < cw ? CS(col + 1) : thiss;
      return (thiss * 3 + nxt + 7) >> 4;
    } else {
      int last = col > 0 ? CS(col - 1) : thiss;
      return (thiss * 3 + last + 8) >> 4;
    }
#undef CS
  }
  /* int_upsample (generic integral replicate) */
  return p[(size_t)(y / ve) * stride + x / he];
}

static int Cr_r[256], Cb_b[256], Cr_g[256], Cb_g[256];
static pthread_once_t g_cc_once = PTHREAD_ONCE_INIT;
static void init_cc(void) {
  /* jdcolor.c build_ycc_rgb_table, SCALEBITS 16 */
  const int64_t one_half = (int64_t)1 << 15;
  const int64_t f1402 = (int64_t)(1.40200 * 65536 + 0.5), f1772 = (int64_t)(1.77200 * 65536 + 0.5);
  const int64_t f0714 = (int64_t)(0.71414 * 65536 + 0.5), f0344 = (int64_t)(0.34414 * 65536 + 0.5);
  for (int i = 0, x = -128; i <= 255; i++, x++) {
    Cr_r[i] = (int)((f1402 * x + one_half) >> 16);
    Cb_b[i] = (int)((f1772 * x + one_half) >> 16);
    Cr_g[i] = (int)(-f0714 * x);
    Cb_g[i] = (int)(-f0344 * x + one_half);
  }
}

static int decode_rgb(const uint8_t *buf, size_t n, uint8_t *out, int dct) {
  pthread_once(&g_rl_once, init_rl);
  pthread_once(&g_cc_once, init_cc);
  jdec_t *d = (jdec_t *)malloc(sizeof(jdec_t));
  int rc = jpeg_parse(buf, n, d);
  if (rc) {
    free(d);
    return rc;
  }
  orc_jpeg_info *in = &d->info;
  coefimg_t ci;
  decode_coefficients(buf, d, &ci);
  uint8_t *plane[4] = {0};
  int stride[4];
  for (int c = 0; c < in->ncomp; c++) {
    stride[c] = ci.bw[c] * 8;
    plane[c] = (uint8_t *)malloc((size_t)stride[c] * ci.bh[c] * 8);
    int16_t qm[64];
    const uint16_t *q = d->qt[in->tq[c]];
    for (int i = 0; i < 64; i++)
      qm[i] = (int16_t)(((int64_t)q[i] * aanscales[i] + (1 << 11)) >> 12);
    for (int by = 0; by < ci.bh[c]; by++)
      for (int bx = 0; bx < ci.bw[c]; bx++) {
        const int16_t *blk = ci.coef[c] + ((size_t)by * ci.bw[c] + bx) * 64;
        uint8_t *o = plane[c] + (size_t)by * 8 * stride[c] + bx * 8;
        if (dct == 1)
          idct_ifast(blk, qm, o, stride[c]);
        else
          idct_islow(blk, q, o, stride[c]);
      }
  }
  for (int y = 0; y < in->height; y++) {
    for (int x = 0; x < in->width; x++) {
      uint8_t *o = out + ((size_t)y * in->width + x) * 3;
      if (in->ncomp == 1) {
        o[0] = o[1] = o[2] = plane[0][(size_t)y * stride[0] + x];
        continue;
      }
      int s[3];
      for (int c = 0; c < 3; c++)
        s[c] = upsample_at(plane[c], stride[c], ci.cw[c], ci.ch[c],
                           in->hmax / in->h[c], in->vmax / in->v[c], y, x);
      if (d->color_rgb) {
        o[0] = (uint8_t)s[0];
        o[1] = (uint8_t)s[1];
        o[2] = (uint8_t)s[2];
      } else {
        int yy = s[0], cb = s[1], cr = s[2];
        o[0] = g_simple_rl[256 + yy + Cr_r[cr]];
        o[1] = g_simple_rl[256 + yy + ((Cb_g[cb] + Cr_g[cr]) >> 16)];
        o[2] = g_simple_rl[256 + yy + Cb_b[cb]];
      }
    }
  }
  for (int c = 0; c < in->ncomp; c++) {
    free(plane[c]);
    free(ci.coef[c]);
  }
  free(d);
  return 0;
}

int orc_jpeg_decode(const uint8_t *buf, size_t n, uint8_t *out_rgb, int dct) {
  return decode_rgb(buf, n, out_rgb, dct);
}

int orc_jpeg_coefficients(const uint8_t *buf, size_t n, int16_t *coefs,
                          size_t max_blocks, size_t *nblocks) {
  jdec_t *d = (jdec_t *)malloc(sizeof(jdec_t));
  int rc = jpeg_parse(buf, n, d);
  if (rc) {
    free(d);
    return rc;
  }
  orc_jpeg_info *in = &d->info;
  coefimg_t ci;
  decode_coefficients(buf, d, &ci);
  /* emit in MCU block order */
  size_t k = 0;
  if (in->ncomp == 1) {
    int sbw = (ci.cw[0] + 7) / 8, sbh = (ci.ch[0] + 7) / 8;
    for (int by = 0; by < sbh; by++)
      for (int bx = 0; bx < sbw; bx++, k++)
        if (k < max_blocks)
          memcpy(coefs + k * 64, ci.coef[0] + ((size_t)by * ci.bw[0] + bx) * 64, 128);
  } else {
    for (int my = 0; my < ci.mcuy; my++)
      for (int mx = 0; mx < ci.mcux; mx++)
        for (int si = 0; si < d->scan_ncomp; si++) {
          int c = d->scan_comp[si];
          for (int yy = 0; yy < in->v[c]; yy++)
            for (int xx = 0; xx < in->h[c]; xx++, k++)
              if (k < max_blocks)
                memcpy(coefs + k * 64,
                       ci.coef[c] + ((size_t)(my * in->v[c] + yy) * ci.bw[c] +
                                     mx * in->h[c] + xx) * 64,
                       128);
        }
  }
  *nblocks = k;
  for (int c = 0; c < in->ncomp; c++) free(ci.coef[c]);
  free(d);
  return 0;
}

/* ======================================================================= */
/* Cutout, normalize, batch driver                                         */
/* ======================================================================= */

/* cutout.py:44 images[i, y:y+c, x:x+c] = fill */
void orc_cutout(uint8_t *img, int h, int w, int y, int x, int c,
                const uint8_t fill[3]) {
  for (int yy = y; yy < y + c && yy < h; yy++)
    for (int xx = x; xx < x + c && xx < w; xx++) {
      uint8_t *p = img + ((size_t)yy * w + xx) * 3;
      p[0] = fill[0];
      p[1] = fill[1];
      p[2] = fill[2];
    }
}

typedef struct {
  const orc_sample *samples;
  int n;
  const int32_t *crops;
  int out_h, out_w;
  const int32_t *cut;
  int cut_size;
  const uint8_t *fill;
  const uint16_t *lut;
  void *out;
  int next;
  pthread_mutex_t mu;
  int err;
} batch_job;

/* Optional external JPEG decoder for the batch driver (bench.py's CPU
 * baseline): libjpeg-turbo itself through oracle/ljt_harness.c ljt_decode,
 * with the reference's TurboJPEG settings (ifast IDCT + fancy upsampling,
 * libffcv.cpp:104-106).  NULL = this file's restatement. */
typedef int (*orc_ext_decode_fn)(const unsigned char *buf, unsigned long n, unsigned char *out,
                                 int dct_method, int fancy, int *w, int *h, int *ncomp);
static orc_ext_decode_fn g_ext_decode;

void orc_set_jpeg_decoder(void *fn) { g_ext_decode = (orc_ext_decode_fn)fn; }

static void run_sample(batch_job *j, int k, uint8_t *tmp) {
  const orc_sample *s = &j->samples[k];
  const uint8_t *img;
  if (s->mode == 0 && g_ext_decode) {
    int w = 0, h = 0, nc = 0;
    int rc = g_ext_decode(s->data, s->size, tmp, 1, 1, &w, &h, &nc);
    if (rc || (uint32_t)w != s->width || (uint32_t)h != s->height) j->err = rc ? rc : -20;
    img = tmp;
  } else if (s->mode == 0) {
    int rc = orc_jpeg_decode(s->data, s->size, tmp, 1);
    if (rc) j->err = rc;
    img = tmp;
  } else {
    img = s->data;
  }
  const int32_t *c = j->crops + 4 * k;
  size_t px_out = (size_t)j->out_h * j->out_w * 3;
  uint8_t *dst8 = j->lut ? (uint8_t *)malloc(px_out) : (uint8_t *)j->out + px_out * k;
  orc_resize_crop(img, s->height, s->width, c[0], c[0] + c[2], c[1], c[1] + c[3],
                  dst8, j->out_h, j->out_w);
  if (j->cut)
    orc_cutout(dst8, j->out_h, j->out_w, j->cut[2 * k], j->cut[2 * k + 1],
               j->cut_size, j->fill);
  if (j->lut) {
    uint16_t *o = (uint16_t *)j->out + px_out * k;
    for (size_t i = 0; i < px_out; i++) o[i] = j->lut[dst8[i] * 3 + i % 3];
    free(dst8);
  }
}

static void *batch_worker(void *arg) {
  batch_job *j = (batch_job *)arg;
  uint32_t maxhw = 0;
  for (int k = 0; k < j->n; k++) {
    uint32_t hw = j->samples[k].height * j->samples[k].width;
    if (hw > maxhw) maxhw = hw;
  }
  uint8_t *tmp = (uint8_t *)malloc((size_t)maxhw * 3 + 64);
  for (;;) {
    pthread_mutex_lock(&j->mu);
    int k = j->next++;
    pthread_mutex_unlock(&j->mu);
    if (k >= j->n) break;
    run_sample(j, k, tmp);
  }
  free(tmp);
  return NULL;
}

/* rgb_image.py:185-210 (+ cutout.py:36-47, normalize.py:89-109) over a batch,
 * one sample per worker at a time like numba prange. */
int orc_rrc_batch(const orc_sample *samples, int n, const int32_t *crops,
                  int out_h, int out_w, const int32_t *cutout_yx,
                  int cutout_size, const uint8_t fill[3], const uint16_t *lut,
                  void *out, int nthreads) {
  batch_job j;
  j.samples = samples;
  j.n = n;
  j.crops = crops;
  j.out_h = out_h;
  j.out_w = out_w;
  j.cut = cutout_yx;
  j.cut_size = cutout_size;
  j.fill = fill;
  j.lut = lut;
  j.out = out;
  j.next = 0;
  j.err = 0;
  pthread_mutex_init(&j.mu, NULL);
  if (nthreads < 1) nthreads = 1;
  pthread_t th[256];
  if (nthreads > 256) nthreads = 256;
  for (int t = 1; t < nthreads; t++) pthread_create(&th[t], NULL, batch_worker, &j);
  batch_worker(&j);
  for (int t = 1; t < nthreads; t++) pthread_join(th[t], NULL);
  pthread_mutex_destroy(&j.mu);
  return j.err;
}

void orc_draw_batch(const uint64_t *ids, const uint32_t *heights,
                    const uint32_t *widths, int n, uint64_t loader_seed,
                    uint64_t epoch, int crop_kind, const double scale[2],
                    const double ratio[2], double center_ratio, int out_h,
                    int out_w, int cutout_size, int32_t *crops,
                    int32_t *cutout_yx) {
  orc_mt *mt = (orc_mt *)malloc(sizeof(orc_mt));
  for (int k = 0; k < n; k++) {
    if (crops) {
      if (crop_kind == 0) {
        orc_mt_seed(mt, orc_sample_seed(loader_seed, epoch, ids[k], 1));
        orc_random_crop(mt, heights[k], widths[k], scale, ratio, crops + 4 * k);
      } else {
        orc_center_crop(heights[k], widths[k], center_ratio, crops + 4 * k);
      }
    }
    if (cutout_yx) {
      orc_mt_seed(mt, orc_sample_seed(loader_seed, epoch, ids[k], 2));
      cutout_yx[2 * k] = (int32_t)orc_randint(mt, out_h - cutout_size + 1);
      cutout_yx[2 * k + 1] = (int32_t)orc_randint(mt, out_w - cutout_size + 1);
    }
  }
  free(mt);
}
