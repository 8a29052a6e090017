// ffcv_cpu_jpeg.hip -- host (CPU) JPEG decoder behind the reference's
// imdecode signature (libffcv.cpp:53-112, bound at ffcv/libffcv.py:34-48).
//
// The reference's CPU Loader decodes every JPEG sample on the host:
// SimpleRGBImageDecoder / ResizedCropRGBImageDecoder call imdecode from numba
// prange workers (rgb_image.py:131,196), which runs TurboJPEG's
// tjDecompress2(TJPF_RGB, TJFLAG_FASTDCT): libjpeg-turbo's ifast IDCT
// (jidctfst.c), fancy upsampling (jdsample.c) and the fixed-point YCbCr->RGB
// tables (jdcolor.c).  This is that decode in plain C++ on the calling thread,
// with the same arithmetic the gfx950 kernels use (ffcv_jpeg.hip), so a
// Loader on device='cpu' -- or on a machine without a GPU -- produces the
// reference's pixels.  The device decoder stays the hot path; this file is
// the CPU boundary only.
//
// Supported: baseline / extended sequential Huffman, 8-bit, 1 or 3
// components in one scan, any sampling factors 1..4, restart intervals.
// Progressive, arithmetic, lossless, 12-bit, multi-scan and CMYK streams
// return -1 (the device path reports FFCV_SAMPLE_UNSUPPORTED for them).
// The tjTransform crop / mirror (enable_crop, hflip) is restated on the
// coefficients (transform_coefs); TurboJPEG's scaled decoding at 1/2, 1/4
// and 1/8 too (decode_scaled, jidctred.c): a request TurboJPEG would decode
// at another factor returns -1.  ffcv itself passes the image's own size and
// False, False, 1, 1.
#include <atomic>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "api_internal.h"

namespace {

// zigzag index -> natural index (jutils.c jpeg_natural_order, padded so a
// corrupt run past 63 lands on 63 like libjpeg's)
const uint8_t kNatural[64 + 16] = {
    0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13,
    6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51, 58, 59, 52, 45, 38, 31,
    39, 46, 53, 60, 61, 54, 47, 55, 62, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63};

// jddctmgr.c: the ifast method's multiplier table (aanscales, CONST_BITS 14)
const int16_t kAanScales[64] = {16384, 22725, 21407, 19266, 16384, 12873, 8867,  4520,  22725, 31521, 29692,
                                26722, 22725, 17855, 12299, 6270,  21407, 29692, 27969, 25172, 21407, 16819,
                                11585, 5906,  19266, 26722, 25172, 22654, 19266, 15137, 10426, 5315,  16384,
                                22725, 21407, 19266, 16384, 12873, 8867,  4520,  12873, 17855, 16819, 15137,
                                12873, 10114, 6967,  3552,  8867,  12299, 11585, 10426, 8867,  6967,  4799,
                                2446,  4520,  6270,  5906,  5315,  4520,  3552,  2446,  1247};

constexpr int kLook = 9;  // first-level lookahead bits

struct Huff {
  bool present = false, bad = false;
  uint8_t bits[17];
  uint8_t vals[256];
  int32_t maxcode[18];  // largest code of each length (left-aligned compare below), -1 if none
  int32_t valoff[17];   // vals index of a length's first code, minus that code
  uint16_t look[1 << kLook];  // code length << 8 | symbol, 0 = longer than kLook bits
};

// jdhuff.c jpeg_make_d_derived_tbl: canonical codes, rejecting over-
// subscribed lengths (and the all-ones code) and DC symbols above 15.
void build_huff(Huff &h, bool dc) {
  int code = 0, k = 0;
  h.bad = false;
  std::memset(h.look, 0, sizeof(h.look));
  for (int l = 1; l <= 16; l++) {
    h.valoff[l] = k - code;
    // jpeg_make_d_derived_tbl rejects an over-subscribed length before any
    // lookup entry is built: a code past 2^l - 1 would index past look[]
    if (code + (int)h.bits[l] >= (1 << l)) {
      h.bad = true;
      break;
    }
    for (int i = 0; i < h.bits[l]; i++, k++, code++)
      if (l <= kLook) {
        const int lo = code << (kLook - l), n = 1 << (kLook - l);
        for (int j = 0; j < n; j++) h.look[lo + j] = (uint16_t)(l << 8 | h.vals[k]);
      }
    h.maxcode[l] = h.bits[l] ? code - 1 : -1;
    code <<= 1;
  }
  h.maxcode[17] = 0x7fffffff;
  if (dc)
    for (int i = 0; i < k; i++)
      if (h.vals[i] > 15) h.bad = true;
}

struct Comp {
  int id, h, v, tq, td, ta;
  int cw, ch;  // downsampled size in samples
  int bw, bh;  // plane size in blocks (whole MCUs)
};

struct Dec {
  int W = 0, H = 0, nc = 0, hmax = 1, vmax = 1, ri = 0;
  Comp c[3];
  int scan[3];
  uint16_t qt[4][64];  // natural order
  bool qtp[4] = {false, false, false, false};
  Huff dc[4], ac[4];
  bool jfif = false, adobe = false, color_rgb = false;
  int adobe_t = 0;
  size_t ecs = 0, ecs_end = 0;  // entropy-coded segment [ecs, ecs_end)
};

int rd16(const uint8_t *p) { return p[0] << 8 | p[1]; }

// Marker walk up to the first SOS (jdmarker.c), with the acceptance rules of
// the device parser (ffcv_jpeg.hip parse_header).  0 or a message.
const char *parse(const uint8_t *b, size_t n, Dec &d) {
  if (n < 4 || b[0] != 0xFF || b[1] != 0xD8) return "not a JPEG (no SOI)";
  size_t p = 2;
  bool sof = false;
  while (p + 4 <= n) {
    if (b[p] != 0xFF) return "corrupt marker stream";
    while (p < n && b[p] == 0xFF) p++;
    if (p >= n) return "truncated marker";
    const int m = b[p++];
    if (m == 0xD8 || (m >= 0xD0 && m <= 0xD7) || m == 0x01) continue;
    if (m == 0xD9) return "EOI before SOS";
    if (p + 2 > n) return "truncated segment";
    const int len = rd16(b + p);
    if (len < 2 || p + (size_t)len > n) return "truncated segment";
    const uint8_t *s = b + p + 2;
    const int sl = len - 2;
    if (m == 0xDB) {  // DQT
      for (int o = 0; o < sl;) {
        const int pq = s[o] >> 4, tq = s[o] & 15;
        o++;
        if (tq > 3 || o + (pq ? 128 : 64) > sl) return "bad DQT";
        for (int i = 0; i < 64; i++) d.qt[tq][kNatural[i]] = (uint16_t)(pq ? rd16(s + o + 2 * i) : s[o + i]);
        o += pq ? 128 : 64;
        d.qtp[tq] = true;
      }
    } else if (m == 0xC4) {  // DHT
      for (int o = 0; o < sl;) {
        const int tc = s[o] >> 4, th = s[o] & 15;
        o++;
        if (tc > 1 || th > 3 || o + 16 > sl) return "bad DHT";
        Huff &h = tc ? d.ac[th] : d.dc[th];
        int total = 0;
        h.bits[0] = 0;
        for (int l = 1; l <= 16; l++) total += (h.bits[l] = s[o + l - 1]);
        o += 16;
        if (total > 256 || o + total > sl) return "bad DHT";
        std::memcpy(h.vals, s + o, (size_t)total);
        o += total;
        h.present = true;
        build_huff(h, tc == 0);
      }
    } else if (m == 0xC0 || m == 0xC1) {  // baseline / extended sequential Huffman
      if (sl < 6 || s[0] != 8) return "unsupported precision";
      d.H = rd16(s + 1);
      d.W = rd16(s + 3);
      d.nc = s[5];
      if (d.nc != 1 && d.nc != 3) return "unsupported component count";
      if (sl < 6 + 3 * d.nc || d.W == 0 || d.H == 0) return "bad SOF";
      for (int i = 0; i < d.nc; i++) {
        Comp &c = d.c[i];
        c.id = s[6 + 3 * i];
        c.h = s[7 + 3 * i] >> 4;
        c.v = s[7 + 3 * i] & 15;
        c.tq = s[8 + 3 * i];
        if (c.h < 1 || c.h > 4 || c.v < 1 || c.v > 4 || c.tq > 3) return "bad sampling factors";
        d.hmax = std::max(d.hmax, c.h);
        d.vmax = std::max(d.vmax, c.v);
      }
      // non-integral ratios (e.g. luma h=3, chroma h=2): libjpeg's
      // JERR_FRACT_SAMPLE_NOTIMPL, and the device parser's rejection
      for (int i = 0; i < d.nc; i++)
        if (d.hmax % d.c[i].h || d.vmax % d.c[i].v) return "unsupported sampling factors";
      sof = true;
    } else if (m >= 0xC2 && m <= 0xCF && m != 0xC4 && m != 0xC8 && m != 0xCC) {
      return "progressive / lossless / arithmetic coding is not supported";
    } else if (m == 0xDD) {
      if (sl < 2) return "bad DRI";
      d.ri = rd16(s);
    } else if (m == 0xE0) {
      if (sl >= 5 && !std::memcmp(s, "JFIF", 5)) d.jfif = true;
    } else if (m == 0xEE) {
      if (sl >= 12 && !std::memcmp(s, "Adobe", 5)) {
        d.adobe = true;
        d.adobe_t = s[11];
      }
    } else if (m == 0xDA) {  // SOS
      if (!sof) return "SOS before SOF";
      if (sl < 1 || s[0] != d.nc || sl < 1 + 2 * d.nc) return "multi-scan streams are not supported";
      for (int i = 0; i < d.nc; i++) {
        const int cid = s[1 + 2 * i], t = s[2 + 2 * i];
        int c = -1;
        for (int k = 0; k < d.nc; k++)
          if (d.c[k].id == cid) c = k;
        if (c < 0) return "bad SOS component";
        d.scan[i] = c;
        d.c[c].td = t >> 4;
        d.c[c].ta = t & 15;
        if (d.c[c].td > 3 || d.c[c].ta > 3) return "bad SOS tables";
      }
      d.ecs = p + (size_t)len;
      size_t q = d.ecs;  // the segment ends at the first marker that is not RSTn
      while (q + 1 < n && !(b[q] == 0xFF && b[q + 1] != 0x00 && !(b[q + 1] >= 0xD0 && b[q + 1] <= 0xD7))) q++;
      d.ecs_end = q + 1 < n ? q : n;
      if (d.nc == 3) {  // jdapimin.c default_decompress_parms
        if (d.jfif)
          d.color_rgb = false;
        else if (d.adobe)
          d.color_rgb = d.adobe_t == 0;
        else
          d.color_rgb = d.c[0].id == 'R' && d.c[1].id == 'G' && d.c[2].id == 'B';
        if (d.adobe && d.adobe_t == 2) return "YCCK is not supported";
      }
      for (int i = 0; i < d.nc; i++) {
        const Comp &c = d.c[i];
        if (!d.qtp[c.tq]) return "missing quantisation table";
        if (!d.dc[c.td].present || !d.ac[c.ta].present) return "missing Huffman table";
        if (d.dc[c.td].bad || d.ac[c.ta].bad) return "bad Huffman table";
      }
      return nullptr;
    }
    p += (size_t)len;
  }
  return "no SOS";
}

// Entropy-coded segment reader: 0xFF00 de-stuffing; at a marker it feeds
// zeros (jdhuff.c jpeg_fill_bit_buffer after a marker).
struct Bits {
  const uint8_t *p, *end;
  uint64_t acc = 0;  // valid bits left-aligned
  int n = 0;
  bool marker = false;
  void fill() {
    // fast path: 8 bytes with no 0xFF among them enter whole
    if (!marker && end - p >= 8) {
      uint64_t v;
      std::memcpy(&v, p, 8);
      const uint64_t x = ~v;  // a 0xFF byte of v is a zero byte of x
      if (!((x - 0x0101010101010101ull) & ~x & 0x8080808080808080ull)) {
        v = __builtin_bswap64(v);
        const int k = (64 - n) >> 3;  // whole bytes that fit
        acc |= (k == 8 ? v : v >> (64 - 8 * k)) << (64 - n - 8 * k);
        n += 8 * k;
        p += k;
        return;
      }
    }
    while (n <= 56) {
      int v = 0;
      if (!marker && p < end) {
        v = *p;
        if (v == 0xFF) {
          const int nx = p + 1 < end ? p[1] : 0xD9;
          if (nx == 0x00) {
            p += 2;
          } else {
            marker = true;
            v = 0;
          }
        } else {
          p++;
        }
      }
      acc |= (uint64_t)v << (56 - n);
      n += 8;
    }
  }
  uint32_t peek16() {
    if (n < 16) fill();
    return (uint32_t)(acc >> 48);
  }
  void skip(int k) {
    acc <<= k;
    n -= k;
  }
  int get(int k) {  // k in 1..16
    if (n < k) fill();
    const int v = (int)(acc >> (64 - k));
    skip(k);
    return v;
  }
  // process_restart: drop the buffered bits, then jdmarker.c next_marker:
  // discard bytes up to the next marker (stuffed FF00 pairs included) and
  // step over it when it is the RSTn
  void restart() {
    acc = 0;
    n = 0;
    const uint8_t *q = p;
    for (;;) {
      while (q < end && *q != 0xFF) q++;
      while (q < end && *q == 0xFF) q++;
      if (q >= end) break;
      if (*q != 0) {
        if (*q >= 0xD0 && *q <= 0xD7) q++;
        break;
      }
      q++;
    }
    p = q;
    marker = false;
  }
};

int decode_sym(Bits &br, const Huff &h) {
  const uint32_t look = br.peek16();
  const uint16_t e = h.look[look >> (16 - kLook)];
  if (e) {
    br.skip(e >> 8);
    return e & 0xff;
  }
  int l = kLook + 1;
  while (l <= 16 && (int32_t)(look >> (16 - l)) > h.maxcode[l]) l++;
  if (l > 16) {  // no such code: libjpeg warns and yields symbol 0 after 16 bits
    br.skip(16);
    return 0;
  }
  br.skip(l);
  return h.vals[(h.valoff[l] + (int)(look >> (16 - l))) & 0xff];
}

inline int extend(int v, int s) { return v < (1 << (s - 1)) ? v - (1 << s) + 1 : v; }  // HUFF_EXTEND

// jdmaster.c prepare_range_limit_table as the IDCT sees it (the +128 centre
// folded in): rl[x & 1023] of a DESCALEd IDCT output x
struct Tables {
  uint8_t rl[1024];
  int cr_r[256], cb_b[256], cr_g[256], cb_g[256];  // jdcolor.c build_ycc_rgb_table
  Tables() {
    for (int v = 0; v < 1024; v++) {
      const int x = v < 512 ? v : v - 1024;  // signed 10-bit
      const int y = x + 128;
      rl[v] = (uint8_t)(y < 0 ? 0 : (y > 255 ? 255 : y));
    }
    const int64_t half = (int64_t)1 << 15;
    const int64_t f1402 = (int64_t)(1.40200 * 65536 + 0.5), f1772 = (int64_t)(1.77200 * 65536 + 0.5);
    const int64_t f0714 = (int64_t)(0.71414 * 65536 + 0.5), f0344 = (int64_t)(0.34414 * 65536 + 0.5);
    for (int i = 0; i < 256; i++) {
      const int64_t x = i - 128;
      cr_r[i] = (int)((f1402 * x + half) >> 16);
      cb_b[i] = (int)((f1772 * x + half) >> 16);
      cr_g[i] = (int)(-f0714 * x);
      cb_g[i] = (int)(-f0344 * x + half);
    }
  }
};
const Tables &tables() {
  static const Tables t;
  return t;
}

// jidctfst.c jpeg_idct_ifast: dequantise by the ifast multipliers, columns
// then rows, CONST_BITS 8 products, PASS1_BITS 2 (the row pass DESCALEs by
// 5 with truncation into the range-limit table).  Zero columns / rows take
// libjpeg's DC shortcut, which gives the same values.
void idct_ifast(const int16_t *in, const int16_t *qm, uint8_t *out, int stride, const uint8_t *rl) {
  auto M = [](int v, int c) { return (int)(((int64_t)v * c) >> 8); };
  int ws[64];
  for (int c = 0; c < 8; c++) {
    const int16_t *ip = in + c;
    const int16_t *q = qm + c;
    int *w = ws + c;
    if (!(ip[8] | ip[16] | ip[24] | ip[32] | ip[40] | ip[48] | ip[56])) {
      const int dc = ip[0] * q[0];
      for (int r = 0; r < 8; r++) w[8 * r] = dc;
      continue;
    }
    int t0 = ip[0] * q[0], t1 = ip[16] * q[16], t2 = ip[32] * q[32], t3 = ip[48] * q[48];
    int t10 = t0 + t2, t11 = t0 - t2, t13 = t1 + t3, t12 = M(t1 - t3, 362) - t13;
    t0 = t10 + t13;
    t3 = t10 - t13;
    t1 = t11 + t12;
    t2 = t11 - t12;
    int t4 = ip[8] * q[8], t5 = ip[24] * q[24], t6 = ip[40] * q[40], t7 = ip[56] * q[56];
    const int z13 = t6 + t5, z10 = t6 - t5, z11 = t4 + t7, z12 = t4 - t7;
    t7 = z11 + z13;
    t11 = M(z11 - z13, 362);
    const int z5 = M(z10 + z12, 473);
    t10 = M(z12, 277) - z5;
    t12 = M(z10, -669) + z5;
    t6 = t12 - t7;
    t5 = t11 - t6;
    t4 = t10 + t5;
    w[0] = t0 + t7;
    w[56] = t0 - t7;
    w[8] = t1 + t6;
    w[48] = t1 - t6;
    w[16] = t2 + t5;
    w[40] = t2 - t5;
    w[32] = t3 + t4;
    w[24] = t3 - t4;
  }
  for (int r = 0; r < 8; r++) {
    const int *w = ws + 8 * r;
    uint8_t *o = out + (size_t)r * stride;
    if (!(w[1] | w[2] | w[3] | w[4] | w[5] | w[6] | w[7])) {
      std::memset(o, rl[(w[0] >> 5) & 1023], 8);
      continue;
    }
    const int t10 = w[0] + w[4], t11 = w[0] - w[4], t13 = w[2] + w[6], t12 = M(w[2] - w[6], 362) - t13;
    const int t0 = t10 + t13, t3 = t10 - t13, t1 = t11 + t12, t2 = t11 - t12;
    const int z13 = w[5] + w[3], z10 = w[5] - w[3], z11 = w[1] + w[7], z12 = w[1] - w[7];
    const int t7 = z11 + z13, u11 = M(z11 - z13, 362), z5 = M(z10 + z12, 473);
    const int u10 = M(z12, 277) - z5, u12 = M(z10, -669) + z5;
    const int t6 = u12 - t7, t5 = u11 - t6, t4 = u10 + t5;
    o[0] = rl[((t0 + t7) >> 5) & 1023];
    o[7] = rl[((t0 - t7) >> 5) & 1023];
    o[1] = rl[((t1 + t6) >> 5) & 1023];
    o[6] = rl[((t1 - t6) >> 5) & 1023];
    o[2] = rl[((t2 + t5) >> 5) & 1023];
    o[5] = rl[((t2 - t5) >> 5) & 1023];
    o[4] = rl[((t3 + t4) >> 5) & 1023];
    o[3] = rl[((t3 - t4) >> 5) & 1023];
  }
}

// Per-thread scratch (the reference keeps per-thread TurboJPEG handles).
struct Scratch {
  std::vector<uint8_t> plane[3];
  std::vector<int> row[3];  // fancy-upsampling work rows
};
thread_local Scratch t_scr;

// Plane geometry of a decode: downsampled sizes, whole-MCU block grids, and
// the ifast multipliers (jddctmgr.c) of each component.
void plane_setup(Dec &d, Scratch &S, int stride[3], int16_t qm[3][64]) {
  const int mcux = (d.W + 8 * d.hmax - 1) / (8 * d.hmax), mcuy = (d.H + 8 * d.vmax - 1) / (8 * d.vmax);
  for (int i = 0; i < d.nc; i++) {
    Comp &c = d.c[i];
    c.cw = (d.W * c.h + d.hmax - 1) / d.hmax;
    c.ch = (d.H * c.v + d.vmax - 1) / d.vmax;
    c.bw = mcux * c.h;
    c.bh = mcuy * c.v;
    stride[i] = c.bw * 8;
    S.plane[i].resize((size_t)stride[i] * c.bh * 8);
    for (int k = 0; k < 64; k++) qm[i][k] = (int16_t)(((int64_t)d.qt[c.tq][k] * kAanScales[k] + (1 << 11)) >> 12);
  }
}

// Huffman decode of the whole scan: emit(component, block x, block y,
// coefficients in natural order with the absolute DC) for every coded block.
// nsym (optional): incremented by the Huffman symbols (DC and AC) decoded.
template <class Emit>
void decode_scan(const uint8_t *b, const Dec &d, Emit &&emit, uint64_t *nsym = nullptr) {
  const int mcux = (d.W + 8 * d.hmax - 1) / (8 * d.hmax), mcuy = (d.H + 8 * d.vmax - 1) / (8 * d.vmax);
  Bits br{b + d.ecs, b + d.ecs_end};
  int pred[3] = {0, 0, 0};
  int left = d.ri;
  // a single-component scan is non-interleaved: its MCU is one block, over the
  // component's own block grid (jdinput.c per_scan_setup)
  const bool single = d.nc == 1;
  const int cw0 = (d.W * d.c[0].h + d.hmax - 1) / d.hmax, ch0 = (d.H * d.c[0].v + d.vmax - 1) / d.vmax;
  const int sbw = single ? (cw0 + 7) / 8 : 0, sbh = single ? (ch0 + 7) / 8 : 0;
  const int nmcu = single ? sbw * sbh : mcux * mcuy;
  alignas(16) int16_t blk[64];
  for (int m = 0; m < nmcu; m++) {
    if (d.ri) {
      if (left == 0) {
        br.restart();
        pred[0] = pred[1] = pred[2] = 0;
        left = d.ri;
      }
      left--;
    }
    for (int si = 0; si < d.nc; si++) {
      const int ci = d.scan[si];
      const Comp &c = d.c[ci];
      const Huff &hd = d.dc[c.td], &ha = d.ac[c.ta];
      const int nh = single ? 1 : c.h, nv = single ? 1 : c.v;
      for (int yy = 0; yy < nv; yy++)
        for (int xx = 0; xx < nh; xx++) {
          const int bx = single ? m % sbw : (m % mcux) * c.h + xx, by = single ? m / sbw : (m / mcux) * c.v + yy;
          std::memset(blk, 0, sizeof(blk));
          int s = decode_sym(br, hd);
          if (s) s = extend(br.get(s), s);
          pred[ci] += s;
          blk[0] = (int16_t)pred[ci];
          uint64_t ns = 1;
          for (int z = 1; z < 64; z++, ns++) {
            const int rs = decode_sym(br, ha), r = rs >> 4;
            s = rs & 15;
            if (s) {
              z += r;
              blk[kNatural[z]] = (int16_t)extend(br.get(s), s);
            } else {
              if (r != 15) {
                ns++;  // (the EOB that ends the loop)
                break;
              }
              z += 15;
            }
          }
          if (nsym) *nsym += ns;
          emit(ci, bx, by, blk);
        }
    }
  }
}

// Huffman decode + IDCT of the whole scan into the component planes.
void decode_planes(const uint8_t *b, Dec &d, Scratch &S, int stride[3]) {
  const Tables &T = tables();
  int16_t qm[3][64];
  plane_setup(d, S, stride, qm);
  decode_scan(b, d, [&](int ci, int bx, int by, const int16_t *blk) {
    idct_ifast(blk, qm[ci], S.plane[ci].data() + (size_t)by * 8 * stride[ci] + bx * 8, stride[ci], T.rl);
  });
}

// TurboJPEG's scaling factors (tjGetScalingFactors, largest first) and
// tjDecompress2's choice among them: the first whose scaled size fits the
// requested width x height.
int tj_scale_choice(int w, int h, uint32_t req_w, uint32_t req_h, int *num, int *den) {
  static const int sf[16][2] = {{2, 1}, {15, 8}, {7, 4}, {13, 8}, {3, 2}, {11, 8}, {5, 4}, {9, 8},
                                {1, 1}, {7, 8},  {3, 4}, {5, 8},  {1, 2}, {3, 8},  {1, 4}, {1, 8}};
  for (int i = 0; i < 16; i++) {
    const int64_t sw = ((int64_t)w * sf[i][0] + sf[i][1] - 1) / sf[i][1];
    const int64_t sh = ((int64_t)h * sf[i][0] + sf[i][1] - 1) / sf[i][1];
    if (sw <= (int64_t)req_w && sh <= (int64_t)req_h) {
      *num = sf[i][0];
      *den = sf[i][1];
      return 0;
    }
  }
  return -1;
}

// tjTransform(TJXOPT_CROP [+ TJXOP_HFLIP]) (libffcv.cpp:78-98), restated on
// the decoded coefficients as libjpeg-turbo's transupp.c does it: the crop
// origin must sit on an iMCU boundary (tjTransform's check); its size is
// clamped to the image (0 = to the edge; jtransform_request_workspace); the
// crop is taken in the transformed frame.  do_crop copies blocks; do_flip_h
// mirrors the whole iMCU columns (block order reversed, odd DCT columns
// negated) and copies the partial iMCU column at the right edge unchanged.
// The output image is d's stream with the new size and coefficients, decoded
// like any other (same tables, colour space and sampling).
const char *transform_coefs(const uint8_t *b, Dec &d, uint32_t x, uint32_t y, uint32_t w, uint32_t h, bool hflip,
                            std::vector<int16_t> dst[3]) {
  const int imw = 8 * d.hmax, imh = 8 * d.vmax;
  if (x % (uint32_t)imw || y % (uint32_t)imh) return "crop origin is not on an iMCU boundary";
  if (x >= (uint32_t)d.W || y >= (uint32_t)d.H) return "crop origin outside the image";
  // jtransform_request_workspace: a set crop size must fit from its origin
  // (JERR_BAD_CROP_SPEC); crop extension (w > W) is refused here whether or
  // not a transform is requested (libjpeg-turbo allows it only without one,
  // padding the image: not restated)
  if (w != 0 && (w > (uint32_t)d.W || x > (uint32_t)d.W - w)) return "bad crop spec (width)";
  if (h != 0 && (h > (uint32_t)d.H || y > (uint32_t)d.H - h)) return "bad crop spec (height)";
  const int rw = (int)(w == 0 ? (uint32_t)d.W - x : w);
  const int rh = (int)(h == 0 ? (uint32_t)d.H - y : h);
  // source coefficients, whole-MCU grids (blocks a non-interleaved scan does not code stay zero)
  const int mcux = (d.W + imw - 1) / imw, mcuy = (d.H + imh - 1) / imh;
  std::vector<int16_t> src[3];
  int sbw[3];
  for (int i = 0; i < d.nc; i++) {
    sbw[i] = mcux * d.c[i].h;
    src[i].assign((size_t)sbw[i] * mcuy * d.c[i].v * 64, 0);
  }
  decode_scan(b, d, [&](int ci, int bx, int by, const int16_t *blk) {
    std::memcpy(src[ci].data() + ((size_t)by * sbw[ci] + bx) * 64, blk, 64 * sizeof(int16_t));
  });
  const int W0 = d.W;
  d.W = rw;
  d.H = rh;
  const int dmcux = (rw + imw - 1) / imw, dmcuy = (rh + imh - 1) / imh;
  for (int i = 0; i < d.nc; i++) {
    const Comp &c = d.c[i];
    const int dbw = dmcux * c.h, dbh = dmcuy * c.v;
    const int wib = (rw * c.h + imw - 1) / imw, hib = (rh * c.v + imh - 1) / imh;  // width/height_in_blocks
    const int xcb = (int)(x / (uint32_t)imw) * c.h, ycb = (int)(y / (uint32_t)imh) * c.v;
    const int comp_width = (W0 / imw) * c.h;  // whole iMCU columns (do_flip_h)
    dst[i].assign((size_t)dbw * dbh * 64, 0);
    for (int by = 0; by < hib; by++)
      for (int bx = 0; bx < wib; bx++) {
        int16_t *o = dst[i].data() + ((size_t)by * dbw + bx) * 64;
        const int sy = ycb + by;
        if (hflip && xcb + bx < comp_width) {
          const int16_t *s = src[i].data() + ((size_t)sy * sbw[i] + (comp_width - xcb - bx - 1)) * 64;
          for (int k = 0; k < 64; k++) o[k] = (k & 1) ? (int16_t)-s[k] : s[k];
        } else {
          std::memcpy(o, src[i].data() + ((size_t)sy * sbw[i] + xcb + bx) * 64, 64 * sizeof(int16_t));
        }
      }
  }
  return nullptr;
}

// jdsample.c fancy upsampling of one component row to full width, as ints:
// h2v1 / h2v2 (triangle filters, the latter on the context rows' 3:1
// vertical sums), h1v2, full size, or integral replication otherwise.
void upsample_row(const Dec &d, int ci, const uint8_t *pl, int stride, int y, int *out) {
  const Comp &c = d.c[ci];
  const int he = d.hmax / c.h, ve = d.vmax / c.v, W = d.W, cw = c.cw, ch = c.ch;
  auto rowp = [&](int r) { return pl + (size_t)(r < 0 ? 0 : (r >= ch ? ch - 1 : r)) * stride; };
  if (he == 1 && ve == 1) {
    const uint8_t *r = pl + (size_t)y * stride;
    for (int x = 0; x < W; x++) out[x] = r[x];
  } else if (he == 2 && ve == 1) {
    const uint8_t *r = pl + (size_t)y * stride;
    for (int x = 0; x < W; x++) {
      const int col = x >> 1;
      if (cw <= 2) {
        out[x] = r[col];
      } else if (x & 1) {
        out[x] = col + 1 >= cw ? r[col] : (r[col] * 3 + r[col + 1] + 2) >> 2;
      } else {
        out[x] = col == 0 ? r[0] : (r[col] * 3 + r[col - 1] + 1) >> 2;
      }
    }
  } else if (he == 1 && ve == 2) {
    const int row = y >> 1;
    const uint8_t *a = rowp(row), *o = rowp(y & 1 ? row + 1 : row - 1);
    const int bias = y & 1 ? 2 : 1;
    for (int x = 0; x < W; x++) out[x] = (a[x] * 3 + o[x] + bias) >> 2;
  } else if (he == 2 && ve == 2) {
    const int row = y >> 1;
    const uint8_t *a = rowp(row), *o = rowp(y & 1 ? row + 1 : row - 1);
    if (cw <= 2) {
      for (int x = 0; x < W; x++) out[x] = pl[(size_t)row * stride + (x >> 1)];
      return;
    }
    // h2v2_fancy_upsample: column sums of the row and its context row, then
    // the 3:1 horizontal triangle with the edge columns replicated
    thread_local std::vector<int> cs;
    cs.resize((size_t)cw + 2);
    int *c = cs.data() + 1;
    for (int col = 0; col < cw; col++) c[col] = a[col] * 3 + o[col];
    c[-1] = c[0];
    c[cw] = c[cw - 1];
    for (int x = 0; x + 1 < W; x += 2) {
      const int col = x >> 1, t = c[col] * 3;
      out[x] = (t + c[col - 1] + 8) >> 4;
      out[x + 1] = (t + c[col + 1] + 7) >> 4;
    }
    if (W & 1) out[W - 1] = (c[(W - 1) >> 1] * 3 + c[((W - 1) >> 1) - 1] + 8) >> 4;
  } else {  // int_upsample
    const uint8_t *r = pl + (size_t)(y / ve) * stride;
    for (int x = 0; x < W; x++) out[x] = r[x / he];
  }
}


// jidctred.c (libjpeg-turbo): the reduced-size IDCTs tjDecompress2 runs at
// scaling factors 1/2, 1/4, 1/8 (DCT_scaled_size 4, 2, 1 -- islow-style,
// CONST_BITS 13, PASS1_BITS 2, the plain quantisation table as multipliers,
// whatever dct_method says), with libjpeg's zero-AC shortcuts (value-neutral)
constexpr int RCB = 13, RP1 = 2;
constexpr int64_t F0_211164243 = 1730, F0_509795579 = 4176, F0_601344887 = 4926, F0_720959822 = 5906,
                  F0_765366865 = 6270, F0_850430095 = 6967, F0_899976223 = 7373, F1_061594337 = 8697,
                  F1_272758580 = 10426, F1_451774981 = 11893, F1_847759065 = 15137, F2_172734803 = 17799,
                  F2_562915447 = 20995, F3_624509785 = 29692;
inline int64_t rdesc(int64_t x, int n) { return (x + ((int64_t)1 << (n - 1))) >> n; }

void idct_4x4(const int16_t *in, const uint16_t *q, uint8_t *out, int stride, const uint8_t *rl) {
  int64_t ws[32];
  for (int c = 0; c < 8; c++) {
    if (c == 4) continue;  // the second pass never reads column 4
    const int16_t *ip = in + c;
    const uint16_t *qp = q + c;
    int64_t *w = ws + c;
    if (!(ip[8] | ip[16] | ip[24] | ip[40] | ip[48] | ip[56])) {
      const int64_t dc = (int64_t)(ip[0] * qp[0]) * (1 << RP1);
      w[0] = w[8] = w[16] = w[24] = dc;
      continue;
    }
    int64_t t0 = (int64_t)(ip[0] * qp[0]) * ((int64_t)1 << (RCB + 1));
    const int64_t z2 = ip[16] * qp[16], z3 = ip[48] * qp[48];
    const int64_t t2 = z2 * F1_847759065 - z3 * F0_765366865;
    const int64_t t10 = t0 + t2, t12 = t0 - t2;
    const int64_t y1 = ip[56] * qp[56], y2 = ip[40] * qp[40], y3 = ip[24] * qp[24], y4 = ip[8] * qp[8];
    t0 = -y1 * F0_211164243 + y2 * F1_451774981 - y3 * F2_172734803 + y4 * F1_061594337;
    const int64_t u2 = -y1 * F0_509795579 - y2 * F0_601344887 + y3 * F0_899976223 + y4 * F2_562915447;
    w[0] = rdesc(t10 + u2, RCB - RP1 + 1);
    w[24] = rdesc(t10 - u2, RCB - RP1 + 1);
    w[8] = rdesc(t12 + t0, RCB - RP1 + 1);
    w[16] = rdesc(t12 - t0, RCB - RP1 + 1);
  }
  for (int r = 0; r < 4; r++) {
    const int64_t *w = ws + 8 * r;
    uint8_t *o = out + (size_t)r * stride;
    if (!(w[1] | w[2] | w[3] | w[5] | w[6] | w[7])) {
      o[0] = o[1] = o[2] = o[3] = rl[rdesc(w[0], RP1 + 3) & 1023];
      continue;
    }
    int64_t t0 = w[0] * ((int64_t)1 << (RCB + 1));
    const int64_t t2 = w[2] * F1_847759065 - w[6] * F0_765366865;
    const int64_t t10 = t0 + t2, t12 = t0 - t2;
    const int64_t y1 = w[7], y2 = w[5], y3 = w[3], y4 = w[1];
    t0 = -y1 * F0_211164243 + y2 * F1_451774981 - y3 * F2_172734803 + y4 * F1_061594337;
    const int64_t u2 = -y1 * F0_509795579 - y2 * F0_601344887 + y3 * F0_899976223 + y4 * F2_562915447;
    const int sh = RCB + RP1 + 3 + 1;
    o[0] = rl[rdesc(t10 + u2, sh) & 1023];
    o[3] = rl[rdesc(t10 - u2, sh) & 1023];
    o[1] = rl[rdesc(t12 + t0, sh) & 1023];
    o[2] = rl[rdesc(t12 - t0, sh) & 1023];
  }
}

void idct_2x2(const int16_t *in, const uint16_t *q, uint8_t *out, int stride, const uint8_t *rl) {
  int64_t ws[16];
  for (int c = 0; c < 8; c++) {
    if (c == 2 || c == 4 || c == 6) continue;  // not read by the second pass
    const int16_t *ip = in + c;
    const uint16_t *qp = q + c;
    int64_t *w = ws + c;
    if (!(ip[8] | ip[24] | ip[40] | ip[56])) {
      const int64_t dc = (int64_t)(ip[0] * qp[0]) * (1 << RP1);
      w[0] = w[8] = dc;
      continue;
    }
    const int64_t t10 = (int64_t)(ip[0] * qp[0]) * ((int64_t)1 << (RCB + 2));
    const int64_t t0 = -(int64_t)(ip[56] * qp[56]) * F0_720959822 + (int64_t)(ip[40] * qp[40]) * F0_850430095 -
                       (int64_t)(ip[24] * qp[24]) * F1_272758580 + (int64_t)(ip[8] * qp[8]) * F3_624509785;
    w[0] = rdesc(t10 + t0, RCB - RP1 + 2);
    w[8] = rdesc(t10 - t0, RCB - RP1 + 2);
  }
  for (int r = 0; r < 2; r++) {
    const int64_t *w = ws + 8 * r;
    uint8_t *o = out + (size_t)r * stride;
    if (!(w[1] | w[3] | w[5] | w[7])) {
      o[0] = o[1] = rl[rdesc(w[0], RP1 + 3) & 1023];
      continue;
    }
    const int64_t t10 = w[0] * ((int64_t)1 << (RCB + 2));
    const int64_t t0 = -w[7] * F0_720959822 + w[5] * F0_850430095 - w[3] * F1_272758580 + w[1] * F3_624509785;
    o[0] = rl[rdesc(t10 + t0, RCB + RP1 + 3 + 2) & 1023];
    o[1] = rl[rdesc(t10 - t0, RCB + RP1 + 3 + 2) & 1023];
  }
}

void idct_1x1(const int16_t *in, const uint16_t *q, uint8_t *out, int, const uint8_t *rl) {
  out[0] = rl[rdesc((int64_t)(in[0] * q[0]), 3) & 1023];
}

// One upsampled component row at a scaled decode (jdsample.c's choice by the
// component's sample group sizes): full size, h2v1 / h2v2 (fancy when fancy
// and the row is wider than 2 samples, else replication), h1v2 fancy, or
// integral replication.
enum UpMode { UP_FULL, UP_H2V1, UP_H2V2, UP_H1V2, UP_INT };
void upsample_row_mode(const uint8_t *pl, int stride, int cw, int ch, UpMode mode, bool fancy, int he, int ve, int y,
                       int W, int *out) {
  auto rowp = [&](int r) { return pl + (size_t)(r < 0 ? 0 : (r >= ch ? ch - 1 : r)) * stride; };
  if (mode == UP_FULL) {
    const uint8_t *r = pl + (size_t)y * stride;
    for (int x = 0; x < W; x++) out[x] = r[x];
  } else if (mode == UP_H2V1) {
    const uint8_t *r = pl + (size_t)y * stride;
    for (int x = 0; x < W; x++) {
      const int col = x >> 1;
      if (!fancy || cw <= 2)
        out[x] = r[col];
      else if (x & 1)
        out[x] = col + 1 >= cw ? r[col] : (r[col] * 3 + r[col + 1] + 2) >> 2;
      else
        out[x] = col == 0 ? r[0] : (r[col] * 3 + r[col - 1] + 1) >> 2;
    }
  } else if (mode == UP_H1V2) {
    const int row = y >> 1;
    const uint8_t *a = rowp(row), *o = rowp(y & 1 ? row + 1 : row - 1);
    const int bias = y & 1 ? 2 : 1;
    for (int x = 0; x < W; x++) out[x] = (a[x] * 3 + o[x] + bias) >> 2;
  } else if (mode == UP_H2V2) {
    const int row = y >> 1;
    if (!fancy || cw <= 2) {
      for (int x = 0; x < W; x++) out[x] = pl[(size_t)row * stride + (x >> 1)];
      return;
    }
    const uint8_t *a = rowp(row), *o = rowp(y & 1 ? row + 1 : row - 1);
    thread_local std::vector<int> cs;
    cs.resize((size_t)cw + 2);
    int *c = cs.data() + 1;
    for (int col = 0; col < cw; col++) c[col] = a[col] * 3 + o[col];
    c[-1] = c[0];
    c[cw] = c[cw - 1];
    for (int x = 0; x + 1 < W; x += 2) {
      const int col = x >> 1, t = c[col] * 3;
      out[x] = (t + c[col - 1] + 8) >> 4;
      out[x + 1] = (t + c[col + 1] + 7) >> 4;
    }
    if (W & 1) out[W - 1] = (c[(W - 1) >> 1] * 3 + c[((W - 1) >> 1) - 1] + 8) >> 4;
  } else {
    const uint8_t *r = pl + (size_t)(y / ve) * stride;
    for (int x = 0; x < W; x++) out[x] = r[x / he];
  }
}

// tjDecompress2 at 1/2, 1/4, 1/8 (sm = the luma DCT_scaled_size 4 / 2 / 1) of
// the coefficients co[] (natural order, absolute DC, whole-MCU block grids):
// libjpeg-turbo's jpeg_core_output_dimensions gives each component the
// largest DCT size (doubling from sm, below 8) that its sampling still
// divides, so 4:2:0 chroma decodes at twice the luma's size with no
// upsampling; 8 is the ifast IDCT, 4 / 2 / 1 the reduced ones; fancy
// upsampling is off at 1/8 (min DCT size 1).  Rows are packed at the
// scaled width.
const char *decode_scaled(const Dec &d, const std::vector<int16_t> co[3], int sm, uint8_t *out) {
  const Tables &T = tables();
  const int W = (d.W * sm + 7) / 8, H = (d.H * sm + 7) / 8;
  const int mcux = (d.W + 8 * d.hmax - 1) / (8 * d.hmax), mcuy = (d.H + 8 * d.vmax - 1) / (8 * d.vmax);
  thread_local std::vector<uint8_t> plane[3];
  thread_local std::vector<int> rows[3];
  int size[3], cw[3], ch[3], stride[3], he[3], ve[3];
  UpMode mode[3];
  const bool fancy = sm > 1;
  for (int i = 0; i < d.nc; i++) {
    const Comp &c = d.c[i];
    int ss = sm;
    while (ss < 8 && (d.hmax * sm) % (c.h * ss * 2) == 0 && (d.vmax * sm) % (c.v * ss * 2) == 0) ss *= 2;
    size[i] = ss;
    cw[i] = (int)(((int64_t)d.W * c.h * ss + (int64_t)d.hmax * 8 - 1) / ((int64_t)d.hmax * 8));
    ch[i] = (int)(((int64_t)d.H * c.v * ss + (int64_t)d.vmax * 8 - 1) / ((int64_t)d.vmax * 8));
    const int bw = mcux * c.h, bh = mcuy * c.v;
    stride[i] = bw * ss;
    plane[i].resize((size_t)stride[i] * bh * ss);
    int16_t qf[64];
    uint16_t qn[64];
    for (int k = 0; k < 64; k++) {
      qn[k] = d.qt[c.tq][k];
      qf[k] = (int16_t)(((int64_t)d.qt[c.tq][k] * kAanScales[k] + (1 << 11)) >> 12);
    }
    for (int by = 0; by < bh; by++)
      for (int bx = 0; bx < bw; bx++) {
        const int16_t *b = co[i].data() + ((size_t)by * bw + bx) * 64;
        uint8_t *o = plane[i].data() + (size_t)by * ss * stride[i] + (size_t)bx * ss;
        if (ss == 8)
          idct_ifast(b, qf, o, stride[i], T.rl);
        else if (ss == 4)
          idct_4x4(b, qn, o, stride[i], T.rl);
        else if (ss == 2)
          idct_2x2(b, qn, o, stride[i], T.rl);
        else
          idct_1x1(b, qn, o, stride[i], T.rl);
      }
    const int hin = c.h * ss / sm, vin = c.v * ss / sm;
    he[i] = ve[i] = 1;
    if (hin == d.hmax && vin == d.vmax)
      mode[i] = UP_FULL;
    else if (hin * 2 == d.hmax && vin == d.vmax)
      mode[i] = UP_H2V1;
    else if (hin * 2 == d.hmax && vin * 2 == d.vmax)
      mode[i] = UP_H2V2;
    else if (hin == d.hmax && vin * 2 == d.vmax && fancy)
      mode[i] = UP_H1V2;
    else {
      if (d.hmax % hin || d.vmax % vin) return "fractional upsampling at this scale";
      mode[i] = UP_INT;
      he[i] = d.hmax / hin;
      ve[i] = d.vmax / vin;
    }
    rows[i].resize((size_t)W);
  }
  for (int y = 0; y < H; y++) {
    uint8_t *o = out + (size_t)y * W * 3;
    if (d.nc == 1) {
      const uint8_t *r = plane[0].data() + (size_t)y * stride[0];
      for (int x = 0; x < W; x++) o[3 * x] = o[3 * x + 1] = o[3 * x + 2] = r[x];
      continue;
    }
    for (int i = 0; i < 3; i++)
      upsample_row_mode(plane[i].data(), stride[i], cw[i], ch[i], mode[i], fancy, he[i], ve[i], y, W, rows[i].data());
    const int *r0 = rows[0].data(), *r1 = rows[1].data(), *r2 = rows[2].data();
    for (int x = 0; x < W; x++) {
      if (d.color_rgb) {
        o[3 * x] = (uint8_t)r0[x];
        o[3 * x + 1] = (uint8_t)r1[x];
        o[3 * x + 2] = (uint8_t)r2[x];
        continue;
      }
      const int yy = r0[x], cb = r1[x], cr = r2[x];
      const int R = yy + T.cr_r[cr], G = yy + ((T.cb_g[cb] + T.cr_g[cr]) >> 16), B = yy + T.cb_b[cb];
      o[3 * x] = (uint8_t)(R < 0 ? 0 : (R > 255 ? 255 : R));
      o[3 * x + 1] = (uint8_t)(G < 0 ? 0 : (G > 255 ? 255 : G));
      o[3 * x + 2] = (uint8_t)(B < 0 ? 0 : (B > 255 ? 255 : B));
    }
  }
  return nullptr;
}

}  // namespace

extern "C" {

int imdecode(unsigned char *input_buffer, uint64_t input_size, uint32_t source_height, uint32_t source_width,
             unsigned char *output_buffer, uint32_t crop_height, uint32_t crop_width, uint32_t offset_x,
             uint32_t offset_y, uint32_t scale_num, uint32_t scale_denom, bool enable_crop, bool hflip) {
  (void)source_height;  // unused by the reference too (libffcv.cpp:53-112)
  (void)source_width;
  if (!input_buffer || !output_buffer || input_size == 0 || crop_height == 0 || crop_width == 0 || scale_num == 0 ||
      scale_denom == 0) {
    ffcv::set_error("imdecode: invalid arguments");
    return -1;
  }
  Dec d;
  if (const char *err = parse(input_buffer, input_size, d)) {
    ffcv::set_error("imdecode: %s", err);
    return -1;
  }
  Scratch &S = t_scr;
  int stride[3] = {0, 0, 0};
  // libffcv.cpp:95-100: crop (always, with the offsets and size) and the
  // optional mirror when enable_crop or hflip, else the stream as it is
  const bool transform = enable_crop || hflip;
  thread_local std::vector<int16_t> tco[3];
  if (transform) {
    if (const char *err = transform_coefs(input_buffer, d, offset_x, offset_y, crop_width, crop_height, hflip, tco)) {
      ffcv::set_error("imdecode: tjTransform: %s", err);
      return -1;
    }
  }
  // libffcv.cpp:101-103 tjDecompress2(width = TJSCALED(crop_width, scaling),
  // height = TJSCALED(crop_height, scaling), pitch 0): TurboJPEG decodes at
  // the largest of its factors whose output fits; rows are packed at the
  // decoded width.  Only the factor 1/1 (ifast 8x8) is restated here.
  const uint32_t req_w = (uint32_t)(((uint64_t)crop_width * scale_num + scale_denom - 1) / scale_denom);
  const uint32_t req_h = (uint32_t)(((uint64_t)crop_height * scale_num + scale_denom - 1) / scale_denom);
  int fn = 0, fd = 0;
  if (tj_scale_choice(d.W, d.H, req_w, req_h, &fn, &fd)) {
    ffcv::set_error("imdecode: the %dx%d image cannot be scaled into %ux%u", d.H, d.W, req_h, req_w);
    return -1;
  }
  if (fn != fd && !(fn == 1 && (fd == 2 || fd == 4 || fd == 8))) {
    ffcv::set_error("imdecode: the %dx%d image would decode at scale %d/%d into %ux%u (only 1/1, 1/2, 1/4 and "
                    "1/8 are supported)", d.H, d.W, fn, fd, req_h, req_w);
    return -1;
  }
  if (fn != fd) {  // jidctred.c's reduced IDCTs (decode_scaled)
    if (!transform) {  // the stream's coefficients
      const int mcux = (d.W + 8 * d.hmax - 1) / (8 * d.hmax), mcuy = (d.H + 8 * d.vmax - 1) / (8 * d.vmax);
      int bw[3];
      for (int i = 0; i < d.nc; i++) {
        bw[i] = mcux * d.c[i].h;
        tco[i].assign((size_t)bw[i] * mcuy * d.c[i].v * 64, 0);
      }
      decode_scan(input_buffer, d, [&](int ci, int bx, int by, const int16_t *blk) {
        std::memcpy(tco[ci].data() + ((size_t)by * bw[ci] + bx) * 64, blk, 64 * sizeof(int16_t));
      });
    }
    if (const char *err = decode_scaled(d, tco, 8 / fd, output_buffer)) {
      ffcv::set_error("imdecode: %s", err);
      return -1;
    }
    return 0;
  }
  if (transform) {
    const Tables &T = tables();
    int16_t qm[3][64];
    plane_setup(d, S, stride, qm);
    for (int i = 0; i < d.nc; i++) {
      const Comp &c = d.c[i];
      for (int by = 0; by < c.bh; by++)
        for (int bx = 0; bx < c.bw; bx++)
          idct_ifast(tco[i].data() + ((size_t)by * c.bw + bx) * 64, qm[i],
                     S.plane[i].data() + (size_t)by * 8 * stride[i] + bx * 8, stride[i], T.rl);
    }
  } else {
    decode_planes(input_buffer, d, S, stride);
  }
  const Tables &T = tables();
  const int W = d.W;
  for (int i = 0; i < d.nc; i++) S.row[i].resize((size_t)W);
  for (int y = 0; y < d.H; y++) {
    uint8_t *o = output_buffer + (size_t)y * W * 3;
    if (d.nc == 1) {
      const uint8_t *r = S.plane[0].data() + (size_t)y * stride[0];
      for (int x = 0; x < W; x++) o[3 * x] = o[3 * x + 1] = o[3 * x + 2] = r[x];
      continue;
    }
    for (int i = 0; i < 3; i++) upsample_row(d, i, S.plane[i].data(), stride[i], y, S.row[i].data());
    const int *r0 = S.row[0].data(), *r1 = S.row[1].data(), *r2 = S.row[2].data();
    if (d.color_rgb) {
      for (int x = 0; x < W; x++) {
        o[3 * x] = (uint8_t)r0[x];
        o[3 * x + 1] = (uint8_t)r1[x];
        o[3 * x + 2] = (uint8_t)r2[x];
      }
      continue;
    }
    for (int x = 0; x < W; x++) {  // jdcolor.c ycc_rgb_convert
      const int yy = r0[x], cb = r1[x], cr = r2[x];
      const int R = yy + T.cr_r[cr], G = yy + ((T.cb_g[cb] + T.cr_g[cr]) >> 16), B = yy + T.cb_b[cb];
      o[3 * x] = (uint8_t)(R < 0 ? 0 : (R > 255 ? 255 : R));
      o[3 * x + 1] = (uint8_t)(G < 0 ? 0 : (G > 255 ? 255 : G));
      o[3 * x + 2] = (uint8_t)(B < 0 ? 0 : (B > 255 ? 255 : B));
    }
  }
  return 0;
}

// The reference's per-sample CPU loop under numba prange (rgb_image.py:
// 123-136 Simple, :185-210 ResizedCrop) as one native call over nthreads
// threads: sample k (bytes data[k][0, sizes[k]), h x w, mode 0 = jpg, 1 =
// raw, anything else = skip) is decoded by imdecode or taken as is, then
// with crops (B x 4: i, j, h, w) cut and resized by resize() (INTER_AREA) to
// out_h x out_w, or without crops written whole, at out + k * out_stride.
// status[k] = 0, or -1 when its decode failed (ffcv_last_error() holds the
// last message).  Samples are handed out one at a time from an atomic
// counter (their sizes differ).
int ffcv_cpu_decode_batch(const uint8_t *const *data, const uint64_t *sizes, const uint32_t *heights,
                          const uint32_t *widths, const uint32_t *modes, int batch, const int32_t *crops,
                          int out_h, int out_w, uint8_t *out, uint64_t out_stride, int nthreads,
                          int32_t *status) {
  if (batch < 0 || (batch > 0 && (!data || !sizes || !heights || !widths || !modes || !out || !status)) ||
      (crops && (out_h <= 0 || out_w <= 0))) {
    ffcv::set_error("ffcv_cpu_decode_batch: invalid arguments");
    return FFCV_EINVAL;
  }
  std::atomic<int> next{0};
  // the first failing sample's message: set_error is thread-local, so a
  // worker's message is copied here and re-raised on the calling thread
  std::mutex err_mu;
  int err_k = batch;
  std::string err_msg;
  auto fail = [&](int k, const char *msg) {
    status[k] = -1;
    std::lock_guard<std::mutex> g(err_mu);
    if (k < err_k) {
      err_k = k;
      err_msg = msg;
    }
  };
  auto work = [&]() {
    std::vector<uint8_t> img;
    for (int k = next.fetch_add(1); k < batch; k = next.fetch_add(1)) {
      const uint32_t h = heights[k], w = widths[k], mode = modes[k];
      status[k] = 0;
      if (mode > 1) continue;
      uint8_t *dst = out + (uint64_t)k * out_stride;
      const uint8_t *src = data[k];
      if (mode == 0) {
        uint8_t *o = dst;
        if (crops) {
          img.resize((size_t)h * w * 3);
          o = img.data();
        }
        if (imdecode(const_cast<uint8_t *>(data[k]), sizes[k], h, w, o, h, w, 0, 0, 1, 1, false, false) != 0) {
          fail(k, ffcv_last_error());
          continue;
        }
        src = o;
      } else if (sizes[k] < (uint64_t)h * w * 3) {  // a truncated / mislabelled raw sample
        char buf[160];
        snprintf(buf, sizeof(buf), "raw sample %d holds %llu bytes, %ux%ux3 needs %llu", k,
                 (unsigned long long)sizes[k], h, w, (unsigned long long)h * w * 3);
        fail(k, buf);
        continue;
      } else if (!crops) {
        std::memcpy(dst, src, (size_t)h * w * 3);
        continue;
      }
      if (crops) {
        const int32_t *c = crops + 4 * k;
        resize(0, (int64_t)(uintptr_t)src, h, w, c[0], c[0] + c[2], c[1], c[1] + c[3], (int64_t)(uintptr_t)dst,
               out_h, out_w);
      }
    }
  };
  const int T = std::max(1, std::min(nthreads, batch));
  std::vector<std::thread> th;
  th.reserve(T - 1);
  for (int t = 1; t < T; t++) th.emplace_back(work);
  work();
  for (auto &x : th) x.join();
  if (err_k < batch) ffcv::set_error("sample %d: %s", err_k, err_msg.c_str());
  return FFCV_OK;
}

// Measurement helper (bench.py's K1 lane-instructions per symbol): per
// image, the Huffman symbols (DC + AC, EOB and ZRL included) and the blocks of
// its scan.  stats[3k..3k+2] = symbols, blocks, entropy-coded bytes; an image
// that does not parse gets zeros and -1 is returned after the rest.
int ffcv_jpeg_scan_stats(const uint8_t *const *data, const uint64_t *sizes, int n, uint64_t *stats) {
  if ((!data || !sizes || !stats) && n > 0) {
    ffcv::set_error("ffcv_jpeg_scan_stats: invalid arguments");
    return FFCV_EINVAL;
  }
  int rc = FFCV_OK;
  for (int k = 0; k < n; k++) {
    uint64_t *o = stats + 3 * (size_t)k;
    o[0] = o[1] = o[2] = 0;
    Dec d;
    if (!data[k] || parse(data[k], sizes[k], d)) {
      rc = -1;
      continue;
    }
    uint64_t nsym = 0, nblk = 0;
    decode_scan(data[k], d, [&](int, int, int, const int16_t *) { nblk++; }, &nsym);
    o[0] = nsym;
    o[1] = nblk;
    o[2] = d.ecs_end - d.ecs;
  }
  return rc;
}

}  // extern "C"
