// ffcv_jpeg.hip -- baseline JPEG decode on gfx950, fused with the RRC crop,
// INTER_AREA resize and the flip / cutout / normalize epilogue.
//
// Reference: rgb_image.py:194-208 decodes every JPEG in full with
// libjpeg-turbo (libffcv.cpp:104-106: tjDecompress2(TJPF_RGB,
// TJFLAG_FASTDCT) = ifast IDCT + fancy upsampling + fixed-point YCbCr->RGB)
// into a temp buffer, then crops and resizes.  Here one 256-lane workgroup
// owns one image and runs, with workgroup barriers between phases:
//
//   P0  marker parse (one lane), geometry / table validation
//   P1  Huffman lookup tables (9-bit fast LUT + canonical slow path) and the
//       ifast dequantisation multipliers, in LDS
//   P2  de-stuffing of the entropy-coded segment (0xFF00 -> 0xFF) into a
//       word-aligned scratch stream (chunked count -> workgroup scan -> copy)
//   P3  self-synchronising parallel Huffman decode: the stream is cut into
//       one bit-range per lane; every lane decodes its range from a guessed
//       decoder state (bit position, coefficient index z, block-in-MCU) and
//       records the state at which it leaves the range.  The guess of lane
//       t+1 is then replaced by lane t's exit state until no guess changes
//       (lane 0 is exact, so after r rounds lanes 0..r are exact; JPEG
//       streams resynchronise within a few codewords, so 1-2 extra rounds
//       suffice in practice).  No restart markers are needed.
//   P4  workgroup prefix scans of blocks-started and per-component DC diffs
//       give every lane its first block index and DC predictor
//   P5  second decode pass writes the quantised coefficients (natural order)
//       of the blocks the crop needs into a plane-ordered scratch
//   P6  dequantise + ifast IDCT (jidctfst.c) of exactly those blocks
//   P7  fancy upsampling (jdsample.c) + YCbCr->RGB (jdcolor.c) of the crop ROI
//   P8  INTER_AREA resize of the ROI (OpenCV 4.5.4) + flip/cutout/LUT
//
// Every integer step is restated from libjpeg-turbo and matches it bit for
// bit (tests/test_jpeg_gpu.py); the float steps of the resize are compiled
// with -ffp-contract=off.
#include "api_internal.h"
#include "device_common.h"

#define JT 256
#define FAST_BITS 9
#define NTAB 8

enum JMode { JM_RRC = 0, JM_FULL = 1, JM_COEF = 2 };

struct HuffTab {
  uint16_t lut[1 << FAST_BITS];  // (len << 8) | sym; len 0 => slow path
  int32_t maxcode[18];
  int32_t valoff[17];
  uint8_t vals[256];
};

struct JShared {
  int status;
  int W, H, ncomp, hmax, vmax;
  int hs[3], vs[3], tq[3], td[3], ta[3], cid[3];
  int color_rgb;
  int mcux, mcuy, bpm, nblocks;
  int cw[3], ch[3], bw[3], bh[3];
  int blk_comp[10], blk_dx[10], blk_dy[10];
  uint32_t scan_off, scan_end;
  uint32_t dqt_off[4];
  int dqt_prec[4], dqt_ok[4];
  uint32_t dht_off[NTAB];
  int dht_ok[NTAB];
  int saw_jfif, saw_adobe, adobe_transform;
  int restart;
  // crop window (full-res pixels) and per-component block windows
  int ri, rj, rh, rw;
  int wx0[3], wx1[3], wy0[3], wy1[3];
  uint64_t coff[3];  // offset (in blocks) of each component in the coef scratch
  uint64_t poff[3];  // offset (bytes) of each component plane
  // destuff
  uint32_t first_marker;
  uint32_t dlen;
  int nthr;
  uint32_t chunk_bits;
  int any;
  HuffTab tab[NTAB];
  int16_t qmul[3][64];
  uint8_t nat[80];
  // per-lane decoder states
  uint32_t g_pos[JT];
  uint32_t e_pos[JT];
  uint8_t g_z[JT], g_ph[JT], e_z[JT], e_ph[JT];
  uint32_t cnt[JT];
  int32_t dcs[3][JT];
  uint32_t scan_tmp[JT];
  int32_t scan_tmp2[3][JT];
};

__constant__ uint8_t c_natural[80] = {
    0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33,
    40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36,
    29, 22, 15, 23, 30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54,
    47, 55, 62, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63};

__constant__ int32_t c_aanscales[64] = {
    16384, 22725, 21407, 19266, 16384, 12873, 8867,  4520,  22725, 31521, 29692, 26722, 22725,
    17855, 12299, 6270,  21407, 29692, 27969, 25172, 21407, 16819, 11585, 5906,  19266, 26722,
    25172, 22654, 19266, 15137, 10426, 5315,  16384, 22725, 21407, 19266, 16384, 12873, 8867,
    4520,  12873, 17855, 16819, 15137, 12873, 10114, 6967,  3552,  8867,  12299, 11585, 10426,
    8867,  6967,  4799,  2446,  4520,  6270,  5906,  5315,  4520,  3552,  2446,  1247};

FFCV_DEV int rd16(const uint8_t *p) { return (p[0] << 8) | p[1]; }

// ----------------------------------------------------------- bit reader --
struct BitReader {
  const uint32_t *w;
  uint32_t nw;
  uint64_t acc;
  int nb;
  uint32_t wi;
  uint32_t pos;
  FFCV_DEV uint32_t ld(uint32_t i) const { return i < nw ? __builtin_bswap32(w[i]) : 0u; }
  FFCV_DEV void init(uint32_t p) {
    wi = p >> 5;
    acc = ((uint64_t)ld(wi) << 32) | (uint64_t)ld(wi + 1);
    acc <<= (p & 31);
    nb = 64 - (int)(p & 31);
    wi += 2;
    pos = p;
  }
  FFCV_DEV uint32_t peek16() const { return (uint32_t)(acc >> 48); }
  FFCV_DEV uint32_t peek(int n) const { return n ? (uint32_t)(acc >> (64 - n)) : 0u; }
  FFCV_DEV void consume(int n) {
    acc <<= n;
    nb -= n;
    pos += n;
    if (nb <= 32) {
      acc |= (uint64_t)ld(wi) << (32 - nb);
      wi++;
      nb += 32;
    }
  }
};

FFCV_DEV int huff_extend(int x, int s) { return x < (1 << (s - 1)) ? x + (int)(0xFFFFFFFFu << s) + 1 : x; }

// Decode one Huffman symbol; returns symbol, consumes its code.
FFCV_DEV int huff_sym(const HuffTab &t, BitReader &br) {
  uint32_t look = br.peek16();
  uint32_t e = t.lut[look >> (16 - FAST_BITS)];
  int len = (int)(e >> 8);
  int sym;
  if (len) {
    sym = (int)(e & 0xff);
  } else {
    sym = 0;
    len = 16;
    for (int l = FAST_BITS + 1; l <= 16; l++) {
      int code = (int)(look >> (16 - l));
      if (code <= t.maxcode[l]) {
        sym = t.vals[(t.valoff[l] + code) & 0xff];
        len = l;
        break;
      }
    }
  }
  br.consume(len);
  return sym;
}

struct DecState {
  uint32_t pos;
  int z;   // 0: next symbol is a DC; else index of next AC coefficient
  int ph;  // block index inside the MCU
};

// Decode units (Huffman symbol + extra bits) from st until the first unit
// boundary at or past end_bit (WRITE mode additionally stops after the last
// block of the image).  SYNC mode counts blocks started and sums DC diffs per
// component; WRITE mode stores coefficients of blocks inside the window.
template <bool WRITE>
FFCV_DEV DecState decode_range(JShared &S, const uint32_t *words, uint32_t nwords, DecState st,
                               uint32_t end_bit, uint32_t *n_started, int32_t dcsum[3], int64_t blk,
                               int32_t pred[3], int16_t *coef) {
  BitReader br;
  br.w = words;
  br.nw = nwords;
  br.init(st.pos);
  int z = st.z, ph = st.ph;
  uint32_t started = 0;
  int comp = S.blk_comp[ph];
  const HuffTab *dct = &S.tab[S.td[comp]];
  const HuffTab *act = &S.tab[4 + S.ta[comp]];
  // block coordinates (WRITE mode)
  int mx = 0, my = 0;
  int16_t *bptr = nullptr;
  bool inwin = false;
  auto locate = [&](int64_t b) {
    int64_t m = b / S.bpm;
    int p = (int)(b - m * S.bpm);
    my = (int)(m / S.mcux);
    mx = (int)(m - (int64_t)my * S.mcux);
    int c = S.blk_comp[p];
    int bx = mx * S.hs[c] + S.blk_dx[p];
    int by = my * S.vs[c] + S.blk_dy[p];
    inwin = b < S.nblocks && bx >= S.wx0[c] && bx <= S.wx1[c] && by >= S.wy0[c] && by <= S.wy1[c];
    bptr = coef + (S.coff[c] + (uint64_t)by * S.bw[c] + bx) * 64;
  };
  if (WRITE && z > 0) locate(blk);  // continuing a block started earlier
  while (br.pos < end_bit) {
    if (WRITE && z == 0 && blk >= S.nblocks) break;
    if (z == 0) {
      int s = huff_sym(*dct, br);
      int diff = 0;
      if (s) {
        diff = huff_extend((int)br.peek(s), s);
        br.consume(s);
      }
      started++;
      if (WRITE) {
        locate(blk);
        pred[comp] += diff;
        if (inwin) bptr[0] = (int16_t)pred[comp];
      } else {
        dcsum[comp] += diff;
      }
      z = 1;
    } else {
      int rs = huff_sym(*act, br);
      int r = rs >> 4, s = rs & 15;
      if (s) {
        z += r;
        int v = huff_extend((int)br.peek(s), s);
        br.consume(s);
        if (WRITE && inwin) bptr[S.nat[z]] = (int16_t)v;
        z++;
      } else if (r == 15) {
        z += 16;
      } else {
        z = 64;
      }
    }
    if (z >= 64) {
      z = 0;
      ph++;
      if (ph == S.bpm) ph = 0;
      comp = S.blk_comp[ph];
      dct = &S.tab[S.td[comp]];
      act = &S.tab[4 + S.ta[comp]];
      if (WRITE) blk++;
    }
  }
  if (n_started) *n_started = started;
  DecState out;
  out.pos = br.pos;
  out.z = z;
  out.ph = ph;
  return out;
}

// Workgroup exclusive scan of one uint32 per lane (returns exclusive prefix).
FFCV_DEV uint32_t wg_exscan_u32(uint32_t v, uint32_t *tmp) {
  const int t = threadIdx.x;
  tmp[t] = v;
  __syncthreads();
  for (int off = 1; off < JT; off <<= 1) {
    uint32_t x = t >= off ? tmp[t - off] : 0u;
    __syncthreads();
    tmp[t] += x;
    __syncthreads();
  }
  uint32_t incl = tmp[t];
  __syncthreads();
  return incl - v;
}
FFCV_DEV int32_t wg_exscan_i32(int32_t v, int32_t *tmp) {
  const int t = threadIdx.x;
  tmp[t] = v;
  __syncthreads();
  for (int off = 1; off < JT; off <<= 1) {
    int32_t x = t >= off ? tmp[t - off] : 0;
    __syncthreads();
    tmp[t] += x;
    __syncthreads();
  }
  int32_t incl = tmp[t];
  __syncthreads();
  return incl - v;
}

// libjpeg post-IDCT range limit: table[x & 1023] (jdmaster.c)
FFCV_DEV uint8_t idct_rl(int x) {
  int v = x & 1023;
  return (uint8_t)(v < 128 ? v + 128 : (v < 512 ? 255 : (v < 896 ? 0 : v - 896)));
}
FFCV_DEV int fmul8(int v, int c) { return (int)(((int64_t)v * c) >> 8); }

// jidctfst.c jpeg_idct_ifast on one block (coefficients already loaded).
FFCV_DEV void idct_ifast_block(const int16_t *in, const int16_t *q, uint8_t *out, int stride) {
  int ws[64];
#pragma unroll
  for (int c = 0; c < 8; c++) {
    int i0 = in[c], i1 = in[8 + c], i2 = in[16 + c], i3 = in[24 + c], i4 = in[32 + c], i5 = in[40 + c],
        i6 = in[48 + c], i7 = in[56 + c];
    if ((i1 | i2 | i3 | i4 | i5 | i6 | i7) == 0) {
      int dc = i0 * q[c];
#pragma unroll
      for (int r = 0; r < 8; r++) ws[8 * r + c] = dc;
      continue;
    }
    int tmp0 = i0 * q[c], tmp1 = i2 * q[16 + c], tmp2 = i4 * q[32 + c], tmp3 = i6 * q[48 + c];
    int tmp10 = tmp0 + tmp2, tmp11 = tmp0 - tmp2;
    int tmp13 = tmp1 + tmp3, tmp12 = fmul8(tmp1 - tmp3, 362) - tmp13;
    tmp0 = tmp10 + tmp13;
    tmp3 = tmp10 - tmp13;
    tmp1 = tmp11 + tmp12;
    tmp2 = tmp11 - tmp12;
    int tmp4 = i1 * q[8 + c], tmp5 = i3 * q[24 + c], tmp6 = i5 * q[40 + c], tmp7 = i7 * q[56 + c];
    int z13 = tmp6 + tmp5, z10 = tmp6 - tmp5, z11 = tmp4 + tmp7, z12 = tmp4 - tmp7;
    tmp7 = z11 + z13;
    tmp11 = fmul8(z11 - z13, 362);
    int z5 = fmul8(z10 + z12, 473);
    tmp10 = fmul8(z12, 277) - z5;
    tmp12 = fmul8(z10, -669) + z5;
    tmp6 = tmp12 - tmp7;
    tmp5 = tmp11 - tmp6;
    tmp4 = tmp10 + tmp5;
    ws[c] = tmp0 + tmp7;
    ws[56 + c] = tmp0 - tmp7;
    ws[8 + c] = tmp1 + tmp6;
    ws[48 + c] = tmp1 - tmp6;
    ws[16 + c] = tmp2 + tmp5;
    ws[40 + c] = tmp2 - tmp5;
    ws[32 + c] = tmp3 + tmp4;
    ws[24 + c] = tmp3 - tmp4;
  }
#pragma unroll
  for (int r = 0; r < 8; r++) {
    const int *w = ws + 8 * r;
    uint8_t o[8];
    if ((w[1] | w[2] | w[3] | w[4] | w[5] | w[6] | w[7]) == 0) {
      uint8_t dc = idct_rl(w[0] >> 5);
#pragma unroll
      for (int k = 0; k < 8; k++) o[k] = dc;
    } else {
      int tmp10 = w[0] + w[4], tmp11 = w[0] - w[4];
      int tmp13 = w[2] + w[6], tmp12 = fmul8(w[2] - w[6], 362) - tmp13;
      int tmp0 = tmp10 + tmp13, tmp3 = tmp10 - tmp13, tmp1 = tmp11 + tmp12, tmp2 = tmp11 - tmp12;
      int z13 = w[5] + w[3], z10 = w[5] - w[3], z11 = w[1] + w[7], z12 = w[1] - w[7];
      int tmp7 = z11 + z13;
      tmp11 = fmul8(z11 - z13, 362);
      int z5 = fmul8(z10 + z12, 473);
      tmp10 = fmul8(z12, 277) - z5;
      tmp12 = fmul8(z10, -669) + z5;
      int tmp6 = tmp12 - tmp7, tmp5 = tmp11 - tmp6, tmp4 = tmp10 + tmp5;
      o[0] = idct_rl((tmp0 + tmp7) >> 5);
      o[7] = idct_rl((tmp0 - tmp7) >> 5);
      o[1] = idct_rl((tmp1 + tmp6) >> 5);
      o[6] = idct_rl((tmp1 - tmp6) >> 5);
      o[2] = idct_rl((tmp2 + tmp5) >> 5);
      o[5] = idct_rl((tmp2 - tmp5) >> 5);
      o[4] = idct_rl((tmp3 + tmp4) >> 5);
      o[3] = idct_rl((tmp3 - tmp4) >> 5);
    }
    uint32_t lo = o[0] | (o[1] << 8) | (o[2] << 16) | ((uint32_t)o[3] << 24);
    uint32_t hi = o[4] | (o[5] << 8) | (o[6] << 16) | ((uint32_t)o[7] << 24);
    uint2 v;
    v.x = lo;
    v.y = hi;
    *(uint2 *)(out + (uint64_t)r * stride) = v;
  }
}

// jdsample.c upsampling of component c at full-resolution sample (y, x),
// with libjpeg's context-row edge replication.
FFCV_DEV int plane_at(const uint8_t *p, int stride, int ch, int y, int x) {
  y = y < 0 ? 0 : (y >= ch ? ch - 1 : y);
  return p[(uint64_t)y * stride + x];
}
FFCV_DEV int upsample_at(const uint8_t *p, int stride, int cw, int ch, int he, int ve, int y, int x) {
  if (he == 1 && ve == 1) return p[(uint64_t)y * stride + x];
  if (he == 2 && ve == 1) {
    int col = x >> 1;
    const uint8_t *row = p + (uint64_t)y * stride;
    if (cw <= 2) return row[col];
    int cur = row[col] * 3;
    if (x & 1) {
      if (col + 1 >= cw) return row[col];
      return (cur + row[col + 1] + 2) >> 2;
    }
    if (col == 0) return row[0];
    return (cur + row[col - 1] + 1) >> 2;
  }
  if (he == 1 && ve == 2) {
    int r = y >> 1, other = (y & 1) ? r + 1 : r - 1;
    int sum = plane_at(p, stride, ch, r, x) * 3 + plane_at(p, stride, ch, other, x);
    return (sum + ((y & 1) ? 2 : 1)) >> 2;
  }
  if (he == 2 && ve == 2) {
    int r = y >> 1, col = x >> 1;
    if (cw <= 2) return p[(uint64_t)r * stride + col];
    int other = (y & 1) ? r + 1 : r - 1;
    int rc = r < 0 ? 0 : (r >= ch ? ch - 1 : r);
    int oc = other < 0 ? 0 : (other >= ch ? ch - 1 : other);
    const uint8_t *r0 = p + (uint64_t)rc * stride, *r1 = p + (uint64_t)oc * stride;
    int thiss = r0[col] * 3 + r1[col];
    if (x & 1) {
      int nxt = col + 1 < cw ? r0[col + 1] * 3 + r1[col + 1] : thiss;
      return (thiss * 3 + nxt + 7) >> 4;
    }
    int last = col > 0 ? r0[col - 1] * 3 + r1[col - 1] : thiss;
    return (thiss * 3 + last + 8) >> 4;
  }
  return p[(uint64_t)(y / ve) * stride + x / he];  // int_upsample
}

// jdcolor.c ycc_rgb_convert with build_ycc_rgb_table's fixed point (16 bits)
FFCV_DEV void ycc_rgb(int y, int cb, int cr, int out[3]) {
  int x_cb = cb - 128, x_cr = cr - 128;
  int r = y + ((91881 * x_cr + 32768) >> 16);
  int g = y + ((-22554 * x_cb + 32768 + -46802 * x_cr) >> 16);
  int b = y + ((116130 * x_cb + 32768) >> 16);
  out[0] = sat_u8i(r);
  out[1] = sat_u8i(g);
  out[2] = sat_u8i(b);
}

struct JpegArgs {
  const uint8_t *base;
  const ffcv_sample *samples;
  const int32_t *crops;
  const int32_t *cut;
  const uint8_t *flips;
  ffcv_rrc_params p;
  void *out;
  uint64_t out_stride;
  int32_t *status;
  // scratch
  uint8_t *dstuff;
  uint64_t dstuff_slot;
  int16_t *coef;
  uint64_t coef_slot;  // in int16 elements
  uint8_t *planes;
  uint64_t plane_slot;
  uint8_t *roi;
  uint64_t roi_slot;
  uint32_t max_h, max_w;
  uint64_t max_blocks;  // JM_COEF output capacity
  uint64_t *dbg;        // optional per-image phase stamps (diagnostic builds)
};

// Diagnostic stamps: lane 0 records s_memtime at phase boundaries into
// dbg[image*16 + slot] (never read by the kernel; off when dbg == nullptr).
#define STAMP(slot)                                                          \
  do {                                                                       \
    if (a.dbg && t == 0) a.dbg[(uint64_t)k * 16 + (slot)] = wall_clock64();  \
  } while (0)

struct RoiScratch {
  const uint8_t *p;
  uint64_t step;
  FFCV_DEV int at(int y, int x, int c) const { return p[(uint64_t)y * step + (uint64_t)x * 3 + c]; }
};

template <int MODE, bool FP16>
__global__ void __launch_bounds__(JT) jpeg_kernel(JpegArgs a) {
  __shared__ JShared S;
  const int t = threadIdx.x;
  const int k = blockIdx.x;
  const ffcv_sample smp = a.samples[k];
  if (smp.mode != 0) {  // raw samples are handled by rrc_raw_kernel / gather
    if (t == 0) a.status[k] = FFCV_SAMPLE_OK;
    return;
  }
  const uint8_t *src = a.base + smp.offset;
  const uint32_t nbytes = (uint32_t)smp.size;

  // ------------------------------------------------------------- P0 ----
  STAMP(0);
  if (t == 0) {
    int st = FFCV_SAMPLE_OK;
    for (int i = 0; i < 4; i++) S.dqt_ok[i] = 0;
    for (int i = 0; i < NTAB; i++) S.dht_ok[i] = 0;
    S.saw_jfif = S.saw_adobe = 0;
    S.adobe_transform = 1;
    S.restart = 0;
    S.ncomp = 0;
    int have_sof = 0, have_sos = 0;
    if (nbytes < 4 || src[0] != 0xFF || src[1] != 0xD8) st = FFCV_SAMPLE_BAD_MARKER;
    uint32_t p = 2;
    while (st == FFCV_SAMPLE_OK && !have_sos) {
      if (p + 4 > nbytes || src[p] != 0xFF) {
        st = FFCV_SAMPLE_BAD_MARKER;
        break;
      }
      while (p < nbytes && src[p] == 0xFF) p++;
      if (p >= nbytes) {
        st = FFCV_SAMPLE_BAD_MARKER;
        break;
      }
      int m = src[p++];
      if (m == 0xD8 || (m >= 0xD0 && m <= 0xD7) || m == 0x01) continue;
      if (m == 0xD9 || p + 2 > nbytes) {
        st = FFCV_SAMPLE_BAD_MARKER;
        break;
      }
      int len = rd16(src + p);
      if (len < 2 || p + (uint32_t)len > nbytes) {
        st = FFCV_SAMPLE_BAD_MARKER;
        break;
      }
      const uint8_t *s = src + p + 2;
      int sl = len - 2;
      if (m == 0xDB) {
        int o = 0;
        while (o < sl) {
          int pq = s[o] >> 4, tq = s[o] & 15;
          if (tq > 3) {
            st = FFCV_SAMPLE_BAD_MARKER;
            break;
          }
          S.dqt_off[tq] = p + 2 + o + 1;
          S.dqt_prec[tq] = pq;
          S.dqt_ok[tq] = 1;
          o += 1 + (pq ? 128 : 64);
        }
      } else if (m == 0xC4) {
        int o = 0;
        while (o < sl) {
          int tc = s[o] >> 4, th = s[o] & 15;
          if (th > 3 || tc > 1) {
            st = FFCV_SAMPLE_BAD_MARKER;
            break;
          }
          int total = 0;
          for (int l = 0; l < 16; l++) total += s[o + 1 + l];
          if (total > 256) {
            st = FFCV_SAMPLE_BAD_MARKER;
            break;
          }
          S.dht_off[tc * 4 + th] = p + 2 + o + 1;
          S.dht_ok[tc * 4 + th] = 1;
          o += 17 + total;
        }
      } else if (m == 0xC0 || m == 0xC1) {
        if (s[0] != 8) {
          st = FFCV_SAMPLE_UNSUPPORTED;
          break;
        }
        S.H = rd16(s + 1);
        S.W = rd16(s + 3);
        S.ncomp = s[5];
        if (S.ncomp != 1 && S.ncomp != 3) {
          st = FFCV_SAMPLE_UNSUPPORTED;
          break;
        }
        S.hmax = S.vmax = 1;
        for (int c = 0; c < S.ncomp; c++) {
          S.cid[c] = s[6 + 3 * c];
          S.hs[c] = s[7 + 3 * c] >> 4;
          S.vs[c] = s[7 + 3 * c] & 15;
          S.tq[c] = s[8 + 3 * c] & 3;
          if (S.hs[c] < 1 || S.hs[c] > 4 || S.vs[c] < 1 || S.vs[c] > 4) st = FFCV_SAMPLE_UNSUPPORTED;
          S.hmax = max(S.hmax, S.hs[c]);
          S.vmax = max(S.vmax, S.vs[c]);
        }
        have_sof = 1;
      } else if (m >= 0xC2 && m <= 0xCF && m != 0xC4 && m != 0xC8 && m != 0xCC) {
        st = FFCV_SAMPLE_UNSUPPORTED;  // progressive / lossless / arithmetic
      } else if (m == 0xDD) {
        S.restart = rd16(s);
      } else if (m == 0xE0) {
        if (sl >= 5 && s[0] == 'J' && s[1] == 'F' && s[2] == 'I' && s[3] == 'F' && s[4] == 0) S.saw_jfif = 1;
      } else if (m == 0xEE) {
        if (sl >= 12 && s[0] == 'A' && s[1] == 'd' && s[2] == 'o' && s[3] == 'b' && s[4] == 'e') {
          S.saw_adobe = 1;
          S.adobe_transform = s[11];
        }
      } else if (m == 0xDA) {
        if (!have_sof) {
          st = FFCV_SAMPLE_BAD_MARKER;
          break;
        }
        int ns = s[0];
        if (ns != S.ncomp) {
          st = FFCV_SAMPLE_UNSUPPORTED;  // multi-scan sequential
          break;
        }
        int order[3];
        for (int i = 0; i < ns; i++) {
          int c = -1;
          for (int q = 0; q < S.ncomp; q++)
            if (S.cid[q] == s[1 + 2 * i]) c = q;
          if (c < 0) {
            st = FFCV_SAMPLE_BAD_MARKER;
            break;
          }
          order[i] = c;
          S.td[c] = s[2 + 2 * i] >> 4;
          S.ta[c] = s[2 + 2 * i] & 15;
          if (S.td[c] > 3 || S.ta[c] > 3) st = FFCV_SAMPLE_BAD_MARKER;
        }
        if (st) break;
        // blocks of one MCU in scan order
        int nb = 0;
        if (S.ncomp == 1) {
          S.blk_comp[0] = order[0];
          S.blk_dx[0] = S.blk_dy[0] = 0;
          nb = 1;
        } else {
          for (int i = 0; i < ns; i++) {
            int c = order[i];
            for (int yy = 0; yy < S.vs[c]; yy++)
              for (int xx = 0; xx < S.hs[c]; xx++) {
                if (nb < 10) {
                  S.blk_comp[nb] = c;
                  S.blk_dx[nb] = xx;
                  S.blk_dy[nb] = yy;
                }
                nb++;
              }
          }
        }
        if (nb > 10) {
          st = FFCV_SAMPLE_UNSUPPORTED;
          break;
        }
        S.bpm = nb;
        S.scan_off = p + (uint32_t)len;
        have_sos = 1;
      }
      p += (uint32_t)len;
    }
    if (st == FFCV_SAMPLE_OK) {
      if (S.restart) st = FFCV_SAMPLE_UNSUPPORTED;
      if (S.W != (int)smp.width || S.H != (int)smp.height) st = FFCV_SAMPLE_GEOMETRY;
      if ((uint32_t)S.W > a.max_w || (uint32_t)S.H > a.max_h) st = FFCV_SAMPLE_TOO_LARGE;
      for (int c = 0; c < S.ncomp && st == FFCV_SAMPLE_OK; c++) {
        if (!S.dqt_ok[S.tq[c]] || !S.dht_ok[S.td[c]] || !S.dht_ok[4 + S.ta[c]]) st = FFCV_SAMPLE_BAD_MARKER;
        if (S.hmax % S.hs[c] || S.vmax % S.vs[c]) st = FFCV_SAMPLE_UNSUPPORTED;
      }
    }
    if (st == FFCV_SAMPLE_OK) {
      if (S.ncomp == 3) {
        if (S.saw_jfif)
          S.color_rgb = 0;
        else if (S.saw_adobe)
          S.color_rgb = S.adobe_transform == 0;
        else
          S.color_rgb = S.cid[0] == 82 && S.cid[1] == 71 && S.cid[2] == 66;
      } else {
        S.color_rgb = 0;
      }
      uint64_t off_blocks = 0, off_plane = 0;
      if (S.ncomp == 1) {
        S.cw[0] = (S.W * S.hs[0] + S.hmax - 1) / S.hmax;
        S.ch[0] = (S.H * S.vs[0] + S.vmax - 1) / S.vmax;
        S.mcux = (S.cw[0] + 7) / 8;
        S.mcuy = (S.ch[0] + 7) / 8;
        S.bw[0] = S.mcux;
        S.bh[0] = S.mcuy;
        S.hs[0] = S.vs[0] = 1;  // non-interleaved scan: one block per MCU
        S.hmax = S.vmax = 1;
      } else {
        S.mcux = (S.W + 8 * S.hmax - 1) / (8 * S.hmax);
        S.mcuy = (S.H + 8 * S.vmax - 1) / (8 * S.vmax);
        for (int c = 0; c < S.ncomp; c++) {
          S.cw[c] = (S.W * S.hs[c] + S.hmax - 1) / S.hmax;
          S.ch[c] = (S.H * S.vs[c] + S.vmax - 1) / S.vmax;
          S.bw[c] = S.mcux * S.hs[c];
          S.bh[c] = S.mcuy * S.vs[c];
        }
      }
      for (int c = 0; c < S.ncomp; c++) {
        S.coff[c] = off_blocks;
        S.poff[c] = off_plane;
        off_blocks += (uint64_t)S.bw[c] * S.bh[c];
        off_plane += (uint64_t)S.bw[c] * S.bh[c] * 64;
      }
      S.nblocks = S.mcux * S.mcuy * S.bpm;
      if (off_blocks * 64 > a.coef_slot || off_plane > a.plane_slot) st = FFCV_SAMPLE_TOO_LARGE;
      if (MODE == JM_COEF && (uint64_t)S.nblocks > a.max_blocks) st = FFCV_SAMPLE_TOO_LARGE;
      // crop window in full-resolution pixels
      if (MODE == JM_RRC) {
        S.ri = a.crops[4 * k];
        S.rj = a.crops[4 * k + 1];
        S.rh = a.crops[4 * k + 2];
        S.rw = a.crops[4 * k + 3];
        if (S.rh <= 0 || S.rw <= 0 || S.ri < 0 || S.rj < 0 || S.ri + S.rh > S.H || S.rj + S.rw > S.W)
          st = FFCV_SAMPLE_GEOMETRY;
      } else {
        S.ri = 0;
        S.rj = 0;
        S.rh = S.H;
        S.rw = S.W;
      }
      if (MODE == JM_RRC && (uint64_t)S.rh * S.rw * 3 > a.roi_slot) st = FFCV_SAMPLE_TOO_LARGE;
      for (int c = 0; c < S.ncomp; c++) {
        int he = S.hmax / S.hs[c], ve = S.vmax / S.vs[c];
        int y0 = S.ri / ve - (ve == 2 ? 1 : 0), y1 = (S.ri + S.rh - 1) / ve + (ve == 2 ? 1 : 0);
        int x0 = S.rj / he - (he == 2 ? 1 : 0), x1 = (S.rj + S.rw - 1) / he + (he == 2 ? 1 : 0);
        y0 = max(y0, 0);
        x0 = max(x0, 0);
        y1 = min(y1, S.ch[c] - 1);
        x1 = min(x1, S.cw[c] - 1);
        if (MODE == JM_COEF) {
          y0 = x0 = 0;
          y1 = S.bh[c] * 8 - 1;
          x1 = S.bw[c] * 8 - 1;
        }
        S.wy0[c] = y0 >> 3;
        S.wy1[c] = y1 >> 3;
        S.wx0[c] = x0 >> 3;
        S.wx1[c] = x1 >> 3;
      }
    }
    S.status = st;
    S.first_marker = 0xFFFFFFFFu;
    S.any = 0;
  }
  __syncthreads();
  if (S.status != FFCV_SAMPLE_OK) {
    // zero-fill this sample's output and report
    if (MODE == JM_RRC) {
      uint64_t bytes = (uint64_t)a.p.out_h * a.p.out_w * 3 * (FP16 ? 2 : 1);
      uint8_t *o = (uint8_t *)a.out + a.out_stride * k;
      for (uint64_t i = t; i < bytes; i += JT) o[i] = 0;
    } else if (MODE == JM_FULL) {
      uint64_t bytes = (uint64_t)smp.height * smp.width * 3;
      uint8_t *o = (uint8_t *)a.out + a.out_stride * k;
      for (uint64_t i = t; i < bytes && i < a.out_stride; i += JT) o[i] = 0;
    }
    if (t == 0) a.status[k] = S.status;
    return;
  }

  // ------------------------------------------------------------- P1 ----
  STAMP(1);
  if (t < NTAB) {
    if (S.dht_ok[t]) {
      HuffTab &T = S.tab[t];
      const uint8_t *d = src + S.dht_off[t];
      int code = 0, kk = 0;
      for (int l = 1; l <= 16; l++) {
        int nl = d[l - 1];
        if (nl) {
          T.valoff[l] = kk - code;
          code += nl;
          kk += nl;
          T.maxcode[l] = code - 1;
        } else {
          T.maxcode[l] = -1;
          T.valoff[l] = 0;
        }
        code <<= 1;
      }
      T.maxcode[17] = 0x7fffffff;
      for (int i = 0; i < kk; i++) T.vals[i] = d[16 + i];
    }
  }
  if (t < 80) S.nat[t] = c_natural[t];
  __syncthreads();
  for (int i = t; i < NTAB * (1 << FAST_BITS); i += JT) {
    int ti = i >> FAST_BITS, v = i & ((1 << FAST_BITS) - 1);
    if (!S.dht_ok[ti]) continue;
    HuffTab &T = S.tab[ti];
    uint16_t e = 0;
    for (int l = 1; l <= FAST_BITS; l++) {
      int code = v >> (FAST_BITS - l);
      if (code <= T.maxcode[l]) {
        e = (uint16_t)((l << 8) | T.vals[(T.valoff[l] + code) & 0xff]);
        break;
      }
    }
    T.lut[v] = e;
  }
  for (int i = t; i < S.ncomp * 64; i += JT) {
    int c = i >> 6, zz = i & 63;  // zz: zigzag index in the DQT
    int tq = S.tq[c];
    const uint8_t *q = src + S.dqt_off[tq];
    int qv = S.dqt_prec[tq] ? rd16(q + 2 * zz) : q[zz];
    int n = c_natural[zz];
    S.qmul[c][n] = (int16_t)(((int64_t)qv * c_aanscales[n] + (1 << 11)) >> 12);
  }

  // zero the coefficient blocks of the window (P5 writes only nonzeros)
  int16_t *coef = a.coef + a.coef_slot * k;
  __syncthreads();
  for (int c = 0; c < S.ncomp; c++) {
    int wbw = S.wx1[c] - S.wx0[c] + 1, wbh = S.wy1[c] - S.wy0[c] + 1;
    int n16 = wbw * wbh * 8;  // 16-byte pieces
    for (int i = t; i < n16; i += JT) {
      int blk = i >> 3, piece = i & 7;
      int by = S.wy0[c] + blk / wbw, bx = S.wx0[c] + blk % wbw;
      uint4 zero = make_uint4(0, 0, 0, 0);
      *(uint4 *)(coef + (S.coff[c] + (uint64_t)by * S.bw[c] + bx) * 64 + piece * 8) = zero;
    }
  }

  // ------------------------------------------------------------- P2 ----
  STAMP(2);
  // entropy-coded segment: [scan_off, first marker)
  const uint32_t seg0 = S.scan_off;
  const uint32_t seglen = nbytes > seg0 ? nbytes - seg0 : 0;
  const uint32_t per = (seglen + JT - 1) / JT;
  const uint32_t c0 = seg0 + min(seglen, per * t), c1 = seg0 + min(seglen, per * (t + 1));
  {
    uint32_t fm = 0xFFFFFFFFu;
    for (uint32_t q = c0; q < c1; q++) {
      if (src[q] == 0xFF) {
        uint8_t nx = q + 1 < nbytes ? src[q + 1] : 0xD9;
        if (nx != 0x00) {
          fm = q;
          break;
        }
      }
    }
    if (fm != 0xFFFFFFFFu) atomicMin(&S.first_marker, fm);
  }
  __syncthreads();
  const uint32_t seg_end = S.first_marker == 0xFFFFFFFFu ? nbytes : S.first_marker;
  uint32_t keep = 0;
  for (uint32_t q = c0; q < min(c1, seg_end); q++)
    keep += !(src[q] == 0x00 && q > seg0 && src[q - 1] == 0xFF);
  uint32_t wpos = wg_exscan_u32(keep, S.scan_tmp);
  uint8_t *ds = a.dstuff + a.dstuff_slot * k;
  for (uint32_t q = c0; q < min(c1, seg_end); q++) {
    if (!(src[q] == 0x00 && q > seg0 && src[q - 1] == 0xFF)) ds[wpos++] = src[q];
  }
  if (t == JT - 1) {
    S.dlen = wpos;
    for (int i = 0; i < 16; i++) ds[wpos + i] = 0;  // zero fill, as libjpeg past a marker
  }
  __syncthreads();
  const uint32_t dlen = S.dlen;
  const uint32_t *words = (const uint32_t *)ds;
  const uint32_t nwords = (dlen + 3) / 4;
  const uint32_t total_bits = dlen * 8;

  // ------------------------------------------------------------- P3 ----
  STAMP(3);
  if (t == 0) {
    // at least ~192 bits per lane so resynchronisation is cheap relative to work
    uint32_t nthr = (total_bits + 191) / 192;
    nthr = max(1u, min(nthr, (uint32_t)JT));
    uint32_t cb = (total_bits + nthr - 1) / nthr;
    S.nthr = (int)nthr;
    S.chunk_bits = cb;
  }
  __syncthreads();
  const int nthr = S.nthr;
  const uint32_t cbits = S.chunk_bits;
  const bool active = t < nthr;
  const uint32_t my_end = active ? (t == nthr - 1 ? total_bits : min(total_bits, (t + 1) * cbits)) : 0;
  DecState g;
  g.pos = active ? t * cbits : 0;
  g.z = 0;
  g.ph = 0;
  uint32_t my_cnt = 0;
  int32_t my_dc[3] = {0, 0, 0};
  DecState e = g;
  if (active) e = decode_range<false>(S, words, nwords, g, my_end, &my_cnt, my_dc, 0, nullptr, nullptr);
  for (int round = 0; round < JT + 1; round++) {
    S.e_pos[t] = e.pos;
    S.e_z[t] = (uint8_t)e.z;
    S.e_ph[t] = (uint8_t)e.ph;
    __syncthreads();
    bool changed = false;
    DecState ng = g;
    if (active && t > 0) {
      ng.pos = S.e_pos[t - 1];
      ng.z = S.e_z[t - 1];
      ng.ph = S.e_ph[t - 1];
      changed = ng.pos != g.pos || ng.z != g.z || ng.ph != g.ph;
    }
    int anyc = __syncthreads_or(changed);
    if (!anyc) {
      if (a.dbg && t == 0) a.dbg[(uint64_t)k * 16 + 12] = (uint64_t)round;
      break;
    }
    if (changed) {
      g = ng;
      my_dc[0] = my_dc[1] = my_dc[2] = 0;
      if (g.pos >= my_end) {  // previous unit already crossed my whole range
        e = g;
        my_cnt = 0;
      } else {
        e = decode_range<false>(S, words, nwords, g, my_end, &my_cnt, my_dc, 0, nullptr, nullptr);
      }
    }
  }
  if (!active) {
    my_cnt = 0;
    my_dc[0] = my_dc[1] = my_dc[2] = 0;
  }

  // ------------------------------------------------------------- P4 ----
  STAMP(4);
  if (a.dbg && t == 0) a.dbg[(uint64_t)k * 16 + 13] = (uint64_t)nthr;
  const uint32_t blk_base = wg_exscan_u32(my_cnt, S.scan_tmp);
  int32_t pred[3];
  for (int c = 0; c < 3; c++) pred[c] = wg_exscan_i32(my_dc[c], S.scan_tmp2[c]);
  if (active) {
    int64_t cur = g.z == 0 ? (int64_t)blk_base : (int64_t)blk_base - 1;
    if (cur < 0 || (cur % S.bpm) != g.ph) S.any = 1;  // inconsistent stream
  }
  __syncthreads();
  if (S.any) {
    if (t == 0) a.status[k] = FFCV_SAMPLE_CORRUPT;
  }

  // ------------------------------------------------------------- P5 ----
  STAMP(5);
  if (active && g.pos < my_end) {
    int64_t cur = g.z == 0 ? (int64_t)blk_base : (int64_t)blk_base - 1;
    if (cur >= 0)
      decode_range<true>(S, words, nwords, g, my_end, nullptr, nullptr, cur, pred, coef);
  }
  __syncthreads();

  if (MODE == JM_COEF) {
    int16_t *o = (int16_t *)a.out + a.out_stride / 2 * k;
    for (int64_t b = t; b < S.nblocks; b += JT) {
      int64_t m = b / S.bpm;
      int ph = (int)(b - m * S.bpm);
      int my = (int)(m / S.mcux), mx = (int)(m - (int64_t)my * S.mcux);
      int c = S.blk_comp[ph];
      int bx = mx * S.hs[c] + S.blk_dx[ph], by = my * S.vs[c] + S.blk_dy[ph];
      const uint4 *sp = (const uint4 *)(coef + (S.coff[c] + (uint64_t)by * S.bw[c] + bx) * 64);
      uint4 *dp = (uint4 *)(o + b * 64);
      for (int i = 0; i < 8; i++) dp[i] = sp[i];
    }
    if (t == 0 && !S.any) a.status[k] = FFCV_SAMPLE_OK;
    return;
  }

  // ------------------------------------------------------------- P6 ----
  STAMP(6);
  uint8_t *planes = a.planes + a.plane_slot * k;
  for (int c = 0; c < S.ncomp; c++) {
    int wbw = S.wx1[c] - S.wx0[c] + 1, wbh = S.wy1[c] - S.wy0[c] + 1;
    int stride = S.bw[c] * 8;
    for (int i = t; i < wbw * wbh; i += JT) {
      int by = S.wy0[c] + i / wbw, bx = S.wx0[c] + i % wbw;
      const int16_t *cp = coef + (S.coff[c] + (uint64_t)by * S.bw[c] + bx) * 64;
      int16_t blk[64];
#pragma unroll
      for (int p8 = 0; p8 < 8; p8++) *(uint4 *)(blk + p8 * 8) = ((const uint4 *)cp)[p8];
      idct_ifast_block(blk, S.qmul[c], planes + S.poff[c] + (uint64_t)by * 8 * stride + bx * 8, stride);
    }
  }
  __syncthreads();

  // ------------------------------------------------------------- P7 ----
  STAMP(7);
  const int rh = S.rh, rw = S.rw, ri = S.ri, rj = S.rj;
  uint8_t *roi;
  uint64_t roi_step;
  if (MODE == JM_FULL) {
    roi = (uint8_t *)a.out + a.out_stride * k;
    roi_step = (uint64_t)S.W * 3;
  } else {
    roi = a.roi + a.roi_slot * k;
    roi_step = (uint64_t)rw * 3;
  }
  for (int i = t; i < rh * rw; i += JT) {
    int y = i / rw, x = i - y * rw;
    int Y = y + ri, X = x + rj;
    int v[3];
    if (S.ncomp == 1) {
      int g0 = planes[S.poff[0] + (uint64_t)Y * (S.bw[0] * 8) + X];
      v[0] = v[1] = v[2] = g0;
    } else {
      int s3[3];
      for (int c = 0; c < 3; c++)
        s3[c] = upsample_at(planes + S.poff[c], S.bw[c] * 8, S.cw[c], S.ch[c], S.hmax / S.hs[c],
                            S.vmax / S.vs[c], Y, X);
      if (S.color_rgb) {
        v[0] = s3[0];
        v[1] = s3[1];
        v[2] = s3[2];
      } else {
        ycc_rgb(s3[0], s3[1], s3[2], v);
      }
    }
    uint8_t *o = roi + (uint64_t)y * roi_step + (uint64_t)x * 3;
    o[0] = (uint8_t)v[0];
    o[1] = (uint8_t)v[1];
    o[2] = (uint8_t)v[2];
  }
  if (MODE == JM_FULL) {
    if (t == 0 && !S.any) a.status[k] = FFCV_SAMPLE_OK;
    return;
  }
  __syncthreads();

  // ------------------------------------------------------------- P8 ----
  STAMP(8);
  __shared__ uint16_t s_lut[FP16 ? 768 : 1];
  if (FP16) {
    for (int i = t; i < 768; i += JT) s_lut[i] = a.p.lut[i];
    __syncthreads();
  }
  RoiScratch rs{roi, roi_step};
  ResizePlan P = make_plan(rw, rh, a.p.out_w, a.p.out_h);
  Epilogue ep;
  ep.out_h = a.p.out_h;
  ep.out_w = a.p.out_w;
  ep.cut_size = a.cut ? a.p.cutout_size : 0;
  ep.cut_y = a.cut ? a.cut[2 * k] : 0;
  ep.cut_x = a.cut ? a.cut[2 * k + 1] : 0;
  ep.flip = a.flips ? a.flips[k] : 0;
  ep.cut_before_flip = a.p.cutout_fill[3];
  ep.fill[0] = a.p.cutout_fill[0];
  ep.fill[1] = a.p.cutout_fill[1];
  ep.fill[2] = a.p.cutout_fill[2];
  const int npx = a.p.out_h * a.p.out_w;
  char *ob = (char *)a.out + a.out_stride * k;
  for (int px = t; px < npx; px += JT) {
    int dy = px / a.p.out_w, dx = px - dy * a.p.out_w;
    int v[3];
    if (ep.in_cut(dy, dx)) {
      v[0] = ep.fill[0];
      v[1] = ep.fill[1];
      v[2] = ep.fill[2];
    } else {
      resize_pixel(P, rs, dy, ep.src_x(dx), v);
    }
    if (FP16) {
      uint16_t *o = (uint16_t *)ob + (uint64_t)px * 3;
      o[0] = s_lut[v[0] * 3];
      o[1] = s_lut[v[1] * 3 + 1];
      o[2] = s_lut[v[2] * 3 + 2];
    } else {
      uint8_t *o = (uint8_t *)ob + (uint64_t)px * 3;
      o[0] = (uint8_t)v[0];
      o[1] = (uint8_t)v[1];
      o[2] = (uint8_t)v[2];
    }
  }
  STAMP(9);
  if (t == 0 && !S.any) a.status[k] = FFCV_SAMPLE_OK;
}

// ---------------------------------------------------------------- ctx -----
struct ffcv_jpeg_ctx {
  uint64_t *dbg;
  int max_batch;
  uint32_t max_h, max_w;
  uint64_t max_bytes;
  uint8_t *dstuff;
  uint64_t dstuff_slot;
  int16_t *coef;
  uint64_t coef_slot;
  uint8_t *planes;
  uint64_t plane_slot;
  uint8_t *roi;
  uint64_t roi_slot;
};

static uint64_t align_up(uint64_t x, uint64_t a) { return (x + a - 1) / a * a; }

extern "C" {

int ffcv_jpeg_create(ffcv_jpeg_ctx **out, int max_batch, uint32_t max_height, uint32_t max_width,
                     uint64_t max_bytes) {
  if (!out || max_batch <= 0 || max_height == 0 || max_width == 0 || max_height > 65535 ||
      max_width > 65535 || max_bytes == 0) {
    ffcv::set_error("ffcv_jpeg_create: invalid arguments");
    return FFCV_EINVAL;
  }
  ffcv_jpeg_ctx *c = new ffcv_jpeg_ctx();
  c->max_batch = max_batch;
  c->max_h = max_height;
  c->max_w = max_width;
  c->max_bytes = max_bytes;
  // blocks of all components, MCU padded (hmax, vmax <= 4)
  uint64_t bw = (max_width + 7) / 8 + 4, bh = (max_height + 7) / 8 + 4;
  uint64_t nblk = 3 * bw * bh;
  c->dstuff_slot = align_up(max_bytes + 64, 256);
  c->coef_slot = align_up(nblk * 64, 128);         // int16 elements
  c->plane_slot = align_up(nblk * 64, 256);        // bytes
  c->roi_slot = align_up((uint64_t)max_height * max_width * 3, 256);
  hipError_t e;
  if ((e = hipMalloc(&c->dstuff, c->dstuff_slot * max_batch)) != hipSuccess ||
      (e = hipMalloc(&c->coef, c->coef_slot * 2 * max_batch)) != hipSuccess ||
      (e = hipMalloc(&c->planes, c->plane_slot * max_batch)) != hipSuccess ||
      (e = hipMalloc(&c->roi, c->roi_slot * max_batch)) != hipSuccess) {
    int rc = ffcv::check_hip(e, "ffcv_jpeg_create: hipMalloc");
    (void)hipFree(c->dstuff);
    (void)hipFree(c->coef);
    (void)hipFree(c->planes);
    (void)hipFree(c->roi);
    delete c;
    return rc;
  }
  *out = c;
  return FFCV_OK;
}

// Diagnostic hook (not in the public header): per-image phase stamps
// (wall_clock64, 100 MHz) into dbg[B][16]; NULL disables.
int ffcv_jpeg_set_debug(ffcv_jpeg_ctx *c, uint64_t *dbg) {
  if (!c) return FFCV_EINVAL;
  c->dbg = dbg;
  return FFCV_OK;
}

int ffcv_jpeg_destroy(ffcv_jpeg_ctx *c) {
  if (!c) return FFCV_OK;
  (void)hipFree(c->dstuff);
  (void)hipFree(c->coef);
  (void)hipFree(c->planes);
  (void)hipFree(c->roi);
  delete c;
  return FFCV_OK;
}

static JpegArgs make_args(ffcv_jpeg_ctx *c, const uint8_t *base, const ffcv_sample *samples, int32_t *status) {
  JpegArgs a = {};
  a.base = base;
  a.samples = samples;
  a.status = status;
  a.dstuff = c->dstuff;
  a.dstuff_slot = c->dstuff_slot;
  a.coef = c->coef;
  a.coef_slot = c->coef_slot;
  a.planes = c->planes;
  a.plane_slot = c->plane_slot;
  a.roi = c->roi;
  a.roi_slot = c->roi_slot;
  a.max_h = c->max_h;
  a.max_w = c->max_w;
  a.dbg = c->dbg;
  return a;
}

static int check_common(const char *fn, ffcv_jpeg_ctx *c, const uint8_t *base, const ffcv_sample *samples,
                        int batch, const void *out, const int32_t *status) {
  if (!c || !base || !samples || !out || !status || batch < 0) {
    ffcv::set_error("%s: invalid arguments", fn);
    return FFCV_EINVAL;
  }
  if (batch > c->max_batch) {
    ffcv::set_error("%s: batch %d exceeds ctx max_batch %d", fn, batch, c->max_batch);
    return FFCV_EINVAL;
  }
  return FFCV_OK;
}

int ffcv_jpeg_rrc_batch(ffcv_jpeg_ctx *c, void *stream, const uint8_t *base, const ffcv_sample *samples,
                        int batch, const int32_t *crops, const int32_t *cutout_yx, const uint8_t *flips,
                        const ffcv_rrc_params *p, void *out, int32_t *status) {
  int rc = check_common("ffcv_jpeg_rrc_batch", c, base, samples, batch, out, status);
  if (rc) return rc;
  if (!p || !crops || p->out_h <= 0 || p->out_w <= 0) {
    ffcv::set_error("ffcv_jpeg_rrc_batch: invalid params");
    return FFCV_EINVAL;
  }
  if (batch == 0) return FFCV_OK;
  JpegArgs a = make_args(c, base, samples, status);
  a.crops = crops;
  a.cut = cutout_yx;
  a.flips = flips;
  a.p = *p;
  a.out = out;
  const bool fp16 = p->lut != nullptr;
  uint64_t dense = (uint64_t)p->out_h * p->out_w * 3 * (fp16 ? 2 : 1);
  a.out_stride = p->out_stride ? p->out_stride : dense;
  if (fp16)
    hipLaunchKernelGGL((jpeg_kernel<JM_RRC, true>), dim3(batch), dim3(JT), 0, ffcv::as_stream(stream), a);
  else
    hipLaunchKernelGGL((jpeg_kernel<JM_RRC, false>), dim3(batch), dim3(JT), 0, ffcv::as_stream(stream), a);
  FFCV_LAUNCH_CHECK("jpeg_kernel<RRC>");
  return FFCV_OK;
}

int ffcv_jpeg_decode_batch(ffcv_jpeg_ctx *c, void *stream, const uint8_t *base, const ffcv_sample *samples,
                           int batch, uint8_t *out, uint64_t out_stride, int32_t *status) {
  int rc = check_common("ffcv_jpeg_decode_batch", c, base, samples, batch, out, status);
  if (rc) return rc;
  if (!out_stride) {
    ffcv::set_error("ffcv_jpeg_decode_batch: out_stride must be > 0");
    return FFCV_EINVAL;
  }
  if (batch == 0) return FFCV_OK;
  JpegArgs a = make_args(c, base, samples, status);
  a.out = out;
  a.out_stride = out_stride;
  hipLaunchKernelGGL((jpeg_kernel<JM_FULL, false>), dim3(batch), dim3(JT), 0, ffcv::as_stream(stream), a);
  FFCV_LAUNCH_CHECK("jpeg_kernel<FULL>");
  return FFCV_OK;
}

int ffcv_jpeg_coefficients_batch(ffcv_jpeg_ctx *c, void *stream, const uint8_t *base,
                                 const ffcv_sample *samples, int batch, int16_t *coefs, uint64_t max_blocks,
                                 int32_t *status) {
  int rc = check_common("ffcv_jpeg_coefficients_batch", c, base, samples, batch, coefs, status);
  if (rc) return rc;
  if (batch == 0) return FFCV_OK;
  JpegArgs a = make_args(c, base, samples, status);
  a.out = coefs;
  a.out_stride = max_blocks * 64 * 2;
  a.max_blocks = max_blocks;
  hipLaunchKernelGGL((jpeg_kernel<JM_COEF, false>), dim3(batch), dim3(JT), 0, ffcv::as_stream(stream), a);
  FFCV_LAUNCH_CHECK("jpeg_kernel<COEF>");
  return FFCV_OK;
}

}  // extern "C"
