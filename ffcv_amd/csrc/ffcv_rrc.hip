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
#include "diag_hooks.h"

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
static_assert(RRC_THREADS == 256, "rrc_band's row staging and walk assume four waves per workgroup");
#ifndef RRC_BAND
#define RRC_BAND 16  // output rows per workgroup
#endif
#ifndef RRC_STAGE_ROWS
#define RRC_STAGE_ROWS 5  // rows a wave stages per batch of loads in flight (2 x 16 B per lane each)
#endif
#ifndef RRC_LDS_BYTES
#define RRC_LDS_BYTES 30464  // source-row stage: the most that keeps 5 workgroups per CU with the LUT and tap tables (28 KB: 1% slower, 24 KB: 15% slower)
#endif

// Crop rows staged in LDS.  LDS row y - r0 holds the 16-byte aligned chunks
// covering crop row y, so the row's first byte sits at its alignment
// offset ((lead + (y - r0) * step) & 15) inside the LDS row.
struct LdsSrc {
  const uint8_t *p;
  int pitch, lead, stepmod, r0;
  FFCV_DEV const uint8_t *row(int y) const {
    const int r = y - r0;
    return p + r * pitch + ((lead + r * stepmod) & 15);
  }
  FFCV_DEV int at(int y, int x, int c) const { return row(y)[x * 3 + c]; }
  FFCV_DEV const uint8_t *pix(int y, int x) const { return row(y) + x * 3; }
};

// One workgroup per band of RRC_BAND output rows of one image.
//   Staging: the band's source rows of the crop (band_rows) are copied into
//   LDS with 16-byte aligned global loads (an aligned chunk holding at least
//   one byte of the row never crosses a page, so the aligned-down/up edges
//   are safe), so each source byte is read from HBM once per band and every
//   tap after that is an LDS read.  Bands whose rows do not fit
//   RRC_LDS_BYTES read their taps from global memory instead.
//   Linear fast path (every crop upscaled along some axis, OpenCV's
//   "area-mode" linear with the SSE2 vertical body on every element): each
//   thread owns four adjacent output columns and walks a slice of the band's
//   rows, keeping the two source rows' horizontal sums in registers; the four
//   pixels leave as one 12-byte (u8) or three 8-byte (fp16) stores, so a wave
//   writes one contiguous run of the output row.
//   Otherwise (area downscale, copy, widths not a multiple of 4): the
//   per-pixel restatement, over the staged rows when they fit.
// rrc_taps_kernel's table: entries per image (even: 16-byte quads stay
// aligned): linear plans use out_w + out_h (columns, then rows), area plans at
// scales < 2 two per column (a 16-byte record: first tap, three weights)
#define RAW_TAPS(p) ((max((p).out_w + (p).out_h, 2 * (p).out_w) + 1) & ~1)
// an area plan whose column records rrc_taps_kernel writes: both scales < 2
// (scale_x = 1 / (dw / sw) < 2 exactly when sw < 2 dw)
FFCV_HD bool area_walk_plan(const ResizePlan &P) { return P.kind == 2 && P.sw < 2 * P.dw && P.sh < 2 * P.dh; }
#ifndef RRC_AREA_MAGIC
#define RRC_AREA_MAGIC 1  // 0: the area walk rounds by v_rndne + v_cvt + v_med3 (A/B builds)
#endif
#ifndef RRC_WPE
#define RRC_WPE 5  // waves per SIMD the raw kernel is compiled for (5 workgroups per CU by LDS)
#endif
// LDS of one band
template <bool FP16>
struct RrcLds {
  uint16_t lut[FP16 ? 768 : 1];
  uint4 src[RRC_LDS_BYTES / 16];
  uint4 rt[RRC_BAND];  // linear row taps: {ra, rb, c0 << 8, c1 << 8}
  AreaTaps at[RRC_BAND];
};

// One band of RRC_BAND output rows of image k.  Every barrier is reached by
// all threads; thread-level returns follow the last one.
template <bool FP16>
FFCV_DEV void rrc_band(const uint8_t *__restrict__ base, const ffcv_sample *__restrict__ samples,
                       const int32_t *__restrict__ crops, const int32_t *__restrict__ cut,
                       const uint8_t *__restrict__ flips, const ffcv_rrc_params &p, uint64_t stride,
                       void *__restrict__ out, const int k, const int band, RrcLds<FP16> &S,
                       const ResizePlan *__restrict__ plans, const uint2 *__restrict__ taps) {
  uint16_t *s_lut = S.lut;
  uint4 *s_src = S.src;
  uint4 *s_rt = S.rt;
  AreaTaps *s_at = S.at;
  const int t = threadIdx.x;
  const ffcv_sample s = samples[k];
  if (FP16) {
    for (int i = t; i < 768; i += RRC_THREADS) s_lut[i] = p.lut[i];
  }
  if (s.mode != 1) return;
  const int oy0 = band * RRC_BAND, oy1 = min(p.out_h, oy0 + RRC_BAND);
  if (oy0 >= p.out_h) return;
  const int ci = crops[4 * k], cj = crops[4 * k + 1], chh = crops[4 * k + 2], cww = crops[4 * k + 3];
  GlobalSrc src{base + s.offset + ((uint64_t)ci * s.width + cj) * 3, (uint64_t)s.width * 3};
  // the image's plan and linear taps from rrc_taps_kernel when the caller gave
  // a workspace (computed once per image, not in each of its band workgroups:
  // the f64 plan and four column taps per thread were a third of this
  // kernel's instructions, profiles/r5c_c5parts.txt)
  const uint2 *itaps = taps ? taps + (uint64_t)k * RAW_TAPS(p) : nullptr;
  ResizePlan P = plans ? plans[k] : make_plan(cww, chh, p.out_w, p.out_h);
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
  // The linear walk's column taps (flip applied, 32 bytes per thread quad),
  // loaded before the band's staging so their latency hides under it (after
  // it, every workgroup waited ~1 us for them: 28 ns per image)
  uint4 tq0 = make_uint4(0, 0, 0, 0), tq1 = tq0;
  {
    int tpg = 64;
    while (tpg < (out_w >> 2)) tpg <<= 1;
    const int qq = t & (tpg - 1);
    // (rrc_taps_kernel writes these entries for linear plans only: an area
    // crop's table holds the area walk's column records, read there)
    if (itaps && P.kind == 3 && qq < (out_w >> 2)) {
      tq0 = *(const uint4 *)(itaps + 4 * qq);
      tq1 = *(const uint4 *)(itaps + 4 * qq + 2);
    }
  }

  RRC_STOP_AT(1, p.cutout_fill[3] != 77);  // diagnostics: the band's set-up only
  // ---- stage the band's source rows into LDS
  int r0, r1;
  band_rows(P, oy0, oy1, &r0, &r1);
  const uint64_t row0 = (uint64_t)(uintptr_t)src.p + (uint64_t)r0 * src.step;
  const int nrows = r1 - r0 + 1;
  const int nch = (15 + P.sw * 3 + 15) >> 4;  // 16-byte chunks per LDS row (any alignment)
  const bool staged = nrows * nch * 16 <= RRC_LDS_BYTES;
  LdsSrc L{(const uint8_t *)s_src, nch * 16, (int)(row0 & 15), (int)(src.step & 15), r0};
  if (staged) {
    // wave w copies rows w, w + 4, ...; lane l the row's 16-byte chunks l and
    // l + 64: the row address and its chunk count are wave-uniform (scalar),
    // a lane's chunk offset is fixed, and a wave has up to RRC_STAGE_ROWS
    // rows' loads in flight before its LDS writes
    const int wv = __builtin_amdgcn_readfirstlane(t >> 6), ln = t & 63;  // (wv scalar: row addresses in SGPRs)
    // (a lane that loads nothing keeps the registers' previous contents: its
    // LDS write is skipped too; zeroing them cost 8 moves per row)
    typedef uint32_t sx4_t __attribute__((ext_vector_type(4)));
    sx4_t v[RRC_STAGE_ROWS][2] = {};
    for (int cg = 0; cg < nch; cg += 128)  // (one pass for rows up to 2 KB: crops up to 677 px wide)
      for (int rb0 = wv; rb0 < nrows; rb0 += (RRC_THREADS / 64) * RRC_STAGE_ROWS) {
#pragma unroll
        for (int q = 0; q < RRC_STAGE_ROWS; q++) {
          const int r = rb0 + (RRC_THREADS / 64) * q;
          const uint64_t ra = row0 + (uint64_t)r * src.step;
          // chunks holding bytes of this row (none past the dataset's end)
          const int lim = r < nrows ? (int)(((ra & 15) + 3 * (uint64_t)P.sw + 15) >> 4) - cg : 0;
          // (a global-address-space pointer: global_load, not flat_load --
          // a flat load also counts in lgkmcnt, so every LDS wait would wait
          // for it too)
          typedef const __attribute__((address_space(1))) uint32_t gu32_t;
          gu32_t *rp = (gu32_t *)(uintptr_t)(ra & ~(uint64_t)15) + 4 * cg;
          if (ln < lim) v[q][0] = (sx4_t){rp[4 * ln], rp[4 * ln + 1], rp[4 * ln + 2], rp[4 * ln + 3]};
          if (ln + 64 < lim) v[q][1] = (sx4_t){rp[4 * ln + 256], rp[4 * ln + 257], rp[4 * ln + 258], rp[4 * ln + 259]};
        }
#pragma unroll
        for (int q = 0; q < RRC_STAGE_ROWS; q++) {
          const int r = rb0 + (RRC_THREADS / 64) * q;
          const uint64_t ra = row0 + (uint64_t)r * src.step;
          const int lim = r < nrows ? (int)(((ra & 15) + 3 * (uint64_t)P.sw + 15) >> 4) - cg : 0;
          if (ln < lim) s_src[r * nch + cg + ln] = __builtin_bit_cast(uint4, v[q][0]);
          if (ln + 64 < lim) s_src[r * nch + cg + ln + 64] = __builtin_bit_cast(uint4, v[q][1]);
        }
      }
  }
  if (P.kind == 3 && !itaps && t < oy1 - oy0) {  // clamped source rows, weights << 8: no per-row clamps in the walk
    const LinTap l = lin_tap(P.scale_y, P.inv_y, P.sh, oy0 + t);
    s_rt[t] = make_uint4((uint32_t)min(max(l.s, 0), P.sh - 1), (uint32_t)min(max(l.s + 1, 0), P.sh - 1),
                         ((uint32_t)l.c0 & 0xfffu) << 8, ((uint32_t)l.c1 & 0xfffu) << 8);
  }
  if (P.kind == 2 && t < oy1 - oy0) s_at[t] = area_taps(P.sh, P.scale_y, oy0 + t);
  __syncthreads();
  RRC_STOP_AT(2, p.cutout_fill[3] != 77);  // diagnostics: set-up + staging

  const bool aligned4 = ((((uintptr_t)out) | stride) & 3) == 0;
  const int nq = out_w >> 2;  // column quads
  if (staged && (out_w & 3) == 0 && nq <= RRC_THREADS && aligned4 &&
      ((P.kind == 3 && P.vec_end == 3 * out_w) || P.kind == 2)) {
    // row groups: tpg threads (a power of two >= nq, >= 64) per group, each
    // group walks its own slice of the band's rows
    int tpg = 64;
    while (tpg < nq) tpg <<= 1;
    const int groups = RRC_THREADS / tpg;
    const int per = (oy1 - oy0 + groups - 1) / groups;
    const int g = t / tpg, q = t - g * tpg;
    // (a row group is whole waves, tpg >= 64: its rows are wave-uniform, so
    // the per-row cutout range test is scalar)
    const int gy0 = __builtin_amdgcn_readfirstlane(oy0 + g * per);
    const int gy1 = __builtin_amdgcn_readfirstlane(min(oy1, gy0 + per));
    if (q >= nq || gy0 >= gy1) return;
    const int dx0 = 4 * q;
    // cutout: the columns of this thread's quad inside the square (bit j =
    // column dx0 + j; flip-aware), tested once; rows test their own range
    uint32_t cmask = 0;
#pragma unroll
    for (int j = 0; j < 4; j++) cmask |= ep.in_cut(ep.cut_y, dx0 + j) ? 1u << j : 0u;
    // one 12-byte (u8) or three 8-byte (fp16) stores of the quad's pixels
    auto put = [&](int dy, int v[12]) {
      if (cmask && dy >= ep.cut_y && dy < ep.cut_y + ep.cut_size) {
#pragma unroll
        for (int j = 0; j < 4; j++)
          if ((cmask >> j) & 1) {
            v[3 * j] = ep.fill[0];
            v[3 * j + 1] = ep.fill[1];
            v[3 * j + 2] = ep.fill[2];
          }
      }
      const uint64_t px = (uint64_t)dy * out_w + dx0;
      if (FP16) {  // 24-byte group, 8-byte aligned (dx0 % 4 == 0)
        uint32_t h[12];
#pragma unroll
        for (int i = 0; i < 12; i++) h[i] = s_lut[v[i] * 3 + i % 3];
        uint2 *o64 = (uint2 *)((uint16_t *)o + px * 3);
        o64[0] = make_uint2(h[0] | (h[1] << 16), h[2] | (h[3] << 16));
        o64[1] = make_uint2(h[4] | (h[5] << 16), h[6] | (h[7] << 16));
        o64[2] = make_uint2(h[8] | (h[9] << 16), h[10] | (h[11] << 16));
      } else {  // 12-byte group, 4-byte aligned
        typedef uint32_t u32x3 __attribute__((ext_vector_type(3)));
        u32x3 w;
        w.x = v[0] | (v[1] << 8) | (v[2] << 16) | (v[3] << 24);
        w.y = v[4] | (v[5] << 8) | (v[6] << 16) | (v[7] << 24);
        w.z = v[8] | (v[9] << 8) | (v[10] << 16) | (v[11] << 24);
        // streaming output: non-temporal (measured +2% over plain stores; 16-byte
        // aligned stores of 4-lane groups exchanged by DPP measured the same)
        __builtin_nontemporal_store(w, (u32x3 *)((uint8_t *)o + px * 3));
      }
    };
    if (P.kind == 2) {  // ResizeArea_Invoker: column taps once per thread, row taps from LDS
      if (area_walk_plan(P)) {
        // Scales in [1, 2): a destination index takes at most 3 consecutive
        // source indices, so a fixed 3-tap horizontal body with zero weights
        // past `hi` is exact (x + S * 0.f == x for the non-negative sums
        // here).  buf of a source row (the horizontal sums)
        // does not depend on the destination row: each destination row dy
        // sums its source rows lo..hi in ascending order (sum = w(lo) * B(lo),
        // then sum += w(r) * B(r): the reference's order), and consecutive
        // rows share at most their boundary source row, so one cached row of
        // sums (Hc, source row cr) covers the reuse (any other reuse
        // recomputes, exactly).  The rows are wave-uniform (a row group is
        // whole waves): the loop bounds and the cache test are scalar.
        int xo[4];  // the first tap pixel's byte offset in a row
        float wx[4][3];
        if (itaps) {  // rrc_taps_kernel's column records (flip applied): one 16-byte load per column
#pragma unroll
          for (int j = 0; j < 4; j++) {
            const uint4 e = *(const uint4 *)(itaps + 2 * (dx0 + j));
            xo[j] = 3 * (int)e.x;
            wx[j][0] = ffcv_u2f_bits(e.y);
            wx[j][1] = ffcv_u2f_bits(e.z);
            wx[j][2] = ffcv_u2f_bits(e.w);
          }
        } else {
#pragma unroll
          for (int j = 0; j < 4; j++) {
            const AreaTaps tx = area_taps(P.sw, P.scale_x, ep.src_x(dx0 + j));
            xo[j] = 3 * tx.lo;
#pragma unroll
            for (int k = 0; k < 3; k++) wx[j][k] = tx.lo + k <= tx.hi ? tx.w(tx.lo + k) : 0.f;
          }
        }
        RRC_STOP_AT(4, p.cutout_fill[3] != 77);  // diagnostics: + the area walk's column taps
        // A column's three tap pixels lo, lo + 1, lo + 2 are 9 consecutive
        // bytes: three ALIGNED 4-byte LDS reads cover them at any alignment
        // and v_alignbyte shifts them into place (bytes at fixed positions,
        // converted by v_cvt_f32_ubyte0-3).  Misaligned LDS reads (the 2- and
        // 4-byte reads the compiler forms from adjacent byte reads) made this
        // walk ~5x slower per pixel than the linear one.  A tap past hi has
        // weight 0 and reads a byte of the staged rows or the LDS that
        // follows them (finite: 0 * x == 0).
        auto hsum = [&](int r, float B[12]) {
          const uint8_t *row = L.row(r);
#pragma unroll
          for (int j = 0; j < 4; j++) {
            const uint8_t *q = row + xo[j];
            const uint32_t *qa = (const uint32_t *)__builtin_align_down(q, 4);
            const uint32_t sh = (uint32_t)(q - (const uint8_t *)qa);  // 0..3
            const uint32_t d0 = qa[0], d1 = qa[1], d2 = qa[2];
            uint32_t e[3];
            e[0] = __builtin_amdgcn_alignbyte(d1, d0, sh);
            e[1] = __builtin_amdgcn_alignbyte(d2, d1, sh);
            e[2] = d2 >> (8 * sh);
#pragma unroll
            for (int c = 0; c < 3; c++) {
              float b = 0.f;
#pragma unroll
              for (int k = 0; k < 3; k++) {
                const int i = 3 * k + c;
                b = b + (float)((e[i >> 2] >> (8 * (i & 3))) & 0xffu) * wx[j][k];
              }
              B[3 * j + c] = b;
            }
          }
        };
        int cr = -1;
        float Hc[12];
#pragma unroll
        for (int i = 0; i < 12; i++) Hc[i] = 0.f;
        for (int dy = gy0; dy < gy1; dy++) {
          const AreaTaps ty = s_at[dy - oy0];
          float S[12];
          for (int r = ty.lo; r <= ty.hi; r++) {
            float H[12];
            if (r == cr) {
#pragma unroll
              for (int i = 0; i < 12; i++) H[i] = Hc[i];
            } else {
              hsum(r, H);
            }
            const float w = ty.w(r);
            if (r == ty.lo) {
#pragma unroll
              for (int i = 0; i < 12; i++) S[i] = w * H[i];
            } else {
#pragma unroll
              for (int i = 0; i < 12; i++) S[i] = S[i] + w * H[i];
            }
            if (r == ty.hi) {
#pragma unroll
              for (int i = 0; i < 12; i++) Hc[i] = H[i];
              cr = r;
            }
          }
#if RRC_AREA_MAGIC
          // cvRound + saturate_cast<uchar>: the sums lie in [0, 255.5) (bytes
          // times weights that sum to 1 up to a few float roundings), so
          // S + 1.5 * 2^23 rounds S half-to-even into the float's low byte and
          // the saturation never acts: one (packed) add per value instead of
          // v_rndne + v_cvt + v_med3, and the u8 bytes packed by v_perm
          uint32_t bz[12];
#pragma unroll
          for (int i = 0; i < 12; i++) bz[i] = ffcv_f2u_bits(S[i] + 12582912.0f);
          if (cmask && dy >= ep.cut_y && dy < ep.cut_y + ep.cut_size) {
#pragma unroll
            for (int j = 0; j < 4; j++)
              if ((cmask >> j) & 1) {
                bz[3 * j] = ep.fill[0];
                bz[3 * j + 1] = ep.fill[1];
                bz[3 * j + 2] = ep.fill[2];
              }
          }
          const uint64_t px = (uint64_t)dy * out_w + dx0;
          if (FP16) {
            uint32_t h[12];
#pragma unroll
            for (int i = 0; i < 12; i++) h[i] = s_lut[(bz[i] & 0xffu) * 3 + i % 3];
            uint2 *o64 = (uint2 *)((uint16_t *)o + px * 3);
            o64[0] = make_uint2(h[0] | (h[1] << 16), h[2] | (h[3] << 16));
            o64[1] = make_uint2(h[4] | (h[5] << 16), h[6] | (h[7] << 16));
            o64[2] = make_uint2(h[8] | (h[9] << 16), h[10] | (h[11] << 16));
          } else {
            typedef uint32_t u32x3 __attribute__((ext_vector_type(3)));
            uint32_t wd[3];
#pragma unroll
            for (int d = 0; d < 3; d++) {  // low bytes of four values: [a, b, 0, 0], [c, d, 0, 0] -> [a, b, c, d]
              const uint32_t lo = __builtin_amdgcn_perm(bz[4 * d + 1], bz[4 * d], 0x0c0c0400u);
              const uint32_t hi = __builtin_amdgcn_perm(bz[4 * d + 3], bz[4 * d + 2], 0x0c0c0400u);
              wd[d] = __builtin_amdgcn_perm(hi, lo, 0x05040100u);
            }
            u32x3 w;
            w.x = wd[0];
            w.y = wd[1];
            w.z = wd[2];
            __builtin_nontemporal_store(w, (u32x3 *)((uint8_t *)o + px * 3));
          }
#else
          int v[12];
#pragma unroll
          for (int i = 0; i < 12; i++) v[i] = sat_u8i(ffcv_f2i_rn(S[i]));
          put(dy, v);
#endif
        }
        return;
      }
      AreaTaps tx[4];
#pragma unroll
      for (int j = 0; j < 4; j++) tx[j] = area_taps(P.sw, P.scale_x, ep.src_x(dx0 + j));
      for (int dy = gy0; dy < gy1; dy++) {
        const AreaTaps ty = s_at[dy - oy0];
        int v[12];
#pragma unroll
        for (int j = 0; j < 4; j++) resize_area_lds(L, tx[j], ty, v + 3 * j);  // (s_src is followed by s_rt: in LDS)
        put(dy, v);
      }
      return;
    }
    int xa[4], xb[4], wa[4], wb[4];
    // (tq0 / tq1: the quad's four column taps, flip applied, loaded before
    // the staging: q below is the same t & (tpg - 1))
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const uint4 &tq = j < 2 ? tq0 : tq1;
      const LinTap l = itaps ? tap_unpack((j & 1) ? make_uint2(tq.z, tq.w) : make_uint2(tq.x, tq.y))
                             : lin_tap(P.scale_x, P.inv_x, P.sw, ep.src_x(dx0 + j));
      // a border tap (src[s] * 2048) as the two-tap form with weights (2048, 0)
      xa[j] = 3 * l.s;
      xb[j] = 3 * (l.border ? l.s : l.s + 1);
      wa[j] = l.border ? 2048 : l.c0;
      wb[j] = l.border ? 0 : l.c1;
    }
    // resize.cpp HResizeLinear of crop row r: sat_s16(h >> 4).  The
    // saturations of this walk never act (so they are not computed): weights
    // are in [0, 2048] with wa + wb <= 2049 (linear_coef rounds each), so
    // 0 <= h >> 4 <= 255 * 2049 >> 4 = 32655 and the vertical sum
    // m0 + m1 <= 32655 * 2049 >> 16 = 1020, (1020 + 2) >> 2 = 255.
    // The row keeps (h >> 4) << 8 (< 2^23), so VResizeLinearVec's
    // (h * c) >> 16 is one 24-bit high multiply by c << 8 (< 2^20):
    // mulhi_u24(h << 8, c << 8) = (h * c * 2^16) >> 32.
    auto hrow = [&](int r, uint32_t H[12]) {
      const uint8_t *row = L.row(r);
#pragma unroll
      for (int j = 0; j < 4; j++)
#pragma unroll
        for (int c = 0; c < 3; c++)
          H[3 * j + c] = (((uint32_t)(row[xa[j] + c] * wa[j] + row[xb[j] + c] * wb[j]) >> 4) & 0x7fffu) << 8;
    };
    auto mulhi24 = [](uint32_t a, uint32_t b) -> uint32_t {  // a, b < 2^24: v_mul_hi_u32_u24
      return (uint32_t)(((uint64_t)(a & 0xffffffu) * (b & 0xffffffu)) >> 32);
    };
    RRC_STOP_AT(3, p.cutout_fill[3] != 77);  // diagnostics: + the linear walk's column taps
    // row taps: from the image's table through the scalar cache (the rows of a
    // row group are wave-uniform) when there is one, else the band's LDS records
    const __attribute__((address_space(4))) uint32_t *rtp =
        itaps ? (const __attribute__((address_space(4))) uint32_t *)(itaps + out_w) : nullptr;
    // the two source rows' horizontal sums live in register sets X and Y;
    // which one is the upper row (A) flips when the walk moves down one
    // source row, instead of copying B into A (12 moves per such row): the
    // flag is wave-uniform, so both orders are separate straight-line code
    uint32_t HX[12], HY[12];
    int cx = -1, cy = -1;  // source rows held by X / Y
    auto emit = [&](int dy, const uint32_t (&A)[12], const uint32_t (&B)[12], uint32_t c0, uint32_t c1) {
      if (FP16) {
        int v[12];
#pragma unroll
        for (int i = 0; i < 12; i++)  // VResizeLinearVec_32s8u: (m0 + 2 + m1) >> 2, no saturation (see hrow)
          v[i] = (int)((mulhi24(A[i], c0) + mulhi24(B[i], c1) + 2u) >> 2);
        put(dy, v);
      } else {
        // u8: t = m0 + m1 + 2 (<= 1022) per value, two values per dword in
        // 16-bit lanes, one packed shift (v_pk_lshrrev_b16) per pair and the
        // low bytes picked by one v_perm per output dword: 5 instructions per
        // dword instead of 8 (a cutout value is fill << 2: exact after >> 2)
        uint32_t tv[12];
#pragma unroll
        for (int i = 0; i < 12; i++) tv[i] = mulhi24(A[i], c0) + mulhi24(B[i], c1) + 2u;
        if (cmask && dy >= ep.cut_y && dy < ep.cut_y + ep.cut_size) {
#pragma unroll
          for (int j = 0; j < 4; j++)
            if ((cmask >> j) & 1) {
              tv[3 * j] = (uint32_t)ep.fill[0] << 2;
              tv[3 * j + 1] = (uint32_t)ep.fill[1] << 2;
              tv[3 * j + 2] = (uint32_t)ep.fill[2] << 2;
            }
        }
        auto shr2 = [](uint32_t x) -> uint32_t {  // both 16-bit halves >> 2
          return __builtin_bit_cast(uint32_t, __builtin_bit_cast(u16x2_t, x) >> (u16x2_t){2, 2});
        };
        typedef uint32_t u32x3 __attribute__((ext_vector_type(3)));
        uint32_t wd[3];
#pragma unroll
        for (int d = 0; d < 3; d++) {
          const uint32_t lo = shr2(tv[4 * d] | (tv[4 * d + 1] << 16)), hi = shr2(tv[4 * d + 2] | (tv[4 * d + 3] << 16));
          wd[d] = __builtin_amdgcn_perm(hi, lo, 0x06040200u);  // bytes lo.0, lo.2, hi.0, hi.2
        }
        u32x3 w;
        w.x = wd[0];
        w.y = wd[1];
        w.z = wd[2];
        // uniform row address (scalar) + this lane's 32-bit offset: the
        // store's saddr form, no 64-bit address arithmetic per row
        typedef __attribute__((address_space(1))) uint8_t gbyte_t;
        typedef __attribute__((address_space(1))) u32x3 gu32x3_t;
        const uint64_t ra64 = (uint64_t)(uintptr_t)o + (uint64_t)(uint32_t)dy * (uint32_t)(3 * out_w);
        gbyte_t *orow = (gbyte_t *)(uintptr_t)(((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(ra64 >> 32)) << 32) |
                                               (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)ra64));
        __builtin_nontemporal_store(w, (gu32x3_t *)(orow + (uint32_t)(3 * dx0)));
      }
    };
    auto row_taps = [&](int dy, int &ra, int &rb, uint32_t &c0, uint32_t &c1) {
      if (rtp) {
        const uint32_t tx = rtp[2 * dy], ty = rtp[2 * dy + 1];
        const int sr = (int)(tx & 0x7fffffffu);
        ra = min(max(sr, 0), P.sh - 1);
        rb = min(max(sr + 1, 0), P.sh - 1);
        c0 = (ty & 0xfffu) << 8;
        c1 = ((ty >> 16) & 0xfffu) << 8;
      } else {
        const uint4 ly = s_rt[dy - oy0];
        ra = (int)ly.x;
        rb = (int)ly.y;
        c0 = ly.z;
        c1 = ly.w;
      }
    };
    // two loops, one per role assignment (a single loop with a role flag was
    // compiled into one shared epilogue fed by 24 register moves per row)
    int dy = gy0;
    while (dy < gy1) {
      for (; dy < gy1; dy++) {  // A = X, B = Y
        int ra, rb;
        uint32_t c0, c1;
        row_taps(dy, ra, rb, c0, c1);
        if (ra != cx && ra == cy) break;  // down one source row: continue with A = Y
        if (ra != cx) {
          hrow(ra, HX);
          cx = ra;
        }
        if (rb != cy) {
          hrow(rb, HY);
          cy = rb;
        }
        emit(dy, HX, HY, c0, c1);
      }
      for (; dy < gy1; dy++) {  // A = Y, B = X
        int ra, rb;
        uint32_t c0, c1;
        row_taps(dy, ra, rb, c0, c1);
        if (ra != cy && ra == cx) break;  // down one source row: continue with A = X
        if (ra != cy) {
          hrow(ra, HY);
          cy = ra;
        }
        if (rb != cx) {
          hrow(rb, HX);
          cx = rb;
        }
        emit(dy, HY, HX, c0, c1);
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
    } else if (staged) {
      resize_pixel(P, L, dy, ep.src_x(dx), v);
    } else {
      resize_pixel(P, src, dy, ep.src_x(dx), v);
    }
    store_px<FP16>(o, (uint64_t)dy * out_w + dx, v, s_lut);
  }
}

template <bool FP16>
__global__ void __launch_bounds__(RRC_THREADS) __attribute__((amdgpu_waves_per_eu(RRC_WPE)))
    rrc_raw_kernel(const uint8_t *__restrict__ base, const ffcv_sample *__restrict__ samples,
                   const int32_t *__restrict__ crops, const int32_t *__restrict__ cut,
                   const uint8_t *__restrict__ flips, ffcv_rrc_params p, uint64_t stride,
                   void *__restrict__ out, const ResizePlan *__restrict__ plans, const uint2 *__restrict__ taps) {
  __shared__ RrcLds<FP16> S;
  rrc_band<FP16>(base, samples, crops, cut, flips, p, stride, out, (int)blockIdx.y, (int)blockIdx.x, S, plans,
                 taps);
}

// Per-image resize plan + linear tap table for rrc_raw_kernel (one thread per
// tap: columns [0, out_w) with the image's flip applied, then rows [out_w,
// out_w + out_h)), the same functions the band workgroups would evaluate
// (resize.cpp linear coefficients, make_plan), so the output is unchanged.
__global__ void __launch_bounds__(256) rrc_taps_kernel(const int32_t *__restrict__ crops,
                                                       const uint8_t *__restrict__ flips, ffcv_rrc_params p,
                                                       ResizePlan *__restrict__ plans, uint2 *__restrict__ taps) {
  const int k = blockIdx.y, i = blockIdx.x * 256 + threadIdx.x;
  const ResizePlan P = make_plan(crops[4 * k + 3], crops[4 * k + 2], p.out_w, p.out_h);
  if (i == 0) plans[k] = P;
  if (area_walk_plan(P)) {  // column records of the area walk: {lo, w(lo), w(lo + 1), w(lo + 2)}, 0 past hi
    if (i >= p.out_w) return;
    const int flip = flips ? flips[k] : 0;
    const AreaTaps a = area_taps(P.sw, P.scale_x, flip ? p.out_w - 1 - i : i);
    uint32_t w[3];
#pragma unroll
    for (int j = 0; j < 3; j++) w[j] = ffcv_f2u_bits(a.lo + j <= a.hi ? a.w(a.lo + j) : 0.f);
    *(uint4 *)(taps + (uint64_t)k * RAW_TAPS(p) + 2 * i) = make_uint4((uint32_t)a.lo, w[0], w[1], w[2]);
    return;
  }
  if (P.kind != 3 || i >= p.out_w + p.out_h) return;
  LinTap l;
  if (i < p.out_w) {
    const int flip = flips ? flips[k] : 0;
    l = lin_tap(P.scale_x, P.inv_x, P.sw, flip ? p.out_w - 1 - i : i);
  } else {
    l = lin_tap(P.scale_y, P.inv_y, P.sh, i - p.out_w);
  }
  taps[(uint64_t)k * RAW_TAPS(p) + i] = tap_pack(l);
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

// normalize.py:64-65: output = table[input * 3 + i % 3] for any table dtype
// (the cupy kernel is templated on T); T is the element's bit pattern, so
// one instantiation per element size serves every dtype of that size.  The
// 768-entry table lives in LDS; 12 elements (4 RGB pixels) per lane, input
// read as three dwords when 4-byte aligned.
template <class T>
__global__ void __launch_bounds__(256) lut_kernel(const uint8_t *__restrict__ in, uint64_t n,
                                                  const T *__restrict__ lut, T *__restrict__ out) {
  __shared__ T s_lut[768];
  for (int i = threadIdx.x; i < 768; i += 256) s_lut[i] = lut[i];
  __syncthreads();
  const uint64_t groups = n / 12;
  const bool aligned = ((uintptr_t)in & 3) == 0;
  for (uint64_t g = (uint64_t)blockIdx.x * 256 + threadIdx.x; g < groups; g += (uint64_t)gridDim.x * 256) {
    const uint8_t *ip = in + g * 12;
    uint8_t v[12];
    if (aligned) {
      const uint32_t *w = (const uint32_t *)ip;
#pragma unroll
      for (int q = 0; q < 3; q++) {
        uint32_t x = w[q];
#pragma unroll
        for (int b = 0; b < 4; b++) v[4 * q + b] = (uint8_t)(x >> (8 * b));
      }
    } else {
#pragma unroll
      for (int e = 0; e < 12; e++) v[e] = ip[e];
    }
    T *op = out + g * 12;
#pragma unroll
    for (int e = 0; e < 12; e++) op[e] = s_lut[v[e] * 3 + (e % 3)];
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

static uint64_t raw_plans_bytes(int batch) { return ((uint64_t)batch * sizeof(ResizePlan) + 255) & ~(uint64_t)255; }

uint64_t ffcv_rrc_raw_workspace_bytes(int batch, int out_h, int out_w) {
  if (batch <= 0 || out_h <= 0 || out_w <= 0) return 0;
  ffcv_rrc_params q{};
  q.out_h = out_h;
  q.out_w = out_w;
  return raw_plans_bytes(batch) + (uint64_t)batch * RAW_TAPS(q) * sizeof(uint2);
}

int ffcv_rrc_raw_batch_ws(void *stream, const uint8_t *base, const ffcv_sample *samples, int batch,
                          const int32_t *crops, const int32_t *cutout_yx, const uint8_t *flips,
                          const ffcv_rrc_params *p, void *out, void *workspace, uint64_t workspace_bytes) {
  if (batch < 0 || !p || !base || !samples || !crops || !out || p->out_h <= 0 || p->out_w <= 0) {
    ffcv::set_error("ffcv_rrc_raw_batch: invalid arguments");
    return FFCV_EINVAL;
  }
  if (batch == 0) return FFCV_OK;
  const ResizePlan *plans = nullptr;
  const uint2 *taps = nullptr;
  if (workspace) {
    const uint64_t need = ffcv_rrc_raw_workspace_bytes(batch, p->out_h, p->out_w);
    if (workspace_bytes < need || ((uintptr_t)workspace & 15)) {
      ffcv::set_error("ffcv_rrc_raw_batch_ws: workspace of %llu bytes (16-byte aligned) needed, got %llu",
                      (unsigned long long)need, (unsigned long long)workspace_bytes);
      return FFCV_EINVAL;
    }
    ResizePlan *wp = (ResizePlan *)workspace;
    uint2 *wt = (uint2 *)((uint8_t *)workspace + raw_plans_bytes(batch));
    hipLaunchKernelGGL(rrc_taps_kernel, dim3((p->out_w + p->out_h + 255) / 256, batch), dim3(256), 0,
                       ffcv::as_stream(stream), crops, flips, *p, wp, wt);
    FFCV_LAUNCH_CHECK("rrc_taps_kernel");
    plans = wp;
    taps = wt;
  }
  const bool fp16 = p->lut != nullptr;
  uint64_t dense = (uint64_t)p->out_h * p->out_w * 3 * (fp16 ? 2 : 1);
  uint64_t stride = p->out_stride ? p->out_stride : dense;
  dim3 grid((p->out_h + RRC_BAND - 1) / RRC_BAND, batch);
  if (fp16)
    hipLaunchKernelGGL(rrc_raw_kernel<true>, grid, dim3(RRC_THREADS), 0, ffcv::as_stream(stream), base,
                       samples, crops, cutout_yx, flips, *p, stride, out, plans, taps);
  else
    hipLaunchKernelGGL(rrc_raw_kernel<false>, grid, dim3(RRC_THREADS), 0, ffcv::as_stream(stream), base,
                       samples, crops, cutout_yx, flips, *p, stride, out, plans, taps);
  FFCV_LAUNCH_CHECK("rrc_raw_kernel");
  return FFCV_OK;
}

int ffcv_rrc_raw_batch(void *stream, const uint8_t *base, const ffcv_sample *samples, int batch,
                       const int32_t *crops, const int32_t *cutout_yx, const uint8_t *flips,
                       const ffcv_rrc_params *p, void *out) {
  return ffcv_rrc_raw_batch_ws(stream, base, samples, batch, crops, cutout_yx, flips, p, out, nullptr, 0);
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

int ffcv_lut_batch(void *stream, const uint8_t *in, uint64_t n, const void *lut, int elem_bytes, void *out) {
  if (!in || !lut || !out || !(elem_bytes == 1 || elem_bytes == 2 || elem_bytes == 4 || elem_bytes == 8)) {
    ffcv::set_error("ffcv_lut_batch: invalid arguments (element size %d)", elem_bytes);
    return FFCV_EINVAL;
  }
  if (n == 0) return FFCV_OK;
  uint64_t groups = n / 12 + 1;
  unsigned gx = (unsigned)((groups + 255) / 256);
  if (gx > 8192) gx = 8192;
  hipStream_t s = ffcv::as_stream(stream);
  switch (elem_bytes) {
    case 1:
      hipLaunchKernelGGL(lut_kernel<uint8_t>, dim3(gx), dim3(256), 0, s, in, n, (const uint8_t *)lut, (uint8_t *)out);
      break;
    case 2:
      hipLaunchKernelGGL(lut_kernel<uint16_t>, dim3(gx), dim3(256), 0, s, in, n, (const uint16_t *)lut,
                         (uint16_t *)out);
      break;
    case 4:
      hipLaunchKernelGGL(lut_kernel<uint32_t>, dim3(gx), dim3(256), 0, s, in, n, (const uint32_t *)lut,
                         (uint32_t *)out);
      break;
    default:
      hipLaunchKernelGGL(lut_kernel<uint64_t>, dim3(gx), dim3(256), 0, s, in, n, (const uint64_t *)lut,
                         (uint64_t *)out);
      break;
  }
  FFCV_LAUNCH_CHECK("lut_kernel");
  return FFCV_OK;
}

int ffcv_normalize_batch(void *stream, const uint8_t *in, uint64_t n, const uint16_t *lut, uint16_t *out) {
  return ffcv_lut_batch(stream, in, n, lut, 2, out);
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
