/*
 * ffcv_oracle.h -- CPU restatement of the reference hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load this library, and only as the
 * checker / reported CPU baseline -- never as the thing measured or shipped.
 *
 * Each function cites the reference code it restates.  Third-party algorithms
 * the reference reaches (libjpeg-turbo 2.1.0 per ffcv-conda.yml:40, OpenCV
 * 4.5.4.58 per ffcv-conda.yml:94, numba 0.54.1 RNG per ffcv-conda.yml:92) are
 * restated from their published algorithms; see DESIGN.md "Oracle" for how
 * each is pinned.
 */
#ifndef FFCV_ORACLE_H
#define FFCV_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- RNG (numpy-legacy MT19937 == numba's per-thread generator) ---- */
typedef struct {
  uint32_t key[624];
  int pos;
} orc_mt;
void orc_mt_seed(orc_mt *s, uint32_t seed);
uint32_t orc_mt_u32(orc_mt *s);
double orc_mt_double(orc_mt *s);
double orc_uniform(orc_mt *s, double lo, double hi);
int64_t orc_randint(orc_mt *s, int64_t high); /* [0, high) legacy masked */

/* Per-sample seeding contract (DESIGN.md "RNG contract"). */
uint64_t orc_splitmix64(uint64_t x);
uint32_t orc_sample_seed(uint64_t loader_seed, uint64_t epoch, uint64_t sample,
                         uint32_t op_id);

/* rgb_image.py:48-72 */
void orc_random_crop(orc_mt *s, uint32_t height, uint32_t width,
                     const double scale[2], const double ratio[2],
                     int32_t out_ijhw[4]);
/* rgb_image.py:75-81 */
void orc_center_crop(uint32_t height, uint32_t width, double ratio,
                     int32_t out_ijhw[4]);

/* ---- OpenCV 4.5.4 cv::resize(INTER_AREA), 8UC3, as called by
 *      libffcv.cpp:33-42 on a ROI.  src points at the ROI's first pixel. ---- */
void orc_resize_area_u8c3(const uint8_t *src, size_t src_step, int sw, int sh,
                          uint8_t *dst, size_t dst_step, int dw, int dh);
/* libffcv.cpp:33-42 signature restated (resize(cresizer, src, sx, sy, r0, r1,
 * c0, c1, dst, tx, ty)). */
void orc_resize_crop(const uint8_t *src, int64_t sx, int64_t sy, int64_t r0,
                     int64_t r1, int64_t c0, int64_t c1, uint8_t *dst,
                     int64_t tx, int64_t ty);

/* ---- libjpeg-turbo decode restatement (tjDecompress2 TJPF_RGB,
 *      TJFLAG_FASTDCT: libffcv.cpp:104-106) ---- */
typedef struct {
  int width, height, ncomp;
  int hmax, vmax;
  int h[4], v[4], tq[4], td[4], ta[4];
  int restart_interval;
  int sof; /* 0xC0.. */
  size_t scan_off, scan_end;
} orc_jpeg_info;
int orc_jpeg_header(const uint8_t *buf, size_t n, orc_jpeg_info *info);
/* dct_method: 1 = ifast (what the reference uses); 0 = islow (used only to
 * cross-check Huffman/upsample/colour against Pillow's default decode). */
int orc_jpeg_decode(const uint8_t *buf, size_t n, uint8_t *out_rgb,
                    int dct_method);
/* Quantised coefficients in MCU block order (natural order inside a block,
 * DC already predicted), for checking the GPU entropy stage on its own. */
int orc_jpeg_coefficients(const uint8_t *buf, size_t n, int16_t *coefs,
                          size_t max_blocks, size_t *nblocks);

/* ---- cutout.py:36-47 (fill a c*c square at (y,x)) ---- */
void orc_cutout(uint8_t *img, int h, int w, int y, int x, int c,
                const uint8_t fill[3]);

/* ---- Whole-sample reference path (CPU baseline + parity):
 *      rgb_image.py:185-210 decode -> crop -> resize, cutout.py, and the
 *      normalize LUT of normalize.py:42-49 (lut == NULL -> u8 output). ---- */
typedef struct {
  const uint8_t *data; /* sample bytes (jpg or raw) */
  uint64_t size;
  uint32_t height, width;
  uint8_t mode; /* 0 jpg, 1 raw (rgb_image.py:21-23) */
} orc_sample;
int orc_rrc_batch(const orc_sample *samples, int n, const int32_t *crops,
                  int out_h, int out_w, const int32_t *cutout_yx,
                  int cutout_size, const uint8_t fill[3],
                  const uint16_t *lut /* [256*3] fp16 bits or NULL */,
                  void *out, int nthreads);
/* Crop + cutout draws for a batch under the seeding contract. */
void orc_draw_batch(const uint64_t *sample_ids, const uint32_t *heights,
                    const uint32_t *widths, int n, uint64_t loader_seed,
                    uint64_t epoch, int crop_kind /*0 random,1 center*/,
                    const double scale[2], const double ratio[2],
                    double center_ratio, int out_h, int out_w,
                    int cutout_size, int32_t *crops, int32_t *cutout_yx);

#ifdef __cplusplus
}
#endif
#endif
