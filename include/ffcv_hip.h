/*
 * ffcv_hip.h -- C ABI of libffcv_hip.so, the MI355X (gfx950) replacement for
 * the reference's native shim.
 *
 * Reference boundary being replaced:
 *   /root/reference/libffcv/libffcv.cpp   (exports resize / my_memcpy /
 *                                          my_fread / imdecode, :33-112)
 *   /root/reference/ffcv/libffcv.py       (ctypes binding, :8-55)
 * The reference binds ONE sample per call from numba prange workers.  This
 * ABI is batch- and device-first: every compute entry point takes a device
 * base pointer to the .beton bytes resident in HBM, a device array of
 * per-sample descriptors, and a hipStream_t (passed as void*) on which all
 * work is enqueued asynchronously.  No torch types, no hidden hipMalloc in a
 * launch, no host synchronisation in a launch (graph-capturable).
 *
 * Ownership: the caller owns every input/output buffer.  The library owns
 * only the scratch inside an ffcv_jpeg_ctx (allocated once at create time).
 *
 * Errors: every function returns an int status (FFCV_OK == 0).  On failure a
 * thread-local message is available from ffcv_last_error().  Per-sample
 * decode failures (corrupt / unsupported JPEG) are reported in a device
 * int32 status array and the sample's output is zero-filled; the reference
 * ignores imdecode's return code (rgb_image.py:131,196) and yields garbage.
 */
#ifndef FFCV_HIP_H
#define FFCV_HIP_H
#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FFCV_HIP_ABI_VERSION 1

enum {
  FFCV_OK = 0,
  FFCV_EINVAL = -1,      /* bad argument */
  FFCV_EHIP = -2,        /* HIP runtime error */
  FFCV_ENOMEM = -3,      /* allocation failed */
  FFCV_EUNSUPPORTED = -4 /* feature not on this path */
};

/* Per-sample status codes written by the device (int32). */
enum {
  FFCV_SAMPLE_OK = 0,
  FFCV_SAMPLE_BAD_MARKER = 1,      /* not a JPEG / truncated header */
  FFCV_SAMPLE_UNSUPPORTED = 2,     /* progressive, arithmetic, 12-bit, DRI, CMYK */
  FFCV_SAMPLE_TOO_LARGE = 3,       /* exceeds the ctx's max size or scratch arena */
  FFCV_SAMPLE_CORRUPT = 4,         /* entropy stream inconsistent */
  FFCV_SAMPLE_GEOMETRY = 5,        /* SOF size != .beton metadata */
  FFCV_SAMPLE_RNG = 6              /* > 623 MT19937 draws for one stream */
};

/* One sample of a batch, as resolved from the .beton metadata + allocation
 * table (rgb_image.py:302-308 metadata; memory_managers/os_cache.py:55-60
 * read).  32 bytes, device-resident array. */
typedef struct ffcv_sample {
  uint64_t offset; /* byte offset of the sample's data from the base pointer */
  uint64_t size;   /* byte count (allocation table 'size') */
  uint32_t height; /* metadata 'height' */
  uint32_t width;  /* metadata 'width' */
  uint32_t mode;   /* 0 = jpg, 1 = raw (rgb_image.py:21-23) */
  uint32_t reserved;
} ffcv_sample;

/* Parameters of a fused decode -> crop -> resize -> cutout -> normalize
 * launch (rgb_image.py:168-212, cutout.py:31-52, normalize.py:58-87). */
typedef struct ffcv_rrc_params {
  int32_t out_h, out_w;    /* output_size (rgb_image.py:145-149) */
  int32_t cutout_size;     /* 0: no cutout; else crop_size (cutout.py:26) */
  uint8_t cutout_fill[4];  /* fill RGB (cutout.py:29); [3] = 1 when the
                              pipeline runs Cutout BEFORE RandomHorizontalFlip
                              (0: flip first, then cutout) */
  const uint16_t *lut;     /* device [256][3] fp16 bits (normalize.py:42-49), or
                              NULL for uint8 output */
  uint64_t out_stride;     /* bytes between samples in the output; 0 = dense */
} ffcv_rrc_params;

/* Crop-draw parameters (rgb_image.py:48-81) + seeding contract
 * (DESIGN.md "RNG contract": one MT19937 per (op, sample, epoch) seeded
 * with low32(splitmix64 chain of loader_seed, epoch, sample index, op id)). */
typedef struct ffcv_draw_params {
  int32_t crop_kind;       /* 0 = get_random_crop, 1 = get_center_crop */
  int32_t out_h, out_w;    /* needed for cutout bounds */
  int32_t cutout_size;     /* 0 = no cutout draw */
  double scale[2];         /* RandomResizedCrop scale (rgb_image.py:234) */
  double ratio[2];         /* RandomResizedCrop ratio */
  double center_ratio;     /* CenterCrop ratio (rgb_image.py:259) */
  uint64_t loader_seed;
  uint64_t epoch;
  double flip_prob;        /* RandomHorizontalFlip probability (flip.py:33) */
} ffcv_draw_params;

/* ---------------------------------------------------------------- misc -- */
int ffcv_abi_version(void);
const char *ffcv_last_error(void);
int ffcv_device_count(int *count);
int ffcv_set_device(int device);
int ffcv_stream_synchronize(void *stream);

/* Device memory helpers (for callers without torch; the Python package uses
 * torch allocations instead). */
int ffcv_malloc(void **dptr, uint64_t bytes);
int ffcv_free(void *dptr);
int ffcv_memcpy_h2d_async(void *dst, const void *src, uint64_t bytes, void *stream);
int ffcv_memcpy_d2h_async(void *dst, const void *src, uint64_t bytes, void *stream);

/* libffcv.cpp:44-46 my_memcpy (host plumbing; SimpleRGBImageDecoder raw on a
 * CPU-only Loader, C1).  Same argument order as the reference. */
void my_memcpy(void *source, void *dst, uint64_t size);

/* libffcv.cpp:48-51 my_fread: fseek((FILE *)fp, offset, SEEK_SET) then
 * fread(destination, 1, size, fp) (host plumbing; exported by the reference,
 * never bound by its Python).  Same arguments; like the reference it returns
 * nothing, and a short read leaves the rest of destination untouched. */
void my_fread(int64_t fp, int64_t offset, void *destination, int64_t size);

/* libffcv.cpp:33-42 resize: cv::resize(src[start_row:end_row,
 * start_col:end_col], dst, (tx rows, ty cols), INTER_AREA) where src is an
 * sx x sy x 3 uint8 image and dst a tx x ty x 3 uint8 buffer, both in host
 * memory (bound as resize_crop, ffcv/libffcv.py:22-31; cresizer unused).
 * Computed on the CPU by the kernels' own INTER_AREA functions.  On an
 * invalid ROI nothing is written and ffcv_last_error() says why. */
void resize(int64_t cresizer, int64_t source_p, int64_t sx, int64_t sy,
            int64_t start_row, int64_t end_row, int64_t start_col,
            int64_t end_col, int64_t dest_p, int64_t tx, int64_t ty);

/* libffcv.cpp:53-112 imdecode (bound at ffcv/libffcv.py:34-48): decode the
 * JPEG input_buffer[input_size] to crop_height x crop_width x 3 RGB in host
 * output_buffer, tjDecompress2(TJPF_RGB, TJFLAG_FASTDCT) semantics (ifast
 * IDCT, fancy upsampling), on the CPU of the calling thread like the
 * reference (ffcv_cpu_jpeg.hip; thread-safe, per-thread scratch).  Baseline
 * / extended sequential Huffman, 8-bit, 1 or 3 components, restart
 * intervals.  With enable_crop or hflip, the reference's tjTransform
 * (TJXOPT_CROP at offset_x, offset_y, crop_width x crop_height, plus
 * TJXOP_HFLIP) is applied to the coefficients first (lossless: the crop origin
 * must be on an iMCU boundary, the size is clamped to the image, the crop is
 * taken in the mirrored frame, the partial iMCU column at the right edge is
 * not mirrored).  As tjDecompress2 does, the decode runs at the largest
 * TurboJPEG scaling factor whose output fits the requested size (scaled by
 * scale_num / scale_denom), rows packed at the decoded width; the factors
 * 1/1, 1/2, 1/4 and 1/8 are restated (libjpeg's reduced IDCTs, bit-exact
 * with libjpeg-turbo).  Returns 0, or -1 on a decode error, an unsupported
 * stream (progressive, arithmetic, multi-scan, CMYK), a misaligned crop, or
 * a request TurboJPEG would decode at another factor -- see
 * ffcv_last_error().  ffcv itself passes the image's size, 0, 0, 1, 1,
 * False, False. */
int imdecode(unsigned char *input_buffer, uint64_t input_size,
             uint32_t source_height, uint32_t source_width,
             unsigned char *output_buffer, uint32_t crop_height,
             uint32_t crop_width, uint32_t offset_x, uint32_t offset_y,
             uint32_t scale_num, uint32_t scale_denom, bool enable_crop,
             bool hflip);

/* The reference's per-sample CPU decode loop (rgb_image.py:123-136 Simple,
 * :185-210 ResizedCrop, under numba prange) as one call over nthreads host
 * threads: sample k (data[k], sizes[k] bytes, heights[k] x widths[k], modes[k]
 * 0 = jpg through imdecode, 1 = raw, other = skipped) is written whole at
 * out + k * out_stride, or, with crops (batch x 4: i, j, h, w), cut and resized
 * by resize() to out_h x out_w there.  status[k] = 0, or -1 when its decode
 * failed.  Returns FFCV_OK or FFCV_EINVAL. */
int ffcv_cpu_decode_batch(const uint8_t *const *data, const uint64_t *sizes,
                          const uint32_t *heights, const uint32_t *widths,
                          const uint32_t *modes, int batch, const int32_t *crops,
                          int out_h, int out_w, uint8_t *out, uint64_t out_stride,
                          int nthreads, int32_t *status);

/* Measurement helper (new; no reference counterpart): per image k of n,
 * stats[3k] = Huffman symbols of its scan (DC + AC, EOB / ZRL included),
 * stats[3k+1] = blocks, stats[3k+2] = entropy-coded bytes (host decode by the
 * CPU decoder's Huffman loop).  bench.py's K1 lane-instructions per symbol.
 * Returns FFCV_OK, -1 when an image does not parse (its stats are 0), or
 * FFCV_EINVAL. */
int ffcv_jpeg_scan_stats(const uint8_t *const *data, const uint64_t *sizes, int n, uint64_t *stats);

/* imdecode's signature and semantics, executed by the gfx950 JPEG kernels
 * (per-thread stream and decoder context; host buffers in and out). */
int ffcv_imdecode_device(unsigned char *input_buffer, uint64_t input_size,
                         uint32_t source_height, uint32_t source_width,
                         unsigned char *output_buffer, uint32_t crop_height,
                         uint32_t crop_width, uint32_t offset_x,
                         uint32_t offset_y, uint32_t scale_num,
                         uint32_t scale_denom, bool enable_crop, bool hflip);

/* Host gather of n byte ranges src + src_off[i] (sizes[i] bytes) to
 * dst + dst_off[i], split over nthreads threads by bytes: the PCIe path's
 * per-batch staging of compressed samples from the mmap'd .beton
 * (memory_managers/os_cache.py:55-60 read, batched). */
int ffcv_host_gather(const uint8_t *src, const uint64_t *src_off, const uint64_t *sizes,
                     const uint64_t *dst_off, int n, uint8_t *dst, int nthreads);

/* ------------------------------------------------------- random draws -- */
/* rgb_image.py:48-81 crop windows (+ cutout.py:38-42 origins, + flip.py:35
 * decisions) for B samples, on the device.
 *   sample_ids : device uint64[B] dataset indices (batch_indices)
 *   samples    : device ffcv_sample[B] (height/width used; may be NULL when
 *                crops is NULL)
 *   crops      : device int32[B][4] (i, j, h, w) out
 *   cutout_yx  : device int32[B][2] out, or NULL
 *   flips      : device uint8[B] out, or NULL
 *   status     : device int32[B] out, or NULL */
int ffcv_draw_batch(void *stream, const uint64_t *sample_ids,
                    const ffcv_sample *samples, int batch,
                    const ffcv_draw_params *p, int32_t *crops,
                    int32_t *cutout_yx, uint8_t *flips, int32_t *status);

/* The same draws on the host (the CPU-device Loader's decoders): heights /
 * widths / sample_ids are host arrays, outputs host arrays. */
int ffcv_draw_batch_host(const uint64_t *sample_ids, const uint32_t *heights,
                         const uint32_t *widths, int batch,
                         const ffcv_draw_params *p, int32_t *crops,
                         int32_t *cutout_yx, uint8_t *flips);

/* ------------------------------------------- raw-mode crop + resize ---- */
/* rgb_image.py:202-208 (raw branch) + libffcv.cpp:33-42 cv::resize
 * INTER_AREA, fused with Cutout (cutout.py:44) and the NormalizeImage LUT
 * (normalize.py:65).  Samples with mode != raw are skipped.
 *   base  : device pointer to the .beton bytes (file offset 0)
 *   out   : device [B][out_h][out_w][3] uint8 (lut==NULL) or fp16 bits */
int ffcv_rrc_raw_batch(void *stream, const uint8_t *base,
                       const ffcv_sample *samples, int batch,
                       const int32_t *crops, const int32_t *cutout_yx,
                       const uint8_t *flips, const ffcv_rrc_params *p,
                       void *out);

/* The same with a caller-provided device workspace (16-byte aligned, at
 * least ffcv_rrc_raw_workspace_bytes(batch, out_h, out_w) bytes; NULL runs
 * ffcv_rrc_raw_batch): each image's resize plan and its linear tap table
 * (or, for INTER_AREA crops at scales < 2, its column records) are computed
 * once (one small kernel, one thread per tap) instead of in every band
 * workgroup of the image.  Output is identical.  The workspace is
 * overwritten by the launch and must not be shared by launches in flight
 * on different streams. */
int ffcv_rrc_raw_batch_ws(void *stream, const uint8_t *base,
                          const ffcv_sample *samples, int batch,
                          const int32_t *crops, const int32_t *cutout_yx,
                          const uint8_t *flips, const ffcv_rrc_params *p,
                          void *out, void *workspace, uint64_t workspace_bytes);
uint64_t ffcv_rrc_raw_workspace_bytes(int batch, int out_h, int out_w);

/* Per-batch descriptor gather: out[k] = table[ids[k]] (the reference reads
 * metadata[source_ix] per sample, rgb_image.py:188-189).  table: device
 * ffcv_sample[N] built once per dataset; ids: device uint64[B]. */
int ffcv_gather_samples(void *stream, const ffcv_sample *table, uint64_t n_table,
                        const uint64_t *ids, int batch, ffcv_sample *out);

/* rgb_image.py:123-136 SimpleRGBImageDecoder raw branch (my_memcpy per
 * sample) as a device gather into [B][H][W][3]. */
int ffcv_gather_raw_batch(void *stream, const uint8_t *base,
                          const ffcv_sample *samples, int batch, uint8_t *out,
                          uint64_t out_stride);

/* ------------------------------------------------------- JPEG decode -- */
/* Baseline-sequential Huffman JPEG, 8-bit, 1 or 3 components, any 1x/2x
 * sampling, bit-exact with libjpeg-turbo tjDecompress2(TJPF_RGB,
 * TJFLAG_FASTDCT) (libffcv.cpp:104-106): ifast IDCT, fancy upsampling,
 * fixed-point YCbCr->RGB.  One context holds the scratch for up to
 * max_batch images of at most max_height x max_width pixels and max_bytes
 * compressed bytes each. */
typedef struct ffcv_jpeg_ctx ffcv_jpeg_ctx;
int ffcv_jpeg_create(ffcv_jpeg_ctx **ctx, int max_batch, uint32_t max_height,
                     uint32_t max_width, uint64_t max_bytes);
/* Scratch is one arena per context, bump-allocated per image by the entropy
 * kernel from the image's own size and crop window (not dataset-max x
 * batch).  ffcv_jpeg_create sizes it for max_batch images of the maximum
 * size; ffcv_jpeg_create_arena takes the size from the caller, e.g. the sum
 * of ffcv_jpeg_scratch_bound over the largest max_batch images of a dataset
 * (a launch can then never exhaust it).  An image that does not fit in what
 * is left of the arena gets FFCV_SAMPLE_TOO_LARGE. */
int ffcv_jpeg_create_arena(ffcv_jpeg_ctx **ctx, int max_batch,
                           uint32_t max_height, uint32_t max_width,
                           uint64_t max_bytes, uint64_t arena_bytes);
/* Upper bound of the arena bytes one image of this size (and compressed
 * size) can take, for any crop (host function, no device access). */
uint64_t ffcv_jpeg_scratch_bound(uint32_t height, uint32_t width,
                                 uint64_t nbytes);
int ffcv_jpeg_destroy(ffcv_jpeg_ctx *ctx);

/* Arena bytes the last entropy launch on `stream` bump-allocated (waits for
 * the stream), and the arena's capacity (may be NULL): the high-water mark
 * for sizing arenas. */
int ffcv_jpeg_arena_used(ffcv_jpeg_ctx *ctx, void *stream, uint64_t *used,
                         uint64_t *capacity);

/* rgb_image.py:185-210 jpg branch fused end to end: decode only the MCUs the
 * crop needs -> crop -> INTER_AREA -> cutout -> LUT.  Samples with mode !=
 * jpg are skipped (call ffcv_rrc_raw_batch for them).  status: device
 * int32[B] (FFCV_SAMPLE_*), required. */
int ffcv_jpeg_rrc_batch(ffcv_jpeg_ctx *ctx, void *stream, const uint8_t *base,
                        const ffcv_sample *samples, int batch,
                        const int32_t *crops, const int32_t *cutout_yx,
                        const uint8_t *flips, const ffcv_rrc_params *p,
                        void *out, int32_t *status);

/* ffcv_gather_samples + ffcv_draw_batch + ffcv_jpeg_rrc_batch in one launch
 * sequence: the entropy kernel reads sample ids[k] of table[n_table] and
 * draws its crop / cutout origin / flip under the seeding contract itself
 * (two fewer small kernels on the slot's stream).  crops (int32[B,4]) is
 * required; cutout_yx (int32[B,2]) and flips (uint8[B]) may be NULL; all
 * three are written for the caller, like ffcv_draw_batch.  samples_out
 * (ffcv_sample[B], may be NULL) receives the gathered descriptors, e.g. for
 * ffcv_rrc_raw_batch on the raw samples of a mixed field.  An RNG overrun
 * sets that sample's status to FFCV_SAMPLE_RNG. */
int ffcv_jpeg_rrc_fused(ffcv_jpeg_ctx *ctx, void *stream, const uint8_t *base,
                        const ffcv_sample *table, uint64_t n_table,
                        const uint64_t *ids, int batch, const ffcv_draw_params *dp,
                        int32_t *crops, int32_t *cutout_yx, uint8_t *flips,
                        ffcv_sample *samples_out, const ffcv_rrc_params *p,
                        void *out, int32_t *status);

/* Entropy index: index[n_samples][64][3] uint32, zero-initialised and owned
 * by the caller (768 B per dataset sample).  With it attached, a
 * ffcv_jpeg_rrc_fused decode of dataset sample ids[k] that finds no record
 * runs the self-synchronising Huffman sync and publishes the converged start
 * state of each lane range; a later decode of the same sample (the next
 * epoch) reads it and skips the sync rounds.  Output is bit-identical either
 * way.  NULL detaches.  Records are written and read with plain memory
 * operations and carry a 64-bit hash of their words, so a launch on another
 * stream that reads a record while it is being published sees a torn record
 * fail the hash and decodes that sample in full. */
int ffcv_jpeg_set_entropy_index(ffcv_jpeg_ctx *ctx, uint32_t *index,
                                uint64_t n_samples);

/* Measurement (no reference counterpart; bench.py's per-kernel roofline):
 * with max_launches > 0 the next max_launches RRC launches on this context
 * record HIP events on their own stream before the entropy kernel, after
 * it, after the IDCT kernel and after the colour/resize kernel; 0 turns it
 * off.  ffcv_jpeg_timing_read waits for the recorded launches and writes
 * ms[3*i + {0,1,2}] = the three kernels' durations of launch i (in launch
 * order, at most max_launches), then starts a new recording. */
int ffcv_jpeg_set_timing(ffcv_jpeg_ctx *ctx, int max_launches);
int ffcv_jpeg_timing_read(ffcv_jpeg_ctx *ctx, float *ms, int max_launches,
                          int *n_launches);

/* rgb_image.py:123-136 SimpleRGBImageDecoder jpg branch (imdecode into the
 * destination, full image) -> device [B][H][W][3] with out_stride bytes per
 * sample. */
int ffcv_jpeg_decode_batch(ffcv_jpeg_ctx *ctx, void *stream,
                           const uint8_t *base, const ffcv_sample *samples,
                           int batch, uint8_t *out, uint64_t out_stride,
                           int32_t *status);

/* Test hook: quantised coefficients (DC predicted, natural order) of every
 * block in MCU order, [B][max_blocks][64] int16, for checking the entropy
 * stage against the oracle on its own. */
int ffcv_jpeg_coefficients_batch(ffcv_jpeg_ctx *ctx, void *stream,
                                 const uint8_t *base,
                                 const ffcv_sample *samples, int batch,
                                 int16_t *coefs, uint64_t max_blocks,
                                 int32_t *status);

/* ---------------------------------------------- standalone transforms -- */
/* cutout.py:36-47 in place on a device [B][H][W][3] uint8 batch. */
int ffcv_cutout_batch(void *stream, uint8_t *images, int batch, int height,
                      int width, const int32_t *cutout_yx, int crop_size,
                      const uint8_t fill[3]);
/* normalize.py:64-65 cupy ElementwiseKernel 'output = table[input*3 + i%3]'
 * (templated on the output type T there): out[i] = lut[in[i]*3 + i%3] over n
 * elements of a channels-last uint8 batch.  lut: device [256][3] table of
 * elem_bytes-wide elements (1, 2, 4 or 8: u8/int16/fp16/fp32/f64 ...). */
int ffcv_lut_batch(void *stream, const uint8_t *in, uint64_t n,
                   const void *lut, int elem_bytes, void *out);
/* ffcv_lut_batch with a fp16 (int16 bits) table (normalize.py:45-48). */
int ffcv_normalize_batch(void *stream, const uint8_t *in, uint64_t n,
                         const uint16_t *lut, uint16_t *out);
/* flip.py:35-40: dst[i] = images[i, :, ::-1] where flips[i] != 0. */
int ffcv_flip_batch(void *stream, const uint8_t *in, uint8_t *out, int batch,
                    int height, int width, int channels_bytes,
                    const uint8_t *flips);

#ifdef __cplusplus
}
#endif
#endif
