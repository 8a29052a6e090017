/*
 * ljt_harness.c -- TEST INFRASTRUCTURE ONLY (oracle pinning).
 *
 * Drives a third-party libjpeg-turbo binary (the copy bundled inside the
 * installed Pillow wheel, libjpeg-turbo 3.1.4, jpeg62 ABI) through dlopen so
 * that the oracle's JPEG restatement (oracle/ffcv_oracle.c) can be checked
 * bit-for-bit against the library the reference calls.  The reference reaches
 * libjpeg-turbo through TurboJPEG:
 *     tjDecompress2(h, buf, n, out, w, 0, h, TJPF_RGB, TJFLAG_FASTDCT|...)
 *     (/root/reference/libffcv/libffcv.cpp:104-106)
 * which is jpeg_read_header + dct_method=JDCT_IFAST + out_color_space=RGB +
 * do_fancy_upsampling=TRUE + jpeg_read_scanlines.  This file sets exactly
 * those fields.
 *
 * No libjpeg header exists in this image, so the few jpeg62 struct offsets we
 * touch are declared here (libjpeg 6b field order, x86-64 LP64).  They are
 * validated at run time: the struct size is probed through
 * jpeg_CreateDecompress's own size check, and the decoded geometry is
 * compared against the SOF dimensions the oracle parses.
 *
 * Never shipped; never linked into the product library.
 */
#include <dlfcn.h>
#include <setjmp.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef void *(*fn_std_error)(void *err);
typedef void (*fn_create)(void *cinfo, int version, size_t structsize);
typedef void (*fn_mem_src)(void *cinfo, const unsigned char *buf, unsigned long n);
typedef int (*fn_read_header)(void *cinfo, int require_image);
typedef int (*fn_start)(void *cinfo);
typedef unsigned (*fn_read_scanlines)(void *cinfo, unsigned char **rows, unsigned max_lines);
typedef int (*fn_finish)(void *cinfo);
typedef void (*fn_destroy)(void *cinfo);
typedef int (*fn_abort)(void *cinfo);

static void *g_lib;
static fn_std_error p_std_error;
static fn_create p_create;
static fn_mem_src p_mem_src;
static fn_read_header p_read_header;
static fn_start p_start;
static fn_read_scanlines p_read_scanlines;
static fn_finish p_finish;
static fn_destroy p_destroy;
static size_t g_structsize;

/* jpeg62 field offsets (libjpeg 6b order; see header comment). */
#define OFF_ERR 0
#define OFF_IMAGE_WIDTH 48
#define OFF_IMAGE_HEIGHT 52
#define OFF_NUM_COMPONENTS 56
#define OFF_OUT_COLOR_SPACE 64
#define OFF_SCALE_NUM 68
#define OFF_SCALE_DENOM 72
#define OFF_DCT_METHOD 96
#define OFF_DO_FANCY 100
#define OFF_OUTPUT_WIDTH 136
#define OFF_OUTPUT_HEIGHT 140
#define OFF_OUTPUT_COMPONENTS 148
#define OFF_OUTPUT_SCANLINE 168

#define JCS_RGB 2

/* error manager: libjpeg's default error_exit calls exit(); ours longjmps. */
typedef struct {
  unsigned char std[512]; /* struct jpeg_error_mgr lives at the front */
  jmp_buf jb;
  int failed;
} err_wrap;

static void my_error_exit(void *cinfo) {
  err_wrap *e = *(err_wrap **)((char *)cinfo + OFF_ERR);
  e->failed = 1;
  longjmp(e->jb, 1);
}
static void my_emit(void *cinfo, int lvl) { (void)cinfo; (void)lvl; }

int ljt_open(const char *path) {
  if (g_lib) return 0;
  g_lib = dlopen(path, RTLD_NOW | RTLD_LOCAL);
  if (!g_lib) return -1;
  p_std_error = (fn_std_error)dlsym(g_lib, "jpeg_std_error");
  p_create = (fn_create)dlsym(g_lib, "jpeg_CreateDecompress");
  p_mem_src = (fn_mem_src)dlsym(g_lib, "jpeg_mem_src");
  p_read_header = (fn_read_header)dlsym(g_lib, "jpeg_read_header");
  p_start = (fn_start)dlsym(g_lib, "jpeg_start_decompress");
  p_read_scanlines = (fn_read_scanlines)dlsym(g_lib, "jpeg_read_scanlines");
  p_finish = (fn_finish)dlsym(g_lib, "jpeg_finish_decompress");
  p_destroy = (fn_destroy)dlsym(g_lib, "jpeg_destroy_decompress");
  if (!p_std_error || !p_create || !p_mem_src || !p_read_header || !p_start ||
      !p_read_scanlines || !p_finish || !p_destroy)
    return -2;
  /* probe sizeof(struct jpeg_decompress_struct) via the library's own check */
  static unsigned char cinfo[4096];
  static err_wrap ew;
  for (size_t sz = 200; sz <= 2048; sz += 8) {
    memset(cinfo, 0, sizeof(cinfo));
    memset(&ew, 0, sizeof(ew));
    p_std_error(ew.std);
    ((void **)ew.std)[0] = (void *)my_error_exit;
    ((void **)ew.std)[1] = (void *)my_emit;
    *(void **)(cinfo + OFF_ERR) = &ew;
    if (setjmp(ew.jb) == 0) {
      p_create(cinfo, 62, sz);
      g_structsize = sz;
      p_destroy(cinfo);
      return 0;
    }
  }
  return -3;
}

size_t ljt_structsize(void) { return g_structsize; }

/* Decode to interleaved RGB.  dct_method: 0 islow, 1 ifast.  fancy: 0/1.
 * Returns 0 on success; writes w/h/components.  out must hold w*h*3 bytes
 * (call with out=NULL to query geometry only). */
int ljt_decode_scaled(const unsigned char *buf, unsigned long n, unsigned char *out,
                      int dct_method, int fancy, int scale_num, int scale_denom, int *w, int *h, int *ncomp);
int ljt_decode(const unsigned char *buf, unsigned long n, unsigned char *out,
               int dct_method, int fancy, int *w, int *h, int *ncomp) {
  return ljt_decode_scaled(buf, n, out, dct_method, fancy, 1, 1, w, h, ncomp);
}

/* As ljt_decode, with libjpeg's DCT scaling (scale_num / scale_denom: the
 * output size TurboJPEG's tjDecompress2 asks for at a scaling factor). */
int ljt_decode_scaled(const unsigned char *buf, unsigned long n, unsigned char *out,
                      int dct_method, int fancy, int scale_num, int scale_denom, int *w, int *h, int *ncomp) {
  if (!g_structsize) return -10;
  unsigned char *cinfo = (unsigned char *)calloc(1, 4096);
  err_wrap *ew = (err_wrap *)calloc(1, sizeof(err_wrap));
  unsigned char **rows = NULL;
  int rc = 0;
  p_std_error(ew->std);
  ((void **)ew->std)[0] = (void *)my_error_exit;
  ((void **)ew->std)[1] = (void *)my_emit;
  *(void **)(cinfo + OFF_ERR) = ew;
  if (setjmp(ew->jb) != 0) {
    rc = -1;
    goto done;
  }
  p_create(cinfo, 62, g_structsize);
  p_mem_src(cinfo, buf, n);
  p_read_header(cinfo, 1);
  *(int *)(cinfo + OFF_OUT_COLOR_SPACE) = JCS_RGB;
  *(int *)(cinfo + OFF_DCT_METHOD) = dct_method;
  *(int *)(cinfo + OFF_DO_FANCY) = fancy;
  *(unsigned *)(cinfo + OFF_SCALE_NUM) = (unsigned)scale_num;
  *(unsigned *)(cinfo + OFF_SCALE_DENOM) = (unsigned)scale_denom;
  *ncomp = *(int *)(cinfo + OFF_NUM_COMPONENTS);
  p_start(cinfo);
  *w = (int)*(unsigned *)(cinfo + OFF_OUTPUT_WIDTH);
  *h = (int)*(unsigned *)(cinfo + OFF_OUTPUT_HEIGHT);
  if (*(int *)(cinfo + OFF_OUTPUT_COMPONENTS) != 3) {
    rc = -2;
    goto done;
  }
  if (out) {
    rows = (unsigned char **)malloc(sizeof(unsigned char *) * (size_t)(*h));
    for (int y = 0; y < *h; y++) rows[y] = out + (size_t)y * (size_t)(*w) * 3;
    while (*(unsigned *)(cinfo + OFF_OUTPUT_SCANLINE) < (unsigned)*h) {
      unsigned line = *(unsigned *)(cinfo + OFF_OUTPUT_SCANLINE);
      p_read_scanlines(cinfo, rows + line, (unsigned)*h - line);
    }
    p_finish(cinfo);
  }
done:
  if (g_structsize) p_destroy(cinfo);
  free(rows);
  free(cinfo);
  free(ew);
  return rc;
}
