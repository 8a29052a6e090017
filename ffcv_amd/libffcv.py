"""ctypes binding of ``libffcv_hip.so`` (include/ffcv_hip.h).

Replaces the reference's ``ffcv/libffcv.py`` (CDLL of ``ffcv._libffcv``,
ffcv/libffcv.py:8-55).  The reference binds one-sample CPU functions
(``resize``, ``imdecode``, ``my_memcpy``) called from numba ``prange``
workers.  This binding exposes the batch/device ABI: every call enqueues HIP
work on the caller's stream (``torch.cuda.current_stream().cuda_stream`` is a
``hipStream_t`` on ROCm) and takes device pointers (``tensor.data_ptr()``).

The library is built in-tree (``python -m ffcv_amd._build``).  There is no CPU
fallback for any compute entry point: if the shared object is missing this
module raises at import of the compute functions.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, 'libffcv_hip.so')

c_void_p = ctypes.c_void_p
c_int = ctypes.c_int
c_int32 = ctypes.c_int32
c_uint32 = ctypes.c_uint32
c_uint64 = ctypes.c_uint64

# per-sample device status codes (FFCV_SAMPLE_*)
SAMPLE_STATUS = {0: 'ok', 1: 'bad marker', 2: 'unsupported JPEG feature',
                 3: 'image larger than decoder context', 4: 'corrupt entropy stream',
                 5: 'geometry mismatch', 6: 'rng stream exhausted'}


class FFCVError(RuntimeError):
    pass


class Sample(ctypes.Structure):
    """ffcv_sample (32 bytes)."""
    _fields_ = [('offset', c_uint64), ('size', c_uint64), ('height', c_uint32),
                ('width', c_uint32), ('mode', c_uint32), ('reserved', c_uint32)]


SAMPLE_DTYPE = np.dtype([('offset', '<u8'), ('size', '<u8'), ('height', '<u4'),
                         ('width', '<u4'), ('mode', '<u4'), ('reserved', '<u4')])
assert SAMPLE_DTYPE.itemsize == ctypes.sizeof(Sample) == 32


class RRCParams(ctypes.Structure):
    _fields_ = [('out_h', c_int32), ('out_w', c_int32), ('cutout_size', c_int32),
                ('cutout_fill', ctypes.c_uint8 * 4), ('lut', c_void_p),
                ('out_stride', c_uint64)]


class DrawParams(ctypes.Structure):
    _fields_ = [('crop_kind', c_int32), ('out_h', c_int32), ('out_w', c_int32),
                ('cutout_size', c_int32), ('scale', ctypes.c_double * 2),
                ('ratio', ctypes.c_double * 2), ('center_ratio', ctypes.c_double),
                ('loader_seed', c_uint64), ('epoch', c_uint64),
                ('flip_prob', ctypes.c_double)]


_lib = None

_SIGS = {
    'ffcv_abi_version': (c_int, []),
    'ffcv_last_error': (ctypes.c_char_p, []),
    'ffcv_device_count': (c_int, [c_void_p]),
    'ffcv_set_device': (c_int, [c_int]),
    'ffcv_stream_synchronize': (c_int, [c_void_p]),
    'ffcv_malloc': (c_int, [c_void_p, c_uint64]),
    'ffcv_free': (c_int, [c_void_p]),
    'ffcv_memcpy_h2d_async': (c_int, [c_void_p, c_void_p, c_uint64, c_void_p]),
    'ffcv_memcpy_d2h_async': (c_int, [c_void_p, c_void_p, c_uint64, c_void_p]),
    'my_memcpy': (None, [c_void_p, c_void_p, c_uint64]),
    'my_fread': (None, [ctypes.c_int64, ctypes.c_int64, c_void_p, ctypes.c_int64]),
    'resize': (None, [ctypes.c_int64] * 11),
    'imdecode': (c_int, [c_void_p, c_uint64, c_uint32, c_uint32, c_void_p, c_uint32, c_uint32,
                         c_uint32, c_uint32, c_uint32, c_uint32, ctypes.c_bool, ctypes.c_bool]),
    'ffcv_cpu_decode_batch': (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_int,
                                      c_int, c_void_p, c_uint64, c_int, c_void_p]),
    'ffcv_imdecode_device': (c_int, [c_void_p, c_uint64, c_uint32, c_uint32, c_void_p, c_uint32, c_uint32,
                                     c_uint32, c_uint32, c_uint32, c_uint32, ctypes.c_bool, ctypes.c_bool]),
    'ffcv_host_gather': (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_int]),
    'ffcv_draw_batch': (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p,
                                c_void_p, c_void_p, c_void_p]),
    'ffcv_draw_batch_host': (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p,
                                     c_void_p]),
    'ffcv_rrc_raw_batch': (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p,
                                   c_void_p, c_void_p, c_void_p]),
    'ffcv_rrc_raw_batch_ws': (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p,
                                      c_void_p, c_void_p, c_void_p, c_void_p, c_uint64]),
    'ffcv_rrc_raw_workspace_bytes': (c_uint64, [c_int, c_int, c_int]),
    'ffcv_gather_samples': (c_int, [c_void_p, c_void_p, c_uint64, c_void_p, c_int, c_void_p]),
    'ffcv_gather_raw_batch': (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_uint64]),
    'ffcv_jpeg_scan_stats': (c_int, [c_void_p, c_void_p, c_int, c_void_p]),
    'ffcv_jpeg_create': (c_int, [c_void_p, c_int, c_uint32, c_uint32, c_uint64]),
    'ffcv_jpeg_destroy': (c_int, [c_void_p]),
    'ffcv_jpeg_create_arena': (c_int, [c_void_p, c_int, c_uint32, c_uint32, c_uint64, c_uint64]),
    'ffcv_jpeg_scratch_bound': (c_uint64, [c_uint32, c_uint32, c_uint64]),
    'ffcv_jpeg_set_diag': (c_int, [c_void_p, c_int, c_int]),
    'ffcv_jpeg_arena_used': (c_int, [c_void_p, c_void_p, c_void_p, c_void_p]),
    'ffcv_jpeg_set_entropy_index': (c_int, [c_void_p, c_void_p, c_uint64]),
    'ffcv_jpeg_set_timing': (c_int, [c_void_p, c_int]),
    'ffcv_jpeg_timing_read': (c_int, [c_void_p, c_void_p, c_int, c_void_p]),
    'ffcv_jpeg_rrc_batch': (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p,
                                    c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    'ffcv_jpeg_rrc_fused': (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_uint64, c_void_p,
                                    c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                    c_void_p, c_void_p, c_void_p]),
    'ffcv_jpeg_decode_batch': (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p,
                                       c_uint64, c_void_p]),
    'ffcv_jpeg_coefficients_batch': (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int,
                                             c_void_p, c_uint64, c_void_p]),
    'ffcv_cutout_batch': (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_int,
                                  c_void_p]),
    'ffcv_normalize_batch': (c_int, [c_void_p, c_void_p, c_uint64, c_void_p, c_void_p]),
    'ffcv_lut_batch': (c_int, [c_void_p, c_void_p, c_uint64, c_void_p, c_int, c_void_p]),
    'ffcv_flip_batch': (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int,
                                c_void_p]),
}

EXPORTED_SYMBOLS = tuple(_SIGS)


def lib():
    """Load libffcv_hip.so (raises if it was not built -- no CPU fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise FFCVError(f'{LIB_PATH} is missing: build it with `python -m ffcv_amd._build` '
                            '(there is no CPU fallback for the decode path)')
        # Load torch's HIP runtime first: libffcv_hip.so's NEEDED
        # libamdhip64.so.7 then binds to the runtime torch already uses
        # (same soname), so tensors and our kernels share one HIP runtime.
        # Loading ours first would pull /opt/rocm's copy and give the process
        # two runtimes ("no ROCm-capable device" in the second).
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        l = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            f = getattr(l, name)
            f.restype = res
            f.argtypes = args
        if l.ffcv_abi_version() != 1:
            raise FFCVError('libffcv_hip.so ABI version mismatch')
        _lib = l
    return _lib


def _check(rc, what):
    if rc != 0:
        msg = lib().ffcv_last_error().decode(errors='replace')
        raise FFCVError(f'{what} failed ({rc}): {msg}')


def _p(x):
    """Device/host pointer of a torch tensor, numpy array, int or None."""
    if x is None:
        return None
    if isinstance(x, int):
        return c_void_p(x)
    if hasattr(x, 'data_ptr'):
        return c_void_p(x.data_ptr())
    if isinstance(x, np.ndarray):
        return c_void_p(x.ctypes.data)
    raise TypeError(type(x))


def _stream(stream):
    if stream is None:
        import torch
        stream = torch.cuda.current_stream()
    return c_void_p(stream.cuda_stream if hasattr(stream, 'cuda_stream') else int(stream))


# ----------------------------------------------------------------- wrappers
def memcpy_h2d_async(dst, src, nbytes: int, stream):
    """hipMemcpyAsync host -> device on ``stream`` (pinned ``src``): one
    library call instead of a torch copy dispatch inside a stream context."""
    _check(lib().ffcv_memcpy_h2d_async(_p(dst), _p(src), int(nbytes), _stream(stream)), 'ffcv_memcpy_h2d_async')


def memcpy_d2h_async(dst, src, nbytes: int, stream):
    """hipMemcpyAsync device -> host on ``stream`` (pinned ``dst``)."""
    _check(lib().ffcv_memcpy_d2h_async(_p(dst), _p(src), int(nbytes), _stream(stream)), 'ffcv_memcpy_d2h_async')


def memcpy(source: np.ndarray, dest: np.ndarray):
    """ffcv/libffcv.py:51-55 memcpy (host plumbing)."""
    lib().my_memcpy(source.ctypes.data, dest.ctypes.data, source.size * source.itemsize)


# --------------------------------------- reference one-sample host API --
# ffcv/libffcv.py:11-48: read (libc pread), resize_crop, imdecode, same
# names and argument meaning, for Operations written against the reference.
_libc = None


def read(fileno: int, destination: np.ndarray, offset: int):
    """pread(fileno, destination, destination.size, offset) (libffcv.py:11-19)."""
    global _libc
    if _libc is None:
        _libc = ctypes.CDLL('libc.so.6', use_errno=True)
        _libc.pread.restype = ctypes.c_ssize_t
        _libc.pread.argtypes = [c_int, c_void_p, ctypes.c_size_t, ctypes.c_int64]
    return _libc.pread(int(fileno), destination.ctypes.data, destination.size, int(offset))


def resize_crop(source, start_row, end_row, start_col, end_col, destination):
    """INTER_AREA resize of source[start_row:end_row, start_col:end_col]
    (HWC uint8) into destination (its shape is the target), libffcv.py:22-31."""
    source = np.asarray(source)
    if source.dtype != np.uint8 or destination.dtype != np.uint8 or not source.flags.c_contiguous \
            or not destination.flags.c_contiguous:
        raise ValueError('resize_crop: source and destination must be C-contiguous uint8 HWC arrays')
    lib().resize(0, source.ctypes.data, source.shape[0], source.shape[1], int(start_row), int(end_row),
                 int(start_col), int(end_col), destination.ctypes.data, destination.shape[0],
                 destination.shape[1])


def imdecode(source: np.ndarray, dst: np.ndarray, source_height: int, source_width: int,
             crop_height=None, crop_width=None, offset_x=0, offset_y=0, scale_factor_num=1,
             scale_factor_denom=1, enable_crop=False, do_flip=False):
    """Decode one JPEG (host bytes) into dst (host HWC uint8), libffcv.py:34-48,
    on the CPU like the reference.  Returns 0 or -1 like tjDecompress2."""
    return _imdecode(lib().imdecode, source, dst, source_height, source_width, crop_height, crop_width,
                     offset_x, offset_y, scale_factor_num, scale_factor_denom, enable_crop, do_flip)


def imdecode_device(source: np.ndarray, dst: np.ndarray, source_height: int, source_width: int,
                    crop_height=None, crop_width=None, offset_x=0, offset_y=0, scale_factor_num=1,
                    scale_factor_denom=1, enable_crop=False, do_flip=False):
    """imdecode executed by the gfx950 JPEG kernels (host buffers in and out)."""
    return _imdecode(lib().ffcv_imdecode_device, source, dst, source_height, source_width, crop_height,
                     crop_width, offset_x, offset_y, scale_factor_num, scale_factor_denom, enable_crop, do_flip)


def _imdecode(fn, source, dst, source_height, source_width, crop_height, crop_width, offset_x, offset_y,
              scale_factor_num, scale_factor_denom, enable_crop, do_flip):
    if crop_height is None:
        crop_height = source_height
    if crop_width is None:
        crop_width = source_width
    return fn(source.ctypes.data, source.size, int(source_height), int(source_width),
              dst.ctypes.data, int(crop_height), int(crop_width), int(offset_x), int(offset_y),
              int(scale_factor_num), int(scale_factor_denom), bool(enable_crop), bool(do_flip))


def jpeg_scan_stats(images):
    """(symbols, blocks, entropy-coded bytes) per JPEG, uint64 (n, 3), from the
    CPU decoder's Huffman loop (ffcv_jpeg_scan_stats); rows of images that
    do not parse are zero."""
    images = [np.ascontiguousarray(im, dtype=np.uint8) for im in images]
    n = len(images)
    ptrs = np.array([im.ctypes.data for im in images], dtype=np.uint64)
    sizes = np.array([im.size for im in images], dtype=np.uint64)
    stats = np.zeros((max(n, 1), 3), dtype=np.uint64)
    rc = lib().ffcv_jpeg_scan_stats(ptrs.ctypes.data, sizes.ctypes.data, n, stats.ctypes.data)
    if rc not in (0, -1):
        raise RuntimeError('ffcv_jpeg_scan_stats: ' + lib().ffcv_last_error().decode(errors='replace'))
    return stats[:n]


def cpu_decode_batch(images, heights, widths, modes, out: np.ndarray, crops=None, nthreads=1):
    """The reference's per-sample CPU decode loop as one native call
    (ffcv_cpu_decode_batch): images[k] are host uint8 arrays (JPEG bytes or
    raw HWC pixels), out is [B, ...] C-contiguous uint8 (the sample's whole
    image, or its crops[k] resized to out.shape[1:3]).  Returns the status
    array (0 / -1 per sample)."""
    B = len(images)
    ptrs = np.array([im.ctypes.data if im is not None else 0 for im in images], np.uint64)
    sizes = np.array([im.size if im is not None else 0 for im in images], np.uint64)
    hs = np.ascontiguousarray(heights, np.uint32)
    ws = np.ascontiguousarray(widths, np.uint32)
    ms = np.ascontiguousarray(modes, np.uint32)
    status = np.zeros(B, np.int32)
    if not out.flags['C_CONTIGUOUS'] or out.dtype != np.uint8:
        raise ValueError('cpu_decode_batch: out must be C-contiguous uint8')
    stride = out[0].nbytes if B else 0
    cr = None
    oh = ow = 0
    if crops is not None:
        cr = np.ascontiguousarray(crops, np.int32)
        oh, ow = int(out.shape[1]), int(out.shape[2])
    rc = lib().ffcv_cpu_decode_batch(ptrs.ctypes.data, sizes.ctypes.data, hs.ctypes.data, ws.ctypes.data,
                                     ms.ctypes.data, B, cr.ctypes.data if cr is not None else None, oh, ow,
                                     out.ctypes.data, stride, int(max(1, nthreads)), status.ctypes.data)
    if rc != 0:
        raise RuntimeError('ffcv_cpu_decode_batch: ' + lib().ffcv_last_error().decode(errors='replace'))
    return status


def host_gather(src: np.ndarray, src_off: np.ndarray, sizes: np.ndarray, dst_off: np.ndarray, dst,
                nthreads=8):
    """Gather byte ranges of a host buffer (e.g. the mmap) into dst (numpy / pinned tensor)."""
    so = np.ascontiguousarray(src_off, dtype=np.uint64)
    sz = np.ascontiguousarray(sizes, dtype=np.uint64)
    do = np.ascontiguousarray(dst_off, dtype=np.uint64)
    _check(lib().ffcv_host_gather(_p(src), _p(so), _p(sz), _p(do), int(len(sz)), _p(dst), int(nthreads)),
           'ffcv_host_gather')


def draw_batch(ids, samples, params: DrawParams, crops=None, cutout_yx=None, flips=None,
               status=None, stream=None):
    _check(lib().ffcv_draw_batch(_stream(stream), _p(ids), _p(samples), int(ids.shape[0]),
                                 ctypes.byref(params), _p(crops), _p(cutout_yx), _p(flips),
                                 _p(status)), 'ffcv_draw_batch')


def draw_batch_host(ids, heights, widths, params: DrawParams, crops=None, cutout_yx=None, flips=None):
    """ffcv_draw_batch on host arrays (the CPU-device decoders' draws)."""
    ids = np.ascontiguousarray(ids, dtype=np.uint64)
    hs = np.ascontiguousarray(heights, dtype=np.uint32) if heights is not None else None
    ws = np.ascontiguousarray(widths, dtype=np.uint32) if widths is not None else None
    _check(lib().ffcv_draw_batch_host(_p(ids), _p(hs), _p(ws), int(ids.size), ctypes.byref(params), _p(crops),
                                      _p(cutout_yx), _p(flips)), 'ffcv_draw_batch_host')


def gather_samples(table, ids, out, stream=None):
    _check(lib().ffcv_gather_samples(_stream(stream), _p(table), int(table.shape[0]), _p(ids),
                                     int(ids.shape[0]), _p(out)), 'ffcv_gather_samples')


def rrc_raw_workspace_bytes(batch, out_h, out_w):
    """Device bytes rrc_raw_batch's workspace needs (per-image plan + taps)."""
    return int(lib().ffcv_rrc_raw_workspace_bytes(int(batch), int(out_h), int(out_w)))


def rrc_raw_batch(base, samples, batch, crops, cutout_yx, flips, params: RRCParams, out,
                  stream=None, workspace=None):
    """Raw-mode RRC (+ cutout / flip / LUT).  With a device uint8 `workspace`
    of rrc_raw_workspace_bytes() the per-image plans and tap tables are
    computed once per image (ffcv_rrc_raw_batch_ws); output is identical."""
    if workspace is not None:
        _check(lib().ffcv_rrc_raw_batch_ws(_stream(stream), _p(base), _p(samples), int(batch),
                                           _p(crops), _p(cutout_yx), _p(flips), ctypes.byref(params),
                                           _p(out), _p(workspace), int(workspace.numel())),
               'ffcv_rrc_raw_batch_ws')
        return
    _check(lib().ffcv_rrc_raw_batch(_stream(stream), _p(base), _p(samples), int(batch),
                                    _p(crops), _p(cutout_yx), _p(flips), ctypes.byref(params),
                                    _p(out)), 'ffcv_rrc_raw_batch')


def gather_raw_batch(base, samples, batch, out, out_stride, stream=None):
    _check(lib().ffcv_gather_raw_batch(_stream(stream), _p(base), _p(samples), int(batch),
                                       _p(out), int(out_stride)), 'ffcv_gather_raw_batch')


def cutout_batch(images, yx, crop_size, fill, stream=None):
    B, H, W = int(images.shape[0]), int(images.shape[1]), int(images.shape[2])
    f = (ctypes.c_uint8 * 3)(*[int(x) for x in fill])
    _check(lib().ffcv_cutout_batch(_stream(stream), _p(images), B, H, W, _p(yx), int(crop_size),
                                   f), 'ffcv_cutout_batch')


def normalize_batch(inp, lut, out, stream=None):
    _check(lib().ffcv_normalize_batch(_stream(stream), _p(inp), int(inp.numel()), _p(lut),
                                      _p(out)), 'ffcv_normalize_batch')


def lut_batch(inp, lut, out, stream=None):
    """out[i] = lut[inp[i]*3 + i%3] for a [256,3] device table of any dtype
    (element size 1/2/4/8)."""
    _check(lib().ffcv_lut_batch(_stream(stream), _p(inp), int(inp.numel()), _p(lut),
                                int(lut.element_size()), _p(out)), 'ffcv_lut_batch')


def flip_batch(inp, out, flips, stream=None):
    B, H, W = int(inp.shape[0]), int(inp.shape[1]), int(inp.shape[2])
    cb = int(inp[0, 0, 0].numel() * inp.element_size())
    _check(lib().ffcv_flip_batch(_stream(stream), _p(inp), _p(out), B, H, W, cb, _p(flips)),
           'ffcv_flip_batch')


def scratch_bound(heights, widths, nbytes):
    """ffcv_jpeg_scratch_bound over arrays (numpy restatement of the C
    formula, checked against it in tests/test_abi.py): the most arena bytes
    one image can take, whatever its crop."""
    h = np.asarray(heights, dtype=np.uint64)
    w = np.asarray(widths, dtype=np.uint64)
    n = np.asarray(nbytes, dtype=np.uint64)

    def a256(x):
        return (x + np.uint64(255)) // np.uint64(256) * np.uint64(256)
    blocks = np.uint64(3) * ((w + np.uint64(7)) // np.uint64(8) + np.uint64(4)) * \
        ((h + np.uint64(7)) // np.uint64(8) + np.uint64(4))
    return (a256(n + np.uint64(64)) + a256(blocks * np.uint64(128)) + a256(blocks * np.uint64(2)) +
            a256(blocks * np.uint64(64)) + a256(h * w * np.uint64(3)))


def arena_for(heights, widths, nbytes, max_batch):
    """Arena bytes that no launch of max_batch images of this dataset can
    exhaust: the sum of the max_batch largest per-image bounds."""
    b = scratch_bound(heights, widths, nbytes)
    if max_batch <= 0:
        return 4096
    if b.size > max_batch:
        b = np.partition(b, b.size - max_batch)[b.size - max_batch:]
    # fewer images than a launch (repeated samples: a small dataset, padded
    # distributed orders, replicated benchmark encodings): each extra slot
    # may hold the largest image again
    extra = max(0, max_batch - b.size) * (int(b.max()) if b.size else 0)
    return int(b.sum()) + extra + 4096


EIDX_LANES, EIDX_WORDS = 64, 3  # entropy index record: words per lane range


class JpegDecoder:
    """Owns an ffcv_jpeg_ctx: launch scratch for up to max_batch images in
    one arena of arena_bytes (default: max_batch images of the maximum size)."""

    def __init__(self, max_batch, max_height, max_width, max_bytes, arena_bytes=0):
        self.handle = c_void_p()
        self.max_batch = int(max_batch)
        self.max_height, self.max_width = int(max_height), int(max_width)
        self.max_bytes = int(max_bytes)
        self.arena_bytes = int(arena_bytes)
        _check(lib().ffcv_jpeg_create_arena(ctypes.byref(self.handle), self.max_batch,
                                            self.max_height, self.max_width, self.max_bytes,
                                            self.arena_bytes), 'ffcv_jpeg_create')

    def rrc(self, base, samples, batch, crops, cutout_yx, flips, params: RRCParams, out,
            status, stream=None):
        _check(lib().ffcv_jpeg_rrc_batch(self.handle, _stream(stream), _p(base), _p(samples),
                                         int(batch), _p(crops), _p(cutout_yx), _p(flips),
                                         ctypes.byref(params), _p(out), _p(status)),
               'ffcv_jpeg_rrc_batch')

    def rrc_fused(self, base, table, ids, draw: DrawParams, crops, cutout_yx, flips,
                  params: RRCParams, out, status, samples_out=None, stream=None):
        """gather + draws + decode/crop/resize/epilogue (ffcv_jpeg_rrc_fused)."""
        _check(lib().ffcv_jpeg_rrc_fused(self.handle, _stream(stream), _p(base), _p(table),
                                         table.numel() // 32, _p(ids), int(ids.shape[0]),
                                         ctypes.byref(draw), _p(crops), _p(cutout_yx), _p(flips),
                                         _p(samples_out), ctypes.byref(params), _p(out),
                                         _p(status)), 'ffcv_jpeg_rrc_fused')

    def decode(self, base, samples, batch, out, out_stride, status, stream=None):
        _check(lib().ffcv_jpeg_decode_batch(self.handle, _stream(stream), _p(base), _p(samples),
                                            int(batch), _p(out), int(out_stride), _p(status)),
               'ffcv_jpeg_decode_batch')

    def set_diag(self, only=7):
        """Diagnostics: kernels a launch runs (bit 0 K1, bit 1 the IDCT
        kernel, bit 2 K2), fixed on this context (never read per launch).  The
        C entry point's third argument (the K2 timing-only flags of rounds
        1-4) must be 0 and is always passed as 0 here."""
        _check(lib().ffcv_jpeg_set_diag(self.handle, int(only), 0), 'ffcv_jpeg_set_diag')

    def arena_used(self, stream=None):
        """(bytes the last entropy launch allocated, arena capacity)."""
        used, cap = c_uint64(), c_uint64()
        _check(lib().ffcv_jpeg_arena_used(self.handle, _stream(stream), ctypes.byref(used), ctypes.byref(cap)),
               'ffcv_jpeg_arena_used')
        return used.value, cap.value

    def set_entropy_index(self, index):
        """Attach (or, with None, detach) an entropy index: a zeroed uint32
        device tensor of shape (n_samples, 64, 3) that fused launches fill
        and then use to skip the Huffman sync of samples decoded before."""
        if index is None:
            _check(lib().ffcv_jpeg_set_entropy_index(self.handle, None, 0), 'ffcv_jpeg_set_entropy_index')
            self._eidx = None
            return
        if index.dim() != 3 or tuple(index.shape[1:]) != (EIDX_LANES, EIDX_WORDS) or \
                index.element_size() != 4 or not index.is_contiguous() or not index.is_cuda:
            raise ValueError('entropy index must be a contiguous 4-byte device tensor of shape '
                             f'(n, {EIDX_LANES}, {EIDX_WORDS})')
        _check(lib().ffcv_jpeg_set_entropy_index(self.handle, _p(index), int(index.shape[0])),
               'ffcv_jpeg_set_entropy_index')
        self._eidx = index  # keep it alive while attached

    def set_timing(self, max_launches):
        """Record HIP events around each kernel of the next max_launches RRC
        launches (0: off); timing_read() returns their durations."""
        self._tcap = int(max_launches)
        _check(lib().ffcv_jpeg_set_timing(self.handle, self._tcap), 'ffcv_jpeg_set_timing')

    def timing_read(self):
        """ms[launch, kernel] (kernel 0 entropy, 1 IDCT, 2 colour/resize) of
        the launches recorded since set_timing / the last read."""
        cap = getattr(self, '_tcap', 0)
        ms = np.zeros((max(1, cap), 3), np.float32)
        n = c_int()
        _check(lib().ffcv_jpeg_timing_read(self.handle, _p(ms), cap, ctypes.byref(n)), 'ffcv_jpeg_timing_read')
        return ms[:n.value]

    def coefficients(self, base, samples, batch, out, max_blocks, status, stream=None):
        _check(lib().ffcv_jpeg_coefficients_batch(self.handle, _stream(stream), _p(base),
                                                  _p(samples), int(batch), _p(out),
                                                  int(max_blocks), _p(status)),
               'ffcv_jpeg_coefficients_batch')

    def close(self):
        if self.handle:
            lib().ffcv_jpeg_destroy(self.handle)
            self.handle = c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
