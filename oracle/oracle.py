"""ctypes front-end to the oracle (TEST INFRASTRUCTURE ONLY).

Only tests/, ``__graft_entry__.smoke()`` and bench.py's ``cpu_baseline`` leg
import this module, and only as the checker / reported CPU baseline.  The
product package ``ffcv_amd`` never imports it.

Everything here restates the reference path (see oracle/ffcv_oracle.c for the
file:line each function follows) or drives the third-party libjpeg-turbo that
the reference calls (oracle/ljt_harness.c).
"""
import ctypes
import os
import subprocess
import glob

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_BUILD = os.path.join(_HERE, 'build')


def build():
    subprocess.check_call(['make', '-s', '-C', _HERE])


def _load(name):
    path = os.path.join(_BUILD, name)
    if not os.path.exists(path):
        build()
    return ctypes.CDLL(path)


_lib = None
_ljt = None


def lib():
    global _lib
    if _lib is None:
        _lib = _load('liboracle.so')
        _lib.orc_sample_seed.restype = ctypes.c_uint32
        _lib.orc_sample_seed.argtypes = [ctypes.c_uint64, ctypes.c_uint64,
                                         ctypes.c_uint64, ctypes.c_uint32]
        _lib.orc_mt_u32.restype = ctypes.c_uint32
        _lib.orc_mt_double.restype = ctypes.c_double
        _lib.orc_uniform.restype = ctypes.c_double
        _lib.orc_uniform.argtypes = [ctypes.c_void_p, ctypes.c_double, ctypes.c_double]
        _lib.orc_randint.restype = ctypes.c_int64
        _lib.orc_randint.argtypes = [ctypes.c_void_p, ctypes.c_int64]
        _lib.orc_mt_seed.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
        _lib.orc_random_crop.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32,
                                         ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        _lib.orc_center_crop.argtypes = [ctypes.c_uint32, ctypes.c_uint32,
                                         ctypes.c_double, ctypes.c_void_p]
        _lib.orc_resize_crop.argtypes = [ctypes.c_void_p] + [ctypes.c_int64] * 6 + \
            [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64]
        _lib.orc_jpeg_decode.argtypes = [ctypes.c_void_p, ctypes.c_size_t,
                                         ctypes.c_void_p, ctypes.c_int]
        _lib.orc_jpeg_header.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
        _lib.orc_jpeg_coefficients.argtypes = [ctypes.c_void_p, ctypes.c_size_t,
                                               ctypes.c_void_p, ctypes.c_size_t,
                                               ctypes.c_void_p]
        _lib.orc_rrc_batch.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                       ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                       ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                       ctypes.c_void_p, ctypes.c_int]
        _lib.orc_set_jpeg_decoder.argtypes = [ctypes.c_void_p]
        _lib.orc_draw_batch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64,
                                        ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.c_double, ctypes.c_int, ctypes.c_int,
                                        ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    return _lib


def _ptr(a):
    return ctypes.c_void_p(a.ctypes.data) if a is not None else None


class MT:
    """numpy-legacy MT19937 (== numba per-thread generator)."""

    def __init__(self, seed):
        self.buf = (ctypes.c_uint8 * (624 * 4 + 16))()
        lib().orc_mt_seed(self.buf, seed)

    def u32(self):
        return lib().orc_mt_u32(self.buf)

    def uniform(self, lo, hi):
        return lib().orc_uniform(self.buf, lo, hi)

    def randint(self, high):
        return lib().orc_randint(self.buf, high)

    def random_crop(self, height, width, scale=(0.08, 1.0), ratio=(0.75, 4 / 3)):
        s = np.array(scale, np.float64)
        r = np.array(ratio, np.float64)
        out = np.zeros(4, np.int32)
        lib().orc_random_crop(self.buf, height, width, _ptr(s), _ptr(r), _ptr(out))
        return tuple(int(x) for x in out)


def sample_seed(loader_seed, epoch, sample, op_id):
    return lib().orc_sample_seed(loader_seed, epoch, sample, op_id)


def center_crop(height, width, ratio):
    out = np.zeros(4, np.int32)
    lib().orc_center_crop(height, width, ratio, _ptr(out))
    return tuple(int(x) for x in out)


def resize_crop(src, r0, r1, c0, c1, out_h, out_w):
    """libffcv.cpp:33-42 resize(): crop rows [r0,r1) cols [c0,c1) -> (out_h,out_w,3)."""
    src = np.ascontiguousarray(src, np.uint8)
    dst = np.zeros((out_h, out_w, 3), np.uint8)
    lib().orc_resize_crop(_ptr(src), src.shape[0], src.shape[1], r0, r1, c0, c1,
                          _ptr(dst), out_h, out_w)
    return dst


class JpegInfo(ctypes.Structure):
    _fields_ = [('width', ctypes.c_int), ('height', ctypes.c_int), ('ncomp', ctypes.c_int),
                ('hmax', ctypes.c_int), ('vmax', ctypes.c_int),
                ('h', ctypes.c_int * 4), ('v', ctypes.c_int * 4), ('tq', ctypes.c_int * 4),
                ('td', ctypes.c_int * 4), ('ta', ctypes.c_int * 4),
                ('restart_interval', ctypes.c_int), ('sof', ctypes.c_int),
                ('scan_off', ctypes.c_size_t), ('scan_end', ctypes.c_size_t)]


def jpeg_header(data):
    data = np.frombuffer(bytes(data), np.uint8) if not isinstance(data, np.ndarray) else data
    info = JpegInfo()
    rc = lib().orc_jpeg_header(_ptr(data), data.size, ctypes.byref(info))
    return rc, info


def jpeg_decode(data, dct='ifast'):
    """Restatement of tjDecompress2(TJPF_RGB, TJFLAG_FASTDCT) (libffcv.cpp:104-106)."""
    data = np.frombuffer(bytes(data), np.uint8) if not isinstance(data, np.ndarray) else data
    rc, info = jpeg_header(data)
    if rc:
        raise ValueError(f'oracle jpeg header error {rc}')
    out = np.zeros((info.height, info.width, 3), np.uint8)
    rc = lib().orc_jpeg_decode(_ptr(data), data.size, _ptr(out), 1 if dct == 'ifast' else 0)
    if rc:
        raise ValueError(f'oracle jpeg decode error {rc}')
    return out


def jpeg_coefficients(data):
    data = np.frombuffer(bytes(data), np.uint8) if not isinstance(data, np.ndarray) else data
    rc, info = jpeg_header(data)
    maxb = ((info.width + 8 * info.hmax - 1) // (8 * info.hmax) + 1) * \
        ((info.height + 8 * info.vmax - 1) // (8 * info.vmax) + 1) * 16
    out = np.zeros((maxb, 64), np.int16)
    n = ctypes.c_size_t()
    rc = lib().orc_jpeg_coefficients(_ptr(data), data.size, _ptr(out), maxb, ctypes.byref(n))
    if rc:
        raise ValueError(f'oracle jpeg error {rc}')
    return out[:n.value]


class Sample(ctypes.Structure):
    _fields_ = [('data', ctypes.c_void_p), ('size', ctypes.c_uint64),
                ('height', ctypes.c_uint32), ('width', ctypes.c_uint32),
                ('mode', ctypes.c_uint8)]


def rrc_batch(samples, crops, out_h, out_w, cutout_yx=None, cutout_size=0,
              fill=(0, 0, 0), lut=None, nthreads=1):
    """rgb_image.py:185-210 + cutout.py:36-47 + normalize LUT over a batch.

    samples: list of (np.uint8 array, height, width, mode)."""
    n = len(samples)
    arr = (Sample * n)()
    keep = []
    for k, (data, h, w, mode) in enumerate(samples):
        data = np.ascontiguousarray(data, np.uint8)
        keep.append(data)
        arr[k] = Sample(data.ctypes.data, data.size, h, w, mode)
    crops = np.ascontiguousarray(crops, np.int32)
    fill_a = np.array(fill, np.uint8)
    if lut is not None:
        lut = np.ascontiguousarray(lut).view(np.uint16)
        out = np.zeros((n, out_h, out_w, 3), np.uint16)
    else:
        out = np.zeros((n, out_h, out_w, 3), np.uint8)
    cut = np.ascontiguousarray(cutout_yx, np.int32) if cutout_yx is not None else None
    rc = lib().orc_rrc_batch(arr, n, _ptr(crops), out_h, out_w, _ptr(cut), cutout_size,
                             _ptr(fill_a), _ptr(lut), _ptr(out), nthreads)
    if rc:
        raise ValueError(f'oracle batch error {rc}')
    return out if lut is None else out.view(np.float16)


def draw_batch(ids, heights, widths, loader_seed, epoch, crop='random',
               scale=(0.08, 1.0), ratio=(0.75, 4 / 3), center_ratio=224 / 256,
               out_h=224, out_w=224, cutout_size=0):
    ids = np.ascontiguousarray(ids, np.uint64)
    hs = np.ascontiguousarray(heights, np.uint32)
    ws = np.ascontiguousarray(widths, np.uint32)
    n = ids.size
    crops = np.zeros((n, 4), np.int32)
    cut = np.zeros((n, 2), np.int32) if cutout_size else None
    s = np.array(scale, np.float64)
    r = np.array(ratio, np.float64)
    lib().orc_draw_batch(_ptr(ids), _ptr(hs), _ptr(ws), n, loader_seed, epoch,
                         0 if crop == 'random' else 1, _ptr(s), _ptr(r), center_ratio,
                         out_h, out_w, cutout_size, _ptr(crops), _ptr(cut))
    return crops, cut


def normalize_lut(mean, std, dtype=np.float16):
    """normalize.py:42-49 verbatim arithmetic: f64 table -> dtype."""
    table = (np.arange(256)[:, None] - np.asarray(mean)[None, :]) / np.asarray(std)[None, :]
    return table.astype(dtype)


# ---------------------------------------------------------------- libjpeg-turbo
def pillow_libjpeg_path():
    import PIL
    d = os.path.join(os.path.dirname(os.path.dirname(PIL.__file__)), 'pillow.libs')
    cands = sorted(glob.glob(os.path.join(d, 'libjpeg-*.so*')))
    return cands[0] if cands else None


def ljt():
    """Third-party libjpeg-turbo (Pillow-bundled) through oracle/ljt_harness.c."""
    global _ljt
    if _ljt is None:
        path = pillow_libjpeg_path()
        if path is None:
            return None
        l = _load('libljt.so')
        l.ljt_decode.argtypes = [ctypes.c_void_p, ctypes.c_ulong, ctypes.c_void_p,
                                 ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                 ctypes.c_void_p, ctypes.c_void_p]
        l.ljt_decode_scaled.argtypes = [ctypes.c_void_p, ctypes.c_ulong, ctypes.c_void_p,
                                        ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        if l.ljt_open(path.encode()) != 0:
            return None
        _ljt = l
    return _ljt


def use_libjpeg_turbo(enable=True):
    """Route rrc_batch's JPEG decode through libjpeg-turbo itself (SIMD,
    ifast + fancy) instead of the restatement; returns whether it is on."""
    l = ljt() if enable else None
    fn = ctypes.cast(l.ljt_decode, ctypes.c_void_p) if l is not None else None
    lib().orc_set_jpeg_decoder(fn)
    return l is not None


def ljt_decode(data, dct='ifast', fancy=True, scale=(1, 1)):
    """tjDecompress2(TJPF_RGB, TJFLAG_FASTDCT) semantics via libjpeg-turbo itself
    (scale: libjpeg's scale_num / scale_denom, TurboJPEG's scaling factor)."""
    l = ljt()
    data = bytes(data)
    w, h, nc = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    buf = ctypes.create_string_buffer(data, len(data))
    m = 1 if dct == 'ifast' else 0
    rc = l.ljt_decode_scaled(buf, len(data), None, m, int(fancy), int(scale[0]), int(scale[1]),
                             ctypes.byref(w), ctypes.byref(h), ctypes.byref(nc))
    if rc:
        raise ValueError(f'libjpeg error {rc}')
    out = np.zeros((h.value, w.value, 3), np.uint8)
    rc = l.ljt_decode_scaled(buf, len(data), ctypes.c_void_p(out.ctypes.data), m, int(fancy),
                             int(scale[0]), int(scale[1]), ctypes.byref(w), ctypes.byref(h), ctypes.byref(nc))
    if rc:
        raise ValueError(f'libjpeg error {rc}')
    return out
