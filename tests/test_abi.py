"""The C-ABI library builds for gfx950, loads, and exports every function
include/ffcv_hip.h declares (CPU: no compute calls)."""
import ctypes

import numpy as np
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    src = open(os.path.join(ROOT, 'include', 'ffcv_hip.h')).read()
    src = re.sub(r'/\*.*?\*/', '', src, flags=re.S)
    names = re.findall(r'^\s*(?:const\s+)?[a-z_0-9]+\s*\*?\s*([a-z_][a-z_0-9]*)\s*\(', src, flags=re.M)
    return sorted(set(n for n in names if n not in ('sizeof',)))


def test_header_declares_expected_entry_points():
    names = declared_functions()
    for must in ['ffcv_jpeg_rrc_batch', 'ffcv_rrc_raw_batch', 'ffcv_draw_batch', 'my_memcpy',
                 'ffcv_jpeg_create', 'ffcv_last_error', 'ffcv_normalize_batch']:
        assert must in names


def test_library_exports_every_declared_symbol(hip_lib):
    lib = ctypes.CDLL(os.path.join(ROOT, 'ffcv_amd', 'libffcv_hip.so'))
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, missing
    assert hip_lib.ffcv_abi_version() == 1
    from ffcv_amd import libffcv
    assert set(declared_functions()) <= set(libffcv.EXPORTED_SYMBOLS) | {'ffcv_jpeg_set_debug'}


def test_code_object_is_gfx950(hip_lib):
    data = open(os.path.join(ROOT, 'ffcv_amd', 'libffcv_hip.so'), 'rb').read()
    assert b'gfx950' in data


def test_host_memcpy_and_errors(hip_lib):
    import numpy as np
    from ffcv_amd import libffcv
    a = np.arange(100, dtype=np.uint8)
    b = np.zeros(100, np.uint8)
    libffcv.memcpy(a, b)
    assert np.array_equal(a, b)
    # argument validation happens before any device call
    rc = hip_lib.ffcv_rrc_raw_batch(None, None, None, 1, None, None, None, None, None)
    assert rc == -1 and b'invalid' in hip_lib.ffcv_last_error()
    rc = hip_lib.ffcv_jpeg_create(None, 0, 0, 0, 0)
    assert rc == -1


def test_host_gather_cpu():
    """ffcv_host_gather (the PCIe path's batch staging) on host memory only."""
    from ffcv_amd import libffcv as L
    rng = np.random.default_rng(0)
    src = rng.integers(0, 256, 100000).astype(np.uint8)
    so = rng.integers(0, 90000, 40).astype(np.uint64)
    sizes = np.minimum(rng.integers(0, 3000, 40).astype(np.uint64), np.uint64(100000) - so)
    sizes[3] = 0
    do = np.zeros(40, np.uint64)
    do[1:] = np.cumsum(sizes)[:-1]
    for nt in (1, 3, 8):
        dst = np.zeros(int(sizes.sum()) + 16, np.uint8)
        L.host_gather(src, so, sizes, do, dst, nthreads=nt)
        for i in range(40):
            assert np.array_equal(dst[int(do[i]):int(do[i] + sizes[i])], src[int(so[i]):int(so[i] + sizes[i])])
        assert not dst[int(sizes.sum()):].any()


def test_host_resize_matches_oracle(oracle):
    """libffcv.cpp:33-42 resize() from libffcv_hip.so (the kernels' own
    INTER_AREA functions compiled for the host) against the oracle's OpenCV
    4.5.4 restatement, bit-exact over random ROIs covering every branch:
    copy, integer-scale area-fast, float area, and the Q11 linear path."""
    from ffcv_amd import libffcv as L
    rng = np.random.default_rng(5)
    img = rng.integers(0, 256, (300, 420, 3), dtype=np.uint8)
    cases = [((0, 64, 0, 64), (64, 64)), ((10, 74, 20, 84), (32, 32)), ((0, 300, 0, 420), (100, 140)),
             ((5, 290, 7, 400), (224, 224)), ((0, 30, 0, 40), (224, 224)), ((3, 123, 9, 9 + 150), (224, 224)),
             ((0, 1, 0, 1), (5, 7)), ((0, 300, 0, 420), (1, 1))]
    for _ in range(60):
        r0 = int(rng.integers(0, 299)); r1 = int(rng.integers(r0 + 1, 301))
        c0 = int(rng.integers(0, 419)); c1 = int(rng.integers(c0 + 1, 421))
        cases.append(((r0, r1, c0, c1), (int(rng.integers(1, 300)), int(rng.integers(1, 300)))))
    for (r0, r1, c0, c1), (th, tw) in cases:
        got = np.zeros((th, tw, 3), np.uint8)
        L.resize_crop(img, r0, r1, c0, c1, got)
        want = oracle.resize_crop(img, r0, r1, c0, c1, th, tw)
        assert np.array_equal(got, want), ((r0, r1, c0, c1), (th, tw))
    # the reference's constant-image invariant (test_rrc.py:63)
    const = np.full((50, 60, 3), 77, np.uint8)
    out = np.zeros((33, 41, 3), np.uint8)
    L.resize_crop(const, 3, 40, 2, 57, out)
    assert (out == 77).all()


def test_host_read_and_imdecode_arguments(tmp_path, hip_lib):
    """read (pread) round trip; imdecode argument validation (no device call)."""
    from ffcv_amd import libffcv as L
    p = tmp_path / 'f.bin'
    data = np.arange(1000, dtype=np.uint16).view(np.uint8)
    p.write_bytes(data.tobytes())
    with open(p, 'rb') as f:
        dst = np.zeros(300, np.uint8)
        assert L.read(f.fileno(), dst, 100) == 300
        assert np.array_equal(dst, data[100:400])
    out = np.zeros((8, 8, 3), np.uint8)
    assert L.imdecode(data, out, 8, 8, enable_crop=True) == -1
    assert b'SOI' in hip_lib.ffcv_last_error()
    assert L.imdecode(data, out, 8, 8, 0, 8) == -1


def test_my_fread(tmp_path, hip_lib):
    """libffcv.cpp:48-51 my_fread(FILE *, offset, destination, size): fseek + fread."""
    p = tmp_path / 'f.bin'
    data = np.random.default_rng(3).integers(0, 256, 5000, dtype=np.uint8)
    p.write_bytes(data.tobytes())
    libc = ctypes.CDLL(None)
    libc.fopen.restype = ctypes.c_void_p
    libc.fopen.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
    libc.fclose.argtypes = [ctypes.c_void_p]
    fp = libc.fopen(str(p).encode(), b'rb')
    assert fp
    try:
        for off, n in [(0, 100), (4321, 679), (17, 1), (1000, 3000)]:
            dst = np.zeros(n, np.uint8)
            hip_lib.my_fread(fp, off, dst.ctypes.data, n)
            assert np.array_equal(dst, data[off:off + n])
        dst = np.full(64, 7, np.uint8)  # short read at the end: the rest stays as it was
        hip_lib.my_fread(fp, 4990, dst.ctypes.data, 64)
        assert np.array_equal(dst[:10], data[4990:]) and (dst[10:] == 7).all()
    finally:
        libc.fclose(fp)


def test_scratch_bound_matches_c(hip_lib):
    """libffcv.scratch_bound (numpy, used to size launch arenas) equals
    ffcv_jpeg_scratch_bound; arena_for sums the largest per-image bounds."""
    from ffcv_amd import libffcv as L
    rng = np.random.default_rng(2)
    hs = rng.integers(1, 5000, 200)
    ws = rng.integers(1, 5000, 200)
    ns = rng.integers(1, 3_000_000, 200)
    got = L.scratch_bound(hs, ws, ns)
    for h, w, n, g in zip(hs, ws, ns, got):
        assert int(g) == L.lib().ffcv_jpeg_scratch_bound(int(h), int(w), int(n))
    assert L.arena_for(hs, ws, ns, 10) == int(np.sort(got)[-10:].sum()) + 4096
    # a launch of 10 from 5 images: the 5 extra slots may repeat the largest
    assert L.arena_for(hs[:5], ws[:5], ns[:5], 10) == int(got[:5].sum() + 5 * got[:5].max()) + 4096
