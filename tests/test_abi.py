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
