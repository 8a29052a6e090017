"""The integer identities the linear walks (K2's fast path in ffcv_jpeg.hip,
the raw kernel's walk in ffcv_rrc.hip) rest on, checked over their whole
input ranges on the host.  Each replaces a step of OpenCV's
HResizeLinear / VResizeLinearVec_32s8u (resize.cpp, the Q11 branch that
INTER_AREA takes for upscaling axes) by cheaper gfx950
forms; DESIGN.md s3 "K2 in detail" states the bounds used here.  The GPU
parity tests compare the kernels themselves with the oracle."""
import numpy as np

# weights: linear_coef rounds each tap separately, so c0 + c1 <= 2049, each in [0, 2048]
W_MAX = 2048


def _weight_pairs():
    a = np.arange(0, W_MAX + 1, dtype=np.int64)
    # both extremes of the sum and a spread of interior pairs
    return [(int(x), int(min(W_MAX, 2049 - x))) for x in a[::37]] + [(2048, 0), (0, 2048), (1024, 1025), (2048, 1)]


def test_horizontal_pass_dot2_mask():
    """hrow: h = p * a + q * b (u8 samples, Q11 weights); the kernel takes
    v_dot2_u32_u16 with the weights pre-scaled by 16 and keeps dot & 0x7fff00,
    which must equal (h >> 4) << 8 (sat_s16 never acts: h >> 4 <= 32655)."""
    p = np.arange(256, dtype=np.int64)[:, None]
    q = np.arange(256, dtype=np.int64)[None, :]
    for a, b in _weight_pairs():
        h = p * a + q * b
        dot = (p * (a << 4) + q * (b << 4)) & 0xFFFFFFFF  # the u32 accumulator
        assert int(dot.max()) < 1 << 32
        assert np.array_equal(dot & 0x7FFF00, (h >> 4) << 8), (a, b)
        assert int((h >> 4).max()) <= 32655


def test_vertical_pass_mulhi24():
    """VResizeLinearVec: (m0 + m1 + 2) >> 2 with m = (H * c) >> 16, H = h >> 4;
    the kernel forms m as v_mul_hi_u32_u24(H << 8, c << 8) (both operands
    below 2^24), and the result never needs the u8 saturation."""
    H = np.arange(0, 32656, dtype=np.int64)
    for c0, c1 in _weight_pairs():
        for Hb in (H, H[::-1]):
            m0 = ((H << 8) * (c0 << 8)) >> 32
            m1 = ((Hb << 8) * (c1 << 8)) >> 32
            assert int((H << 8).max()) < 1 << 24 and (c0 << 8) < 1 << 24
            assert np.array_equal(m0, (H * c0) >> 16)
            assert np.array_equal(m1, (Hb * c1) >> 16)
            assert int(((m0 + m1 + 2) >> 2).max()) <= 255


def test_lut_address_from_vertical_sum():
    """lut_q<FP16> (ffcv_jpeg.hip): the channel-0 LUT entry of value
    v = (x + 2) >> 2 sits at byte base + 2 v of the channel-major LDS table;
    the kernel computes it as ((x + 2 + 2 base) >> 1) & ~1 (base even), and a
    cutout fill f as base + 2 f."""
    x = np.arange(0, 1021, dtype=np.int64)  # m0 + m1 <= 1020
    for base in (0, 2, 512, 1536, 26622, 65534):
        lq = 2 + 2 * base
        addr = ((x + lq) >> 1) & ~1
        assert np.array_equal(addr, base + 2 * ((x + 2) >> 2)), base
        assert int(((x + 2) >> 2).max()) <= 255
        # channel c's table: + 512 c bytes, inside the 1,536-byte LUT
        assert int(addr.max()) + 2 * 512 + 2 <= base + 1536
