"""The oracle is pinned before it is trusted (CPU only).

* crops / center crops / cutout origins / normalize LUT: golden vectors
  produced by the REFERENCE's own Python (tests/golden/make_golden.py).
* JPEG: bit-exact against libjpeg-turbo 3.1.4 (Pillow-bundled) driven with
  the reference's TurboJPEG settings (ifast + fancy upsampling, RGB) through
  oracle/ljt_harness.c, and (islow) against Pillow's own decode.
* INTER_AREA: OpenCV is absent (parity unpinned beyond invariants): the
  reference's constant-image invariant (test_rrc.py:63), copy at scale 1,
  exact block means at integer scales.
"""
import io
import os

import numpy as np
import pytest

from ffcv_amd.synthetic import natural_image, encode_jpeg

GOLD = os.path.join(os.path.dirname(__file__), 'golden')


def test_random_crops_match_reference(oracle):
    g = np.load(os.path.join(GOLD, 'crops.npz'))['random']
    bad = 0
    for row in g:
        seed, H, W, s0, s1, r0, r1, i, j, h, w = row
        got = oracle.MT(int(seed)).random_crop(int(H), int(W), (s0, s1), (r0, r1))
        bad += got != (int(i), int(j), int(h), int(w))
    assert bad == 0 and len(g) == 24000


def test_center_crops_match_reference(oracle):
    g = np.load(os.path.join(GOLD, 'crops.npz'))['center']
    for H, W, ratio, i, j, h, w in g:
        assert oracle.center_crop(int(H), int(W), ratio) == (int(i), int(j), int(h), int(w))


def test_cutout_draws_match_reference(oracle):
    rows = np.load(os.path.join(GOLD, 'cutout.npz'))['rows']
    for seed, H, W, c, y, x in rows:
        mt = oracle.MT(int(seed))
        assert (mt.randint(int(H - c + 1)), mt.randint(int(W - c + 1))) == (y, x)


def test_normalize_lut_matches_reference(oracle):
    from ffcv_amd.transforms.lut import make_lut
    g = np.load(os.path.join(GOLD, 'normalize_lut.npz'))
    for n in ['imagenet', 'test']:
        assert np.array_equal(oracle.normalize_lut(g['mean_' + n], g['std_' + n]).view(np.int16), g['lut_' + n])
        assert np.array_equal(make_lut(g['mean_' + n], g['std_' + n]).view(np.int16), g['lut_' + n])


def _jpegs(rng, n):
    out = []
    for k in range(n):
        h, w = int(rng.integers(1, 260)), int(rng.integers(1, 260))
        img = natural_image(rng, h, w)
        if k % 9 == 8:
            img = img[:, :, 0].copy()
        out.append(encode_jpeg(img, [50, 75, 90, 95, 100][k % 5], ['4:2:0', '4:2:2', '4:4:4'][k % 3]))
    return out


def test_jpeg_oracle_matches_libjpeg_turbo(oracle):
    if oracle.ljt() is None:
        pytest.skip('Pillow-bundled libjpeg-turbo not found')
    rng = np.random.default_rng(0)
    for data in _jpegs(rng, 45):
        assert np.array_equal(oracle.jpeg_decode(data, 'ifast'), oracle.ljt_decode(data, 'ifast', True))


def test_jpeg_oracle_islow_matches_pillow(oracle):
    from PIL import Image
    rng = np.random.default_rng(1)
    for data in _jpegs(rng, 30):
        ref = np.asarray(Image.open(io.BytesIO(data.tobytes())).convert('RGB'))
        assert np.array_equal(oracle.jpeg_decode(data, 'islow'), ref)


def test_jpeg_flat_image_exact(oracle):
    # reference test_image_pipeline.py:68-71: constant 500x300 q95 -> exact
    for v in [0, 7, 128, 254]:
        img = np.full((500, 300, 3), v, np.uint8)
        assert (oracle.jpeg_decode(encode_jpeg(img, 95)) == v).all()


def test_resize_invariants(oracle):
    rng = np.random.default_rng(2)
    for _ in range(40):
        H, W = int(rng.integers(1, 600)), int(rng.integers(1, 600))
        v = int(rng.integers(0, 256))
        img = np.full((H, W, 3), v, np.uint8)
        i, j = int(rng.integers(0, H)), int(rng.integers(0, W))
        h, w = int(rng.integers(1, H - i + 1)), int(rng.integers(1, W - j + 1))
        out = oracle.resize_crop(img, i, i + h, j, j + w, 160, 160)
        assert (out == v).all()       # test_rrc.py:63 constant-image invariant
    img = natural_image(rng, 300, 300)
    assert np.array_equal(oracle.resize_crop(img, 10, 234, 5, 229, 224, 224), img[10:234, 5:229])
    # integer 2x downscale (cn=3 -> float path: rint(sum * 0.25))
    out = oracle.resize_crop(img, 0, 224, 0, 224, 112, 112)
    s = img[:224, :224].astype(np.int64).reshape(112, 2, 112, 2, 3).sum((1, 3))
    assert np.array_equal(out, np.rint(s.astype(np.float32) * np.float32(0.25)).astype(np.uint8))


def test_contract_seed_python_equals_oracle(oracle):
    from ffcv_amd.transforms.rng import contract_seed
    rng = np.random.default_rng(3)
    for _ in range(500):
        s, e, i, o = (int(rng.integers(0, 2 ** 63)), int(rng.integers(0, 1000)),
                      int(rng.integers(0, 2 ** 40)), int(rng.integers(1, 4)))
        assert contract_seed(s, e, i, o) == oracle.sample_seed(s, e, i, o)
    # numpy legacy RandomState is the same generator as the oracle's MT
    for seed in [0, 1, 12345, 2 ** 32 - 1]:
        rs = np.random.RandomState(seed)
        mt = oracle.MT(seed)
        assert [rs.randint(1000) for _ in range(20)] == [mt.randint(1000) for _ in range(20)]
        rs = np.random.RandomState(seed)
        mt = oracle.MT(seed)
        assert [rs.uniform(0, 1) for _ in range(20)] == [mt.uniform(0, 1) for _ in range(20)]
