"""Parity on a real photograph: the reference's own test image.

tests/golden/photo.npz holds JPEG encodings of /root/reference/test_data/
pig.png made the way the reference's JPEG decode benchmark makes them
(ffcv/benchmarks/suites/jpeg_decode.py:14-41: INTER_AREA to widths 500 / 256 /
1024, quality 50 and 90), plus q95 4:4:4 and q75 4:2:2 encodings, and the
SHA-256 of libjpeg-turbo's own ifast + fancy decode of each
(tests/golden/make_photo.py; only the bytes are committed).  Natural-photo
entropy streams -- long codes, dense AC blocks, 300 KB scans at 1024 px --
are what the synthetic generator does not produce.

CPU tests pin libjpeg-turbo (the box's Pillow-bundled copy must decode to the
committed digests), the oracle's decode and the CPU imdecode to it; the GPU
tests run the full-image decode and the fused RRC + Cutout + flip + fp16 LUT
on these images through the C ABI, bit-exact against the oracle.
"""
import hashlib
import os

import numpy as np
import pytest

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden', 'photo.npz')


def _photos():
    z = np.load(GOLD)
    data, offs = z['data'], z['offs']
    blobs = [data[offs[i]:offs[i + 1]].copy() for i in range(len(offs) - 1)]
    return blobs, [tuple(int(v) for v in s) for s in z['shapes']], list(z['sha256']), list(z['cases'])


def test_photo_fixture_pins_libjpeg_turbo(oracle):
    blobs, shapes, digests, cases = _photos()
    assert len(blobs) == 10 and max(s[1] for s in shapes) == 1024
    for b, (h, w), d, c in zip(blobs, shapes, digests, cases):
        got = oracle.ljt_decode(b)
        assert got.shape == (h, w, 3), c
        assert hashlib.sha256(got.tobytes()).hexdigest() == d, f'{c}: libjpeg-turbo decodes differently'


def test_photo_oracle_and_cpu_imdecode_match_libjpeg_turbo(hip_lib, oracle):
    from ffcv_amd import libffcv as L
    blobs, shapes, _, cases = _photos()
    for b, (h, w), c in zip(blobs, shapes, cases):
        want = oracle.ljt_decode(b)
        assert np.array_equal(oracle.jpeg_decode(b), want), f'{c}: oracle restatement'
        out = np.zeros((h, w, 3), np.uint8)
        assert L.imdecode(b, out, h, w, h, w, 0, 0, 1, 1, False, False) == 0
        assert np.array_equal(out, want), f'{c}: CPU imdecode'


def _torch():
    import torch
    if not torch.cuda.is_available():
        pytest.skip('no HIP device')
    return torch


def _dev_set(blobs, shapes, reps=1):
    torch = _torch()
    from ffcv_amd.libffcv import SAMPLE_DTYPE
    from ffcv_amd.synthetic import pack
    buf, offs, sizes = pack(blobs)
    n = len(blobs) * reps
    smp = np.zeros(n, SAMPLE_DTYPE)
    idx = np.arange(n) % len(blobs)
    smp['offset'] = offs[idx]
    smp['size'] = sizes[idx]
    smp['height'] = [shapes[i][0] for i in idx]
    smp['width'] = [shapes[i][1] for i in idx]
    d_buf = torch.from_numpy(buf).to('cuda:0')
    d_smp = torch.from_numpy(smp.view(np.uint8)).to('cuda:0')
    return d_buf, d_smp, idx


@pytest.mark.gpu
def test_photo_full_decode_matches_libjpeg_turbo(hip_lib, oracle):
    torch = _torch()
    from ffcv_amd import libffcv as L
    blobs, shapes, _, cases = _photos()
    d_buf, d_smp, _ = _dev_set(blobs, shapes)
    B = len(blobs)
    maxh, maxw = max(s[0] for s in shapes), max(s[1] for s in shapes)
    dec = L.JpegDecoder(B, maxh, maxw, max(len(b) for b in blobs))
    stride = maxh * maxw * 3
    out = torch.zeros(B * stride, dtype=torch.uint8, device='cuda:0')
    status = torch.full((B,), -1, dtype=torch.int32, device='cuda:0')
    dec.decode(d_buf, d_smp, B, out, stride, status)
    torch.cuda.synchronize()
    st, o = status.cpu().numpy(), out.cpu().numpy()
    for k, ((h, w), c) in enumerate(zip(shapes, cases)):
        assert st[k] == 0, (c, st[k])
        got = o[k * stride:k * stride + h * w * 3].reshape(h, w, 3)
        assert np.array_equal(got, oracle.ljt_decode(blobs[k])), c


@pytest.mark.gpu
@pytest.mark.parametrize('out_hw', [(224, 224), (448, 448)])
def test_photo_rrc_cutout_flip_fp16_matches_oracle(hip_lib, oracle, out_hw):
    """Twelve random crops (and two centre crops) of each photo, RRC to out_hw
    + Cutout + flip + NormalizeImage fp16 LUT, the C3 epilogue; 448 x 448 has
    no per-image tap table (out_w + out_h > K2_TAPS) and more area crops."""
    torch = _torch()
    from ffcv_amd import libffcv as L
    from tests.test_kernels_gpu import _draw, _oracle_post
    blobs, shapes, _, cases = _photos()
    reps = 14
    d_buf, d_smp, idx = _dev_set(blobs, shapes, reps)
    B = len(idx)
    hs = np.array([shapes[i][0] for i in idx], np.uint32)
    ws = np.array([shapes[i][1] for i in idx], np.uint32)
    ids = np.arange(B, dtype=np.uint64) + 5000
    cs = 32 if out_hw[0] == 224 else 64
    crops, cut, flips = _draw(hip_lib, ids, hs, ws, 11, 0, cutout=cs, flip_p=0.5, out=out_hw)
    ccrops, _, _ = _draw(hip_lib, ids, hs, ws, 11, 0, crop_kind=1, out=out_hw)
    center = np.arange(B) // len(blobs) >= reps - 2  # the last two rounds: centre crops
    crops[center] = ccrops[center]
    lut = oracle.normalize_lut(np.array([0.485, 0.456, 0.406]) * 255, np.array([0.229, 0.224, 0.225]) * 255)
    dec = L.JpegDecoder(B, int(hs.max()), int(ws.max()), max(len(b) for b in blobs))
    p = L.RRCParams()
    p.out_h, p.out_w = out_hw
    p.cutout_size = cs
    for i, f in enumerate((124, 116, 103)):
        p.cutout_fill[i] = f
    d_lut = torch.from_numpy(lut.view(np.int16)).to('cuda:0')
    p.lut = d_lut.data_ptr()
    out = torch.zeros((B, *out_hw, 3), dtype=torch.float16, device='cuda:0')
    status = torch.full((B,), -1, dtype=torch.int32, device='cuda:0')
    dec.rrc(d_buf, d_smp, B, torch.from_numpy(crops).to('cuda:0'), torch.from_numpy(cut).to('cuda:0'),
            torch.from_numpy(flips).to('cuda:0'), p, out, status)
    torch.cuda.synchronize()
    assert (status.cpu().numpy() == 0).all()
    oracle.use_libjpeg_turbo(True)
    try:
        u8 = oracle.rrc_batch([(blobs[i], shapes[i][0], shapes[i][1], 0) for i in idx], crops, *out_hw,
                              nthreads=8)
    finally:
        oracle.use_libjpeg_turbo(False)
    want = _oracle_post(u8, flips, cut, cs, (124, 116, 103), lut)
    got = out.cpu().numpy()
    bad = np.argwhere((got.view(np.uint16) != want.view(np.uint16)).reshape(B, -1).any(1)).ravel()
    assert bad.size == 0, [(int(k), cases[idx[k]], crops[k].tolist()) for k in bad[:6]]
