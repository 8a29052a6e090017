"""imdecode on the CPU (libffcv.cpp:53-112 signature; ffcv_cpu_jpeg.hip)
against libjpeg-turbo 3.1.4 itself (Pillow-bundled, through the oracle's
jpeg62 harness with the reference's TurboJPEG settings: ifast IDCT, fancy
upsampling, RGB out).  No GPU: the reference's CPU Loader decodes here."""
import io
import threading

import numpy as np
from PIL import Image

from ffcv_amd.synthetic import natural_image, encode_jpeg, imagenet_like_shape


def _set(rng, n, max_side=300):
    imgs, blobs = [], []
    subs = ['4:2:0', '4:2:2', '4:4:4']
    for k in range(n):
        if k % 5 == 4:
            h, w = int(rng.integers(1, 300)), int(rng.integers(1, 300))
        else:
            h, w = imagenet_like_shape(rng, max_side)
        img = natural_image(rng, h, w)
        if k % 11 == 10:
            img = img[:, :, 0].copy()
        q = [90, 95, 75, 50, 100, 1, 30][k % 7]
        blobs.append(encode_jpeg(img, q, subs[k % 3], optimize=k % 4 == 3))
        imgs.append(img)
    return imgs, blobs


def _pil(img, **kw):
    b = io.BytesIO()
    Image.fromarray(img).save(b, 'JPEG', **kw)
    return np.frombuffer(b.getvalue(), np.uint8).copy()


def test_cpu_imdecode_matches_libjpeg_turbo(hip_lib, oracle):
    from ffcv_amd import libffcv as L
    rng = np.random.default_rng(41)
    imgs, blobs = _set(rng, 56)
    # restart intervals (DRI + RSTn every 1 / 3 MCUs or every MCU row), and
    # 4:1:1 / 4:4:0 style layouts Pillow writes with explicit factors
    extra = []
    for k in range(6):
        h, w = imagenet_like_shape(rng, 200)
        img = natural_image(rng, h, w)
        extra.append((img, _pil(img, quality=85, restart_marker_blocks=[1, 3, 7][k % 3])))
        extra.append((img, _pil(img, quality=92, restart_marker_rows=1, subsampling=k % 3)))
    for img, b in extra:
        imgs.append(img)
        blobs.append(b)
    errors = []

    def work(ks):
        for k in ks:
            h, w = imgs[k].shape[:2]
            out = np.zeros((h, w, 3), np.uint8)
            rc = L.imdecode(blobs[k], out, h, w, h, w, 0, 0, 1, 1, False, False)
            want = oracle.ljt_decode(blobs[k])
            if rc != 0 or not np.array_equal(out, want):
                errors.append((k, rc, int((out != want).sum())))
    ths = [threading.Thread(target=work, args=(range(t, len(imgs), 4),)) for t in range(4)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    assert not errors, errors


def test_cpu_imdecode_rejects(hip_lib):
    from ffcv_amd import libffcv as L
    rng = np.random.default_rng(3)
    img = natural_image(rng, 40, 56)
    blob = encode_jpeg(img, 90)
    out = np.zeros((40, 56, 3), np.uint8)
    assert L.imdecode(blob, out, 40, 56) == 0
    bad = blob.copy()
    bad[:2] = 0  # no SOI
    assert L.imdecode(bad, out, 40, 56) == -1
    assert b'SOI' in L.lib().ffcv_last_error()
    # tjDecompress2 decodes at the largest scaling factor that fits the
    # request: 41 x 56 fits only 1/1 (rows packed at the image's width) ...
    big = np.full((41, 56, 3), 7, np.uint8)
    assert L.imdecode(blob, big, 40, 56, 41, 56) == 0
    assert np.array_equal(big[:40], out) and (big[40] == 7).all()
    # ... 45 x 63 fits 9/8, a scaled decode this restatement does not do
    assert L.imdecode(blob, np.zeros((45, 63, 3), np.uint8), 40, 56, 45, 63) == -1
    assert b'scale 9/8' in L.lib().ffcv_last_error()
    # 3/8 (jidctint.c's 3x3 IDCT) is not restated; 1/2, 1/4, 1/8 are (below)
    assert L.imdecode(blob, np.zeros((15, 21, 3), np.uint8), 40, 56, 40, 56, 0, 0, 3, 8) == -1
    assert b'scale 3/8' in L.lib().ffcv_last_error()
    # the lossless crop's origin must be on an iMCU boundary (16 x 16 at 4:2:0)
    assert L.imdecode(blob, out, 40, 56, 24, 24, 8, 0, enable_crop=True) == -1
    assert b'iMCU' in L.lib().ffcv_last_error()
    assert L.imdecode(blob, out, 40, 56, 8, 8, 64, 0, enable_crop=True) == -1  # origin outside
    prog = _pil(img, quality=90, progressive=True)
    assert L.imdecode(prog, out, 40, 56) == -1
    assert b'progressive' in L.lib().ffcv_last_error()
    # truncated stream: decodes (zeros past the end, like libjpeg's warning path), never crashes
    assert L.imdecode(blob[: len(blob) // 2], out, 40, 56) in (0, -1)
    # an over-subscribed DHT with an unchanged symbol count
    # (three 1-bit codes) is rejected before any lookup entry is built
    b = bytes(blob)
    dht = b.index(b'\xff\xc4') + 4  # Tc/Th byte of the first table
    bits = dht + 1
    assert b[bits] == 0 and b[bits + 2] >= 3, 'expected the standard luma DC table'
    over = bytearray(b)
    over[bits] = 3
    over[bits + 2] -= 3
    assert L.imdecode(np.frombuffer(bytes(over), np.uint8), out, 40, 56) == -1
    assert b'Huffman' in L.lib().ffcv_last_error()
    # non-integral sampling ratios (luma h = 3, chroma h = 2)
    sof = b.index(b'\xff\xc0') + 2 + 2 + 6  # first component's id
    assert b[sof + 1] == 0x22 and b[sof + 4] == 0x11
    frac = bytearray(b)
    frac[sof + 1] = 0x32
    frac[sof + 4] = 0x21
    assert L.imdecode(np.frombuffer(bytes(frac), np.uint8), out, 40, 56) == -1
    assert b'sampling' in L.lib().ffcv_last_error()


def test_cpu_imdecode_transform(hip_lib):
    """libffcv.cpp:78-103: tjTransform(TJXOPT_CROP [+ TJXOP_HFLIP]) then
    tjDecompress2, restated on the coefficients (transupp.c do_crop /
    do_flip_h).  Parity unpinned: libturbojpeg (the transform) is not in this
    image, only Pillow's libjpeg; these are the properties the lossless
    transforms guarantee."""
    from ffcv_amd import libffcv as L
    rng = np.random.default_rng(8)

    def dec(blob, h, w, ch, cw, ox=0, oy=0, crop=False, flip=False):
        out = np.full((ch, cw, 3), 3, np.uint8)
        rc = L.imdecode(blob, out, h, w, ch, cw, ox, oy, 1, 1, crop, flip)
        assert rc == 0, L.lib().ffcv_last_error()
        return out

    # the full image as the crop: the same coefficients, the same pixels
    img = natural_image(rng, 72, 100)
    b420 = _pil(img, quality=90, subsampling=2)
    full = dec(b420, 72, 100, 72, 100)
    assert np.array_equal(dec(b420, 72, 100, 72, 100, crop=True), full)
    # 4:4:4 (no upsampling): a block-aligned crop is exactly the crop of the decode
    b444 = _pil(img, quality=90, subsampling=0)
    f444 = dec(b444, 72, 100, 72, 100)
    assert np.array_equal(dec(b444, 72, 100, 24, 40, 16, 8, crop=True), f444[8:32, 16:56])
    # a set crop size past the image edge is refused, as transupp.c's
    # jtransform_request_workspace does (JERR_BAD_CROP_SPEC: tjTransform and
    # so the reference's imdecode return -1); size 0 still means "to the edge"
    out = np.zeros((20, 56, 3), np.uint8)
    assert L.imdecode(b444, out, 72, 100, 20, 56, 48, 56, 1, 1, True, False) == -1
    assert b'bad crop spec' in L.lib().ffcv_last_error()
    assert L.imdecode(b444, out, 72, 100, 16, 56, 48, 56, 1, 1, True, False) == -1  # x + w > W
    assert L.imdecode(b444, out, 72, 100, 20, 52, 48, 56, 1, 1, True, False) == -1  # y + h > H
    edge = dec(b444, 72, 100, 16, 52, 48, 56, crop=True)  # exactly to the corner
    assert np.array_equal(edge, f444[56:, 48:])
    # 4:2:0: away from the crop's borders the fancy upsampling sees the same chroma
    c = dec(b420, 72, 100, 40, 48, 32, 16, crop=True)
    assert np.array_equal(c[2:-2, 2:-2], full[18:54, 34:78])
    # horizontal mirror, grey, width 8k + 3: the whole blocks are mirrored (odd
    # DCT columns negated: the same pixels up to the IDCT's rounding), the
    # partial block at the right edge stays where it is, unchanged
    g = natural_image(rng, 40, 67)[:, :, 0].copy()
    bg = _pil(g, quality=90)
    fg = dec(bg, 40, 67, 40, 67)
    fl = dec(bg, 40, 67, 40, 67, flip=True)
    assert np.array_equal(fl[:, 64:], fg[:, 64:])
    d = np.abs(fl[:, :64].astype(int) - fg[:, 63::-1].astype(int))
    assert d.max() <= 2 and d.mean() < 0.5, (d.max(), d.mean())
    # the crop is taken in the mirrored frame: columns [8, 24) of the mirror
    assert np.array_equal(dec(bg, 40, 67, 16, 16, 8, 8, crop=True, flip=True), fl[8:24, 8:24])
    # hflip alone still crops with the given offsets and size (libffcv.cpp:89-93)
    assert np.array_equal(dec(bg, 40, 67, 16, 24, 16, 8, flip=True), fl[8:24, 16:40])


def test_cpu_imdecode_scaled_matches_libjpeg_turbo(hip_lib, oracle):
    """libffcv.cpp:101-103 tjDecompress2 at scaling factors 1/2, 1/4, 1/8
    (scale_num / scale_denom): jidctred.c's reduced IDCTs, libjpeg-turbo's
    per-component DCT sizes (4:2:0 chroma at twice the luma's size, no
    upsampling), non-fancy upsampling at 1/8 -- bit-exact against
    libjpeg-turbo 3.1.4 itself (the harness sets scale_num / scale_denom)."""
    from ffcv_amd import libffcv as L
    rng = np.random.default_rng(5)
    cases = []
    for h, w in [(61, 83), (64, 64), (17, 33), (120, 91), (9, 7)]:
        img = natural_image(rng, h, w)
        cases += [(img, encode_jpeg(img, 90, '4:2:0')), (img, encode_jpeg(img, 85, '4:2:2')),
                  (img, encode_jpeg(img, 95, '4:4:4')), (img[:, :, 0].copy(), _pil(img[:, :, 0].copy(), quality=90)),
                  (img, _pil(img, quality=90, subsampling=2))]
    bad = []
    for img, b in cases:
        h, w = img.shape[:2]
        for den in (2, 4, 8):
            want = oracle.ljt_decode(b, scale=(1, den))
            out = np.zeros(want.shape, np.uint8)
            rc = L.imdecode(b, out, h, w, h, w, 0, 0, 1, den, False, False)
            if rc != 0 or not np.array_equal(out, want):
                bad.append((h, w, den, rc))
    assert not bad, bad
    # crop then scale: at 4:4:4 (no upsampling) each block scales on its own,
    # so a block-aligned crop at 1/2 is the crop of the 1/2 decode
    img = natural_image(rng, 72, 100)
    b = _pil(img, quality=90, subsampling=0)
    half = oracle.ljt_decode(b, scale=(1, 2))
    out = np.zeros((12, 20, 3), np.uint8)
    assert L.imdecode(b, out, 72, 100, 24, 40, 16, 8, 1, 2, True, False) == 0
    assert np.array_equal(out, half[4:16, 8:28])


def test_cpu_decode_batch(hip_lib, oracle):
    """ffcv_cpu_decode_batch: the per-sample CPU loop as one threaded call --
    JPEG and raw samples, whole images and crops resized by INTER_AREA, a
    skipped sample, and a corrupt one reported in its status only."""
    from ffcv_amd import libffcv as L
    rng = np.random.default_rng(7)
    imgs = [natural_image(rng, int(rng.integers(40, 120)), int(rng.integers(40, 120))) for _ in range(12)]
    blobs = [encode_jpeg(im, 90, ['4:2:0', '4:4:4'][k % 2]) for k, im in enumerate(imgs)]
    modes = np.array([0, 1] * 6, np.uint32)
    srcs = [blobs[k] if modes[k] == 0 else imgs[k].reshape(-1) for k in range(12)]
    hs = np.array([im.shape[0] for im in imgs], np.uint32)
    ws = np.array([im.shape[1] for im in imgs], np.uint32)
    decoded = [oracle.ljt_decode(blobs[k]) if modes[k] == 0 else imgs[k] for k in range(12)]
    # crops resized to 32 x 48
    crops = np.array([[k % 5, k % 7, int(hs[k]) // 2, int(ws[k]) // 2] for k in range(12)], np.int32)
    out = np.zeros((12, 32, 48, 3), np.uint8)
    st = L.cpu_decode_batch(srcs, hs, ws, modes, out, crops, nthreads=4)
    assert (st == 0).all()
    for k in range(12):
        i, j, h, w = crops[k]
        want = oracle.resize_crop(decoded[k], i, i + h, j, j + w, 32, 48)
        assert np.array_equal(out[k], want), k
    # whole images (the Simple decoder): a fixed-size destination per sample
    H, W = int(hs.max()), int(ws.max())
    full = np.zeros((12, H, W, 3), np.uint8)
    modes2 = modes.copy()
    modes2[3] = 2  # skipped: left untouched
    bad = [s.copy() for s in srcs]
    bad[4] = bad[4].copy()
    bad[4][:2] = 0  # corrupt JPEG
    st = L.cpu_decode_batch(bad, hs, ws, modes2, full, nthreads=3)
    assert st[4] == -1 and (np.delete(st, 4) == 0).all()
    for k in range(12):
        if k in (3, 4):
            continue
        h, w = int(hs[k]), int(ws[k])
        got = full[k].reshape(-1)[:h * w * 3].reshape(h, w, 3)
        assert np.array_equal(got, decoded[k]), k
    assert not full[3].any()
    # the first failing sample's message reaches the calling thread
    assert b'sample 4' in L.lib().ffcv_last_error()
    # a raw sample shorter than h x w x 3 fails, with no read past it
    short = [s.copy() for s in srcs]
    short[5] = short[5][:-7]
    st = L.cpu_decode_batch(short, hs, ws, modes, full, nthreads=3)
    assert st[5] == -1 and (np.delete(st, 5) == 0).all()
    assert b'raw sample 5' in L.lib().ffcv_last_error()


def test_jpeg_scan_stats(hip_lib):
    """ffcv_jpeg_scan_stats (bench.py's K1 symbols per image): a constant
    image codes every block as DC + EOB, so symbols == 2 x blocks exactly;
    the block count follows the MCU grid; a natural image has more symbols
    than a constant one of the same size; junk reports zeros and -1."""
    from ffcv_amd import libffcv as L
    flat = np.full((48, 40, 3), 117, np.uint8)
    nat = natural_image(np.random.default_rng(3), 48, 40)
    blobs = [encode_jpeg(flat, 90, '4:2:0'), encode_jpeg(flat, 90, '4:4:4'), encode_jpeg(nat, 90, '4:2:0')]
    st = L.jpeg_scan_stats([np.frombuffer(b, np.uint8) for b in blobs])
    # 4:2:0: 48 x 40 -> 3 x 3 MCUs (16 x 16) of 4 Y + Cb + Cr; 4:4:4: 6 x 5 MCUs of 3 blocks
    assert st[0, 1] == 3 * 3 * 6 and st[1, 1] == 6 * 5 * 3 and st[2, 1] == st[0, 1]
    assert st[0, 0] == 2 * st[0, 1] and st[1, 0] == 2 * st[1, 1]
    assert st[2, 0] > st[0, 0] and 0 < st[0, 2] < len(blobs[0])
    bad = L.jpeg_scan_stats([np.zeros(64, np.uint8)])
    assert bad.tolist() == [[0, 0, 0]]
