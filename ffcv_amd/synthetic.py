"""Synthetic "natural" test images and JPEG encodings shared by tests and bench.

Images: seeded smooth noise + gradients + rectangles (SURVEY.md 8(d) C2
generator).  JPEGs are encoded with Pillow (libjpeg-turbo): baseline,
standard Huffman tables, no restart markers -- the stream cv2.imencode
produces for the reference's writer (rgb_image.py:26-34).
"""
import io

import numpy as np


def natural_image(rng, h, w):
    y = np.linspace(0, 1, h, dtype=np.float32)[:, None, None]
    x = np.linspace(0, 1, w, dtype=np.float32)[None, :, None]
    f = rng.uniform(2, 9, size=(2, 3)).astype(np.float32)
    ph = rng.uniform(0, 6.28, size=3).astype(np.float32)
    img = 128 + 70 * np.sin(f[0] * x * 3 + f[1] * y * 2 + ph) * np.cos(f[1] * x - f[0] * y)
    # low-frequency noise: coarse grid upsampled
    gh, gw = max(2, h // 16), max(2, w // 16)
    g = rng.normal(0, 25, size=(gh, gw, 3)).astype(np.float32)
    yi = (np.arange(h) * gh // h)[:, None]
    xi = (np.arange(w) * gw // w)[None, :]
    img = img + g[yi, xi]
    for _ in range(int(rng.integers(1, 5))):
        y0, x0 = int(rng.integers(0, h)), int(rng.integers(0, w))
        y1, x1 = min(h, y0 + int(rng.integers(1, h // 2 + 2))), min(w, x0 + int(rng.integers(1, w // 2 + 2)))
        img[y0:y1, x0:x1] = img[y0:y1, x0:x1] * 0.5 + rng.uniform(0, 255, 3) * 0.5
    img = img + rng.normal(0, 6, size=img.shape)
    return np.clip(img, 0, 255).astype(np.uint8)


def encode_jpeg(img, quality=90, subsampling='4:2:0', optimize=False):
    from PIL import Image
    b = io.BytesIO()
    mode = 'L' if img.ndim == 2 else 'RGB'
    Image.fromarray(img, mode).save(b, format='JPEG', quality=quality, subsampling=subsampling,
                                    optimize=optimize)
    return np.frombuffer(b.getvalue(), np.uint8).copy()


def imagenet_like_shape(rng, max_side=256):
    """Long side = max_side, aspect U(3/4, 4/3) (rgb_image.py:37-45 resizer)."""
    ar = rng.uniform(3 / 4, 4 / 3)
    if ar >= 1:
        return int(round(max_side / ar)), max_side
    return max_side, int(round(max_side * ar))


def pack(blobs):
    """Concatenate sample byte strings into one buffer (8-byte aligned) and
    return (buffer, offsets, sizes)."""
    offs, sizes = [], []
    total = 0
    for b in blobs:
        offs.append(total)
        sizes.append(len(b))
        total += (len(b) + 7) // 8 * 8
    buf = np.zeros(total + 64, np.uint8)
    for o, b in zip(offs, blobs):
        buf[o:o + len(b)] = np.frombuffer(bytes(b), np.uint8) if not isinstance(b, np.ndarray) else b
    return buf, np.array(offs, np.uint64), np.array(sizes, np.uint64)
