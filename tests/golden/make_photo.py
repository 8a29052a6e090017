"""Real-photo JPEG fixtures from the reference's own test image (this
container only: /root/reference does not exist on the GPU box).

The reference's JPEG decode benchmark (ffcv/benchmarks/suites/jpeg_decode.py:
14-41) loads test_data/pig.png (1023 x 642), resizes it with INTER_AREA to
widths 500 / 256 / 1024 (height int(642 * width / 1023)) and encodes it with
cv2.imencode at quality 50 and 90, then decodes it with imdecode.  This script
does the same with the repository's INTER_AREA restatement (oracle/) and
Pillow's libjpeg-turbo encoder (4:2:0, standard tables: the stream
cv2.imencode writes), adds q95 4:4:4 and q75 4:2:2 encodings of two widths, and
commits ONLY the JPEG bytes plus the SHA-256 of libjpeg-turbo's own ifast +
fancy decode of each (TurboJPEG's TJFLAG_FASTDCT, libffcv.cpp:104-106), so a
box whose libjpeg-turbo decodes differently fails loudly instead of silently
moving the goalposts.  The PNG itself is data, read here; nothing else from
the reference is used.

Run:  python tests/golden/make_photo.py   ->  tests/golden/photo.npz
"""
import hashlib
import io
import os
import sys

import numpy as np
from PIL import Image

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from oracle import oracle as O  # noqa: E402

SRC = '/root/reference/test_data/pig.png'
# (width, quality, subsampling): the reference suite's 3 widths x 2 qualities,
# then two extra layouts
CASES = [(w, q, '4:2:0') for w in (500, 256, 1024) for q in (50, 90)] + \
        [(500, 95, '4:4:4'), (256, 95, '4:4:4'), (256, 75, '4:2:2'), (500, 75, '4:2:2')]


def main():
    img = np.asarray(Image.open(SRC).convert('RGB'))
    H, W = img.shape[:2]
    blobs, shapes, digests, meta = [], [], [], []
    for w, q, sub in CASES:
        h = int(H * (w / W))  # jpeg_decode.py:32-34
        small = O.resize_crop(img, 0, H, 0, W, h, w)  # cv2.resize(..., INTER_AREA)
        b = io.BytesIO()
        Image.fromarray(small).save(b, 'JPEG', quality=q, subsampling=sub)
        data = np.frombuffer(b.getvalue(), np.uint8)
        dec = O.ljt_decode(data)
        assert dec.shape == (h, w, 3)
        blobs.append(data)
        shapes.append((h, w))
        digests.append(hashlib.sha256(dec.tobytes()).hexdigest())
        meta.append(f'{w}x{h} q{q} {sub}')
        print(meta[-1], len(data), 'bytes')
    offs = np.cumsum([0] + [len(b) for b in blobs])
    np.savez_compressed(os.path.join(HERE, 'photo.npz'), data=np.concatenate(blobs), offs=offs,
                        shapes=np.array(shapes, np.int32), sha256=np.array(digests), cases=np.array(meta))


if __name__ == '__main__':
    main()
