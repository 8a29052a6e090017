"""The CPU-device JPEG Loader (the reference's CPU path for C2/C3-shaped data):
JPEG .beton of N synthetic ImageNet-shape images (256 px, q90 4:2:0),
Loader(device='cpu') with RandomResizedCropRGBImageDecoder((224, 224)) +
ToTensor and IntDecoder, batch 512, RANDOM order, on `--workers` host
threads (imdecode on the CPU + INTER_AREA resize per sample, one native call
per batch: ffcv_cpu_decode_batch).  The first batch is checked against the
oracle (libjpeg-turbo decode + C restatement).

    python tools/cpu_jpeg_bench.py [--n 8192] [--epochs 3] [--workers 8]
"""
import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--n', type=int, default=8192)
    ap.add_argument('--epochs', type=int, default=3)
    ap.add_argument('--workers', type=int, default=8)
    args = ap.parse_args()
    from ffcv_amd.writer import DatasetWriter
    from ffcv_amd.fields import RGBImageField, IntField
    from ffcv_amd.fields.decoders import RandomResizedCropRGBImageDecoder, IntDecoder
    from ffcv_amd.transforms import ToTensor
    from ffcv_amd.loader import Loader, OrderOption
    from ffcv_amd.synthetic import natural_image, imagenet_like_shape
    from tests.helpers import samples_of, expected_rrc
    from oracle import oracle as O

    rng = np.random.default_rng(0)
    base = [natural_image(rng, *imagenet_like_shape(rng, 256)) for _ in range(256)]

    class DS:
        def __len__(self):
            return args.n

        def __getitem__(self, i):  # 256 base images, mirrored / shifted per index
            im = base[i % 256]
            im = im[:, ::-1] if (i // 256) % 2 else im
            return np.ascontiguousarray(np.roll(im, i // 512, axis=1)), i % 1000

    d = tempfile.mkdtemp()
    fn = os.path.join(d, 'cpu_jpeg.beton')
    t0 = time.perf_counter()
    DatasetWriter(fn, {'image': RGBImageField(write_mode='jpg', jpeg_quality=90), 'label': IntField()},
                  num_workers=min(8, os.cpu_count())).from_indexed_dataset(DS())
    t_write = time.perf_counter() - t0
    loader = Loader(fn, batch_size=512, num_workers=args.workers, order=OrderOption.RANDOM, seed=3,
                    drop_last=True, device='cpu',
                    pipelines={'image': [RandomResizedCropRGBImageDecoder((224, 224)), ToTensor()],
                               'label': [IntDecoder(), ToTensor()]})
    times = []
    n = 0
    for e in range(args.epochs):
        t0 = time.perf_counter()
        n = 0
        for b, (images, labels) in enumerate(loader):
            if e == 0 and b == 0:
                O.build()
                ids = np.random.default_rng(3).permutation(args.n)[:512]
                want = expected_rrc(O, samples_of(fn), ids, 3, 0, (224, 224))
                assert np.array_equal(images.numpy(), want), 'first batch differs from the oracle'
            n += images.shape[0]
        times.append(time.perf_counter() - t0)
    best = min(times[1:]) if len(times) > 1 else times[0]
    print(json.dumps({'config': 'CPU Loader, JPEG 256px q90 -> RRC 224 u8, batch 512, RANDOM, drop_last',
                      'samples_per_epoch': n, 'images_per_s': round(n / best, 1),
                      'epoch_s_all': [round(t, 3) for t in times], 'write_s': round(t_write, 2),
                      'workers': args.workers, 'host_cpus': os.cpu_count(),
                      'first_batch': 'bit-exact vs the oracle (libjpeg-turbo decode + C INTER_AREA)'}))


if __name__ == '__main__':
    main()
