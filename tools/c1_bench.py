"""C1 (BASELINE.json configs[0]): CIFAR-shape raw 32x32 RGBImageField
+ IntField .beton of 50,000 samples, default pipelines (SimpleRGBImageDecoder +
ToTensor, IntDecoder + ToTensor), batch 512, SEQUENTIAL, drop_last, on a
CPU-only Loader.  Reference figure: 0.02828 s per epoch = ~1.76 M images/s
(docs/ffcv_examples/custom_transforms.rst:133-156, its hardware, 8 workers).

    python tools/c1_bench.py [--n 50000] [--epochs 5] [--workers 8]
"""
import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--n', type=int, default=50000)
    ap.add_argument('--epochs', type=int, default=5)
    ap.add_argument('--workers', type=int, default=8)
    args = ap.parse_args()
    from ffcv_amd.writer import DatasetWriter
    from ffcv_amd.fields import RGBImageField, IntField
    from ffcv_amd.loader import Loader, OrderOption

    rng = np.random.default_rng(0)
    imgs = rng.integers(0, 256, (args.n, 32, 32, 3), dtype=np.uint8)

    class DS:
        def __len__(self):
            return args.n

        def __getitem__(self, i):
            return imgs[i], i % 10

    d = tempfile.mkdtemp()
    fn = os.path.join(d, 'c1.beton')
    t0 = time.perf_counter()
    DatasetWriter(fn, {'image': RGBImageField(write_mode='raw'), 'label': IntField()},
                  num_workers=min(8, os.cpu_count())).from_indexed_dataset(DS())
    t_write = time.perf_counter() - t0
    loader = Loader(fn, batch_size=512, num_workers=args.workers, order=OrderOption.SEQUENTIAL,
                    drop_last=True, device='cpu')
    times = []
    for e in range(args.epochs + 1):
        t0 = time.perf_counter()
        n = 0
        for images, labels in loader:
            n += images.shape[0]
        times.append(time.perf_counter() - t0)
    # exactness of the first batch (images and labels) against the source
    first, first_labels = next(iter(loader))
    ok = bool(np.array_equal(first.numpy(), imgs[:512])
              and np.array_equal(np.asarray(first_labels).reshape(-1), np.arange(512) % 10))
    assert ok, 'C1 first batch differs from the source samples'
    best = min(times[1:])
    print(json.dumps({'config': 'C1: raw 32x32 + int, batch 512, SEQUENTIAL, drop_last, CPU Loader',
                      'value': round(n / best, 1), 'unit': 'images/s',
                      'first_batch_exact': ok,
                      'samples_per_epoch': n, 'epoch_s_best': round(best, 5),
                      'images_per_s': round(n / best, 1), 'epoch_s_all': [round(t, 5) for t in times],
                      'first_epoch_s': round(times[0], 5), 'write_s': round(t_write, 2),
                      'workers': args.workers, 'host_cpus': os.cpu_count(),
                      'reference': '0.02828 s/epoch = 1.76 M images/s (docs, its hardware)'}))


if __name__ == '__main__':
    main()
