"""Loader-level throughput of the north-star pipeline through the drop-in API.

    python tools/loader_bench.py [--n 20000] [--epochs 2] [--batch 512]

Writes a synthetic ImageNet-shape JPEG .beton (256-px long side, q90 4:2:0,
the bench generator) with ffcv_amd.writer.DatasetWriter, then iterates

    Loader(fn, batch_size=512, order=RANDOM, pipelines={'image': [
        RandomResizedCropRGBImageDecoder((224, 224)), Cutout(32, (124, 116, 103)),
        ToTensor(), ToDevice('cuda:0'), ToTorchImage(), NormalizeImage(mean, std, fp16)],
        'label': [IntDecoder(), ToTensor(), ToDevice('cuda:0')]})

in four modes and prints one JSON line per mode:
  * device_cache   : the .beton is copied to HBM once; per batch only indices
                     move (the bench.py workload, seen through the Loader);
                     the Loader's default entropy index is filled by the
                     warm-up epoch, so the timed epochs skip the sync rounds
  * device_cache_noindex : the same with entropy_index=False (every epoch
                     decodes like the first)
  * pcie_in        : device_cache=False: per batch the compressed byte ranges
                     are gathered from the mmap into pinned staging and copied
                     host -> device (hipMemcpyAsync) before decoding
  * pcie_in_out    : as pcie_in, and each decoded fp16 batch is copied back to
                     pinned host memory (the path starts and ends in host memory)
  * pcie_in_process_cache : as pcie_in with os_cache=False: the page scheduler
                     preads the batches' .beton pages into a slot pool and
                     the native gather reads the samples out of the slots
  * link           : bare pinned hipMemcpyAsync H2D and D2H rates of one
                     decoded fp16 batch (154 MB), the ceiling of pcie_in_out
Images/s is measured over whole epochs after one warm-up epoch.  In
pcie_in_out the decoded batches leave on a dedicated copy stream into a
ring of pinned host buffers (double-buffered), so the D2H of batch b
overlaps the decode of the following batches.
"""
import argparse
import json
import os
import sys
import tempfile
import time
import types

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--n', type=int, default=20000)
    ap.add_argument('--epochs', type=int, default=2)
    ap.add_argument('--batch', type=int, default=512)
    ap.add_argument('--dir', default=None)
    ap.add_argument('--modes', default='link,device_cache,device_cache_noindex,pcie_in,pcie_in_out,'
                                       'pcie_in_process_cache')
    args = ap.parse_args()

    import torch
    from bench import make_unique, IMAGENET_MEAN, IMAGENET_STD
    from ffcv_amd.writer import DatasetWriter
    from ffcv_amd.fields import RGBImageField, IntField
    from ffcv_amd.fields.decoders import RandomResizedCropRGBImageDecoder, IntDecoder
    from ffcv_amd.transforms import ToTensor, ToDevice, ToTorchImage, NormalizeImage, Cutout
    from ffcv_amd.loader import Loader, OrderOption

    tile, offs, sizes, hs, ws = make_unique('jpg', 256, 4096, 0, 16)

    class DS:  # pre-encoded JPEG bytes, written as-is (RGBImageField jpg passthrough)
        def __len__(self):
            return args.n

        def __getitem__(self, i):
            u = i % len(offs)
            return (tile[offs[u]:offs[u] + sizes[u]], int(hs[u]), int(ws[u])), i % 1000

    d = args.dir or tempfile.mkdtemp(dir='/tmp')
    fn = os.path.join(d, f'loader_bench_{args.n}.beton')
    if not os.path.exists(fn):
        t0 = time.perf_counter()
        field = RGBImageField(write_mode='jpg')
        field.encode = types.MethodType(_encode_prepared, field)  # stays an RGBImageField
        DatasetWriter(fn, {'image': field, 'label': IntField()}, num_workers=1).from_indexed_dataset(DS())
        print(f'# wrote {fn} ({os.path.getsize(fn) / 1e6:.1f} MB) in {time.perf_counter() - t0:.1f}s',
              file=sys.stderr)
    dev = torch.device('cuda:0')
    for mode in args.modes.split(','):
        if mode == 'link':
            print(json.dumps(link_rates(torch, dev, args.batch * 224 * 224 * 3 * 2)), flush=True)
            continue
        loader = Loader(fn, batch_size=args.batch, order=OrderOption.RANDOM, seed=0, drop_last=True,
                        device=dev, device_cache=mode.startswith('device_cache'),
                        entropy_index=(mode != 'device_cache_noindex'),
                        os_cache=(mode != 'pcie_in_process_cache'),
                        pipelines={'image': [RandomResizedCropRGBImageDecoder((224, 224)),
                                             Cutout(32, (124, 116, 103)), ToTensor(), ToDevice(dev),
                                             ToTorchImage(), NormalizeImage(IMAGENET_MEAN, IMAGENET_STD,
                                                                            np.float16)],
                                   'label': [IntDecoder(), ToTensor(), ToDevice(dev)]})
        # the batch comes back in its channels-last memory order (the
        # ToTorchImage view's storage), so the D2H copy is one memcpy
        nbuf = 3
        hosts = [torch.empty((args.batch, 224, 224, 3), dtype=torch.float16).pin_memory() for _ in range(nbuf)]
        copy_stream = torch.cuda.Stream(dev)
        copied = [None] * nbuf
        k = 0
        n_img = 0
        t0 = None
        for ep in range(args.epochs + 1):
            if ep == 1:
                torch.cuda.synchronize()
                t0 = time.perf_counter()
            for images, labels in loader:
                if mode == 'pcie_in_out':
                    slot = k % nbuf
                    if copied[slot] is not None:
                        copied[slot].synchronize()  # the host buffer is free again
                    copy_stream.wait_stream(torch.cuda.current_stream(dev))
                    with torch.cuda.stream(copy_stream):
                        hosts[slot].copy_(images.permute(0, 2, 3, 1), non_blocking=True)
                        images.record_stream(copy_stream)
                        ev = torch.cuda.Event()
                        ev.record(copy_stream)
                    copied[slot] = ev
                    k += 1
                if ep >= 1:
                    n_img += images.shape[0]
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        print(json.dumps({'mode': mode, 'images_per_s': round(n_img / el, 1), 'images': n_img,
                          'seconds': round(el, 3), 'batch': args.batch, 'dataset': args.n,
                          'beton_mb': round(os.path.getsize(fn) / 1e6, 1)}), flush=True)


def link_rates(torch, dev, nbytes, reps=20):
    """Pinned host <-> HBM copy rates (GB/s) for a buffer of nbytes."""
    d = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    h = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
    out = {'mode': 'link', 'bytes': nbytes}
    for name, dst, src in (('h2d', d, h), ('d2h', h, d)):
        for _ in range(3):
            dst.copy_(src, non_blocking=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            dst.copy_(src, non_blocking=True)
        torch.cuda.synchronize()
        out[name + '_gbs'] = round(nbytes * reps / (time.perf_counter() - t0) / 1e9, 2)
    return out


def _encode_prepared(self, destination, item, malloc):
    """RGBImageField.encode for bytes that are already a JPEG (the bench
    generator's encodings), laid out exactly as the jpg branch writes them."""
    data, h, w = item
    destination['mode'] = 0  # IMAGE_MODES['jpg']
    destination['height'], destination['width'] = h, w
    destination['data_ptr'], storage = malloc(data.nbytes)
    storage[:] = data


if __name__ == '__main__':
    main()
