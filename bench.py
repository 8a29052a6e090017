"""Benchmark of the MI355X decode-and-augment path (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3|c2|c5]

Workload (default, BASELINE.json configs[2] "C3"): an ImageNet-shape
1,281,167-sample JPEG dataset (synthetic natural images, long side 256,
aspect U(3/4,4/3), q90 4:2:0 baseline -- ~17 KB each like ImageNet at
max_resolution 256, docs/benchmarks.rst:43), resident in HBM; per step one
batch of 512 random-order samples goes through the hot path

    RandomResizedCropRGBImageDecoder((224,224)) -> Cutout(32,(124,116,103))
      -> ToTensor -> ToDevice -> ToTorchImage -> NormalizeImage(imagenet, fp16)

which lowers to: descriptor gather -> device crop/cutout draws ->
jpeg_entropy_kernel<RRC> (parse, de-stuff, parallel Huffman, IDCT of the crop's
MCUs) + jpeg_color_resize_kernel (upsample+colour, INTER_AREA, cutout, LUT).
The 1.28M-entry dataset
is built from U unique encodings replicated at distinct HBM addresses.

Multi-GPU: one process per GPU (torchrun), the epoch order sharded like
DistributedSampler (perm[rank::world]); no collective on the data path, a
barrier around the timed region; value = all ranks' images / max rank time.
"""
import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# 16 HIP hardware queues so the --inflight batches' streams do not share a
# queue.  HIP's default (and what the GPU box exports) is 4, so this is an
# override, set before torch initialises HIP; 8 batches in flight on 16
# queues measured fastest, more in flight far slower.
os.environ['GPU_MAX_HW_QUEUES'] = os.environ.get('FFCV_BENCH_HWQ', '16')

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec

CONFIGS = {
    # name: (mode, max_side, out, batch, cutout, normalize, dataset_size)
    'c3': ('jpg', 256, 224, 512, 32, True, 1281167),
    'c2': ('jpg', 256, 224, 256, 0, False, 10000),
    'c5': ('raw', 512, 448, 256, 64, False, 10000),
}
WORKLOAD = {
    'c3': 'C3: ImageNet-shape 1.28M-JPEG .beton (synthetic 256px q90 4:2:0), '
          'RRC 224 + Cutout(32) + NormalizeImage fp16, batch 512',
    'c2': 'C2: 10k-JPEG .beton (synthetic 256px q90), RRC 224 u8, batch 256',
    'c5': 'C5: raw 512x512 RGB .beton, RRC 448 + Cutout(64) u8, batch 256',
}
# batches in flight per config on 16 HW queues (A/B, 3 runs each):
# C3 10 vs 8 +1.5%, C5 4 vs 8 +1%; C2 (half-size batches) 14 vs 8 +25%, 16 collapses
INFLIGHT = {'c3': 10, 'c2': 14, 'c5': 4}
IMAGENET_MEAN = np.array([0.485, 0.456, 0.406]) * 255
IMAGENET_STD = np.array([0.229, 0.224, 0.225]) * 255


def _gen_one(args):
    from ffcv_amd.synthetic import natural_image, encode_jpeg, imagenet_like_shape
    i, mode, side, seed = args
    rng = np.random.default_rng(seed * 1000003 + i)
    if mode == 'raw':
        img = natural_image(rng, side, side)
        return img.reshape(-1).copy(), side, side
    h, w = imagenet_like_shape(rng, side)
    img = natural_image(rng, h, w)
    return encode_jpeg(img, 90, '4:2:0'), h, w


def make_unique(mode, side, n_unique, seed, workers):
    """Deterministic unique sample set; cached in /tmp across processes."""
    key = hashlib.sha1(f'{mode}-{side}-{n_unique}-{seed}-v1'.encode()).hexdigest()[:12]
    path = f'/tmp/ffcv_amd_bench_{key}.npz'
    if os.path.exists(path):
        z = np.load(path)
        return z['tile'], z['offs'], z['sizes'], z['hs'], z['ws']
    jobs = [(i, mode, side, seed) for i in range(n_unique)]
    if workers > 1:
        import multiprocessing as mp
        with mp.get_context('fork').Pool(workers) as pool:
            res = pool.map(_gen_one, jobs, chunksize=32)
    else:
        res = [_gen_one(j) for j in jobs]
    from ffcv_amd.synthetic import pack
    tile, offs, sizes = pack([r[0] for r in res])
    hs = np.array([r[1] for r in res], np.uint32)
    ws = np.array([r[2] for r in res], np.uint32)
    tmp = path + f'.{os.getpid()}.tmp.npz'
    np.savez(tmp, tile=tile, offs=offs, sizes=sizes, hs=hs, ws=ws)
    os.replace(tmp, path)
    return tile, offs, sizes, hs, ws


def cpu_threads():
    n = os.environ.get('OMP_NUM_THREADS')
    if n and n.isdigit() and int(n) > 0:
        return int(n)
    return len(os.sched_getaffinity(0))


def cpu_model():
    try:
        with open('/proc/cpuinfo') as f:
            for line in f:
                if line.startswith('model name'):
                    return line.split(':', 1)[1].strip()
    except OSError:
        pass
    return 'unknown'


def cpu_baseline(cfg, tile, offs, sizes, hs, ws, budget_s=10.0):
    """Oracle restatement of the same per-sample path, timed on host cores
    (all cores the process may use, plus 1 core)."""
    from oracle import oracle as O
    mode, side, out, batch, cut, norm, _ = CONFIGS[cfg]
    n_u = len(offs)
    lut = O.normalize_lut(IMAGENET_MEAN, IMAGENET_STD) if norm else None

    def run(threads, budget, bsz):
        done, b = 0, 0
        t0 = time.perf_counter()
        while True:
            idx = (np.arange(bsz) + b * bsz) % n_u
            samples = [(tile[offs[i]:offs[i] + sizes[i]], int(hs[i]), int(ws[i]), 0 if mode == 'jpg' else 1)
                       for i in idx]
            crops, cyx = O.draw_batch(idx.astype(np.uint64), hs[idx], ws[idx], 0, 0, out_h=out, out_w=out,
                                      cutout_size=cut)
            O.rrc_batch(samples, crops, out, out, cutout_yx=cyx, cutout_size=cut,
                        fill=(124, 116, 103), lut=lut, nthreads=threads)
            done += bsz
            b += 1
            el = time.perf_counter() - t0
            if el >= budget and b >= 2:
                return done, b, el

    threads = cpu_threads()
    done, b, el = run(threads, budget_s, batch)
    d1, b1, el1 = run(1, max(1.0, budget_s / 5), 32)  # 1 core, batches of 32
    what = ('scalar libjpeg-turbo ifast restatement + OpenCV INTER_AREA restatement' if mode == 'jpg'
            else 'raw crop view + OpenCV INTER_AREA restatement')
    return {'value': round(done / el, 1), 'unit': 'images/s', 'cores': threads, 'kind': 'port',
            'value_1core': round(d1 / el1, 1), 'cpu_model': cpu_model(),
            'sample': f'{done} images ({b} batches of {batch}) of the same workload cycled over '
                      f'{n_u} unique samples; oracle/ffcv_oracle.c ({what}), one sample per thread like '
                      f'numba prange, {el:.1f}s wall; 1 core: {d1} images in {el1:.1f}s'}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=400)
    ap.add_argument('--warmup', type=int, default=20)
    ap.add_argument('--config', default='c3', choices=list(CONFIGS))
    ap.add_argument('--unique', type=int, default=4096)
    ap.add_argument('--dataset-size', type=int, default=None)
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--cpu-budget', type=float, default=10.0)
    ap.add_argument('--batch', type=int, default=0, help='diagnostic: override the config batch size')
    ap.add_argument('--unfused', action='store_true',
                    help='separate gather / draw kernels before the decode (the Loader\'s staged path)')
    ap.add_argument('--only', type=int, default=0,
                    help='diagnostic: timed steps launch only these decode kernels (bit 0 K1, bit 2 K2)')
    ap.add_argument('--inflight', type=int, default=0,
                    help='batches in flight on separate HIP streams (Loader batches_ahead analogue); '
                         'default per config (INFLIGHT)')
    args = ap.parse_args()

    import torch
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    dist = None
    # one process per GPU; FFCV_BENCH_BACKEND=gloo + several ranks per GPU
    # (local % device_count) only rehearse the N>1 path on a 1-GPU box
    ndev = max(1, torch.cuda.device_count())
    gpu = local % ndev
    backend = os.environ.get('FFCV_BENCH_BACKEND', 'nccl')
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(gpu)
        if backend == 'nccl':
            dist.init_process_group('nccl', device_id=torch.device('cuda', gpu))
        else:
            dist.init_process_group(backend)
    dev = torch.device('cuda', gpu)
    torch.cuda.set_device(dev)

    from ffcv_amd import _build
    if local == 0:
        _build.build()
    if dist:
        dist.barrier()
    from ffcv_amd import libffcv as L

    mode, side, out, batch, cut, norm, default_n = CONFIGS[args.config]
    if args.batch:  # diagnostic: launch granularity (not the BASELINE config)
        batch = args.batch
    N = args.dataset_size or default_n
    workers = max(1, min(16, cpu_threads() // max(1, world)))
    if local == 0:
        tile, offs, sizes, hs, ws = make_unique(mode, side, args.unique, 0, workers)
    if dist:
        dist.barrier()
    if local != 0:
        tile, offs, sizes, hs, ws = make_unique(mode, side, args.unique, 0, workers)
    U = len(offs)
    tile_len = int(offs[-1] + (sizes[-1] + 7) // 8 * 8)
    reps = (N + U - 1) // U

    # ---- HBM-resident dataset: U encodings replicated at distinct addresses
    d_tile = torch.from_numpy(tile[:tile_len]).to(dev)
    d_data = torch.empty(reps * tile_len + 64, dtype=torch.uint8, device=dev)
    for r in range(reps):
        d_data[r * tile_len:(r + 1) * tile_len].copy_(d_tile)
    del d_tile
    k = np.arange(N)
    table = np.zeros(N, L.SAMPLE_DTYPE)
    table['offset'] = (k // U).astype(np.uint64) * tile_len + offs[k % U]
    table['size'] = sizes[k % U]
    table['height'] = hs[k % U]
    table['width'] = ws[k % U]
    table['mode'] = 0 if mode == 'jpg' else 1
    d_table = torch.from_numpy(table.view(np.uint8)).to(dev)
    mean_bytes = float(sizes.mean())

    # ---- epoch order, DistributedSampler-style sharding, resident on device
    perm = np.random.default_rng(0).permutation(N)
    if world > 1:
        total = (N + world - 1) // world * world
        perm = np.concatenate([perm, perm[:total - N]])[rank::world]
    need = (args.warmup + args.steps) * batch
    order = np.resize(perm, need).astype(np.int64)
    d_order = torch.from_numpy(order).to(dev)

    # ---- per-slot buffers: --inflight batches overlap on their own HIP
    # streams (the Loader's batches_ahead slots do the same), each slot with
    # its own decoder scratch; a slot's next batch is ordered behind its last.
    K = max(1, args.inflight or INFLIGHT[args.config])
    out_dtype = torch.float16 if norm else torch.uint8
    streams = [torch.cuda.Stream(dev) for _ in range(K)]
    slots = []
    for _ in range(K):
        slots.append({
            'smp': torch.empty(batch * 32, dtype=torch.uint8, device=dev),
            'crops': torch.empty((batch, 4), dtype=torch.int32, device=dev),
            'cut': torch.empty((batch, 2), dtype=torch.int32, device=dev) if cut else None,
            'status': torch.empty(batch, dtype=torch.int32, device=dev),
            'rstat': torch.empty(batch, dtype=torch.int32, device=dev),
            'out': torch.empty((batch, out, out, 3), dtype=out_dtype, device=dev),
            'dec': (L.JpegDecoder(batch, int(hs.max()), int(ws.max()), int(sizes.max()))
                    if mode == 'jpg' else None),
        })
    d_lut = None
    rp = L.RRCParams()
    rp.out_h = rp.out_w = out
    rp.cutout_size = cut
    for i, f in enumerate((124, 116, 103) if cut == 32 else (0, 0, 0)):
        rp.cutout_fill[i] = f
    if norm:
        from ffcv_amd.transforms.lut import make_lut as normalize_lut
        d_lut = torch.from_numpy(normalize_lut(IMAGENET_MEAN, IMAGENET_STD).view(np.int16)).to(dev)
        rp.lut = d_lut.data_ptr()
    dp = L.DrawParams()
    dp.crop_kind = 0
    dp.out_h = dp.out_w = out
    dp.cutout_size = cut
    dp.scale[0], dp.scale[1] = 0.08, 1.0
    dp.ratio[0], dp.ratio[1] = 0.75, 4 / 3
    dp.loader_seed = 0
    dp.epoch = 0
    torch.cuda.synchronize()

    def step(i, ev=None):
        sl = slots[i % K]
        stream = streams[i % K]
        ids = d_order[i * batch:(i + 1) * batch]
        if sl['dec'] is not None and not args.unfused:
            # gather + draws fused into the entropy kernel (ffcv_jpeg_rrc_fused)
            if ev is not None:
                ev[0].record(stream)
            sl['dec'].rrc_fused(d_data, d_table, ids, dp, sl['crops'], sl['cut'], None, rp, sl['out'],
                                sl['status'], stream=stream)
            if ev is not None:
                ev[1].record(stream)
            return
        L.gather_samples(d_table, ids, sl['smp'], stream)
        L.draw_batch(ids, sl['smp'], dp, sl['crops'], sl['cut'], None, sl['rstat'], stream)
        if ev is not None:
            ev[0].record(stream)
        if sl['dec'] is not None:
            sl['dec'].rrc(d_data, sl['smp'], batch, sl['crops'], sl['cut'], None, rp, sl['out'], sl['status'],
                          stream)
        else:
            L.rrc_raw_batch(d_data, sl['smp'], batch, sl['crops'], sl['cut'], None, rp, sl['out'], stream)
        if ev is not None:
            ev[1].record(stream)

    for i in range(args.warmup):
        step(i)
    torch.cuda.synchronize()
    if mode == 'jpg':
        for sl in slots:
            st = sl['status'].cpu().numpy()
            assert (st == 0).all(), f'decode status {np.unique(st)}'
    events = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(args.steps)]
    if args.only:
        os.environ['FFCV_JPEG_ONLY'] = str(args.only)
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(args.warmup + i, events[i])
    host_s = time.perf_counter() - t0  # host submission time of the K steps
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in events]))
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev if backend == 'nccl' else 'cpu')
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    imgs = world * batch * args.steps
    value = imgs / elapsed
    if mode == 'jpg':
        unit_bytes = mean_bytes + out * out * 3 * (2 if norm else 1)
        roof_note = (f'S_jpeg + {out}*{out}*3*{2 if norm else 1} ({"fp16" if norm else "u8"} out) '
                     f'per image (SURVEY 8d {args.config.upper()})')
    else:
        # crop ROI read (E[h*w]/(H*W) measured per batch below) + output write
        crops_np = slots[0]['crops'].cpu().numpy()
        unit_bytes = float((crops_np[:, 2].astype(np.float64) * crops_np[:, 3] * 3).mean()) + out * out * 3
        roof_note = '3*h*w crop ROI read + 448*448*3 write per image (SURVEY 8d C5)'
    achieved = unit_bytes * batch / (kern_ms * 1e-3) / 1e9
    res = {
        'metric': 'device-resident images/s, JPEG->RRC 224x224 batch 512; HBM GB/s vs peak',
        'value': round(value, 1),
        'unit': 'images/s',
        'n_gpus': world,
        'steps': args.steps,
        'warmup': args.warmup,
        'ms_per_step': round(elapsed / args.steps * 1e3, 4),
        'host_submit_ms_per_step': round(host_s / args.steps * 1e3, 4),
        'higher_is_better': True,
        'scaling': 'weak',
        'vs_baseline': None,
        'dtype': 'u8',
        'data': f'synthetic ({U} unique encodings replicated to {N} HBM-resident samples)',
        'config': {'workload': WORKLOAD[args.config], 'global_batch': batch * world,
                   'per_gpu_batch': batch, 'inflight_batches': K,
                   'hip_hw_queues': int(os.environ['GPU_MAX_HW_QUEUES']), 'dataset_size': N, 'mean_sample_bytes': round(mean_bytes, 1),
                   'parallelism': f'dp{world} (traversal-order sharding, no collectives)'},
        'roofline': {'bound': 'hbm', 'achieved': round(achieved, 2), 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                     'frac': round(achieved / HBM_PEAK_GBS, 5), 'traffic': None,
                     'kernel': ('jpeg_entropy_kernel<RRC> + jpeg_color_resize_kernel<RRC,fp16> '
                                '(one decode launch sequence, HIP events on the slot stream)'
                                if mode == 'jpg' else 'rrc_raw_kernel'),
                     'kernel_ms': round(kern_ms, 4), 'algorithmic_bytes_per_image': round(unit_bytes, 1),
                     'note': roof_note,
                     # launches overlap (K in flight), so one launch's duration includes
                     # GPU time it shares: the whole-job algorithmic rate beside it
                     'job_achieved': round(value * unit_bytes / 1e9, 2),
                     'job_frac': round(value * unit_bytes / 1e9 / HBM_PEAK_GBS, 5)},
        'cpu_baseline': None,
    }
    # HBM traffic of the same kernels from the committed rocprofv3 PMC passes
    # (tools/profile.sh -> tools/pmc_summary.py), per launch like `achieved`
    prof = os.path.join(ROOT, 'profiles', f'traffic_{args.config}.json')
    if os.path.exists(prof):
        pm = json.load(open(prof))
        names = (['jpeg_entropy_kernel<0>', 'jpeg_color_resize_kernel<0, true>']
                 if mode == 'jpg' else ['rrc_raw_kernel<false>'])
        if all(n in pm and 'fetch_size_kb' in pm[n] and 'write_size_kb' in pm[n] for n in names):
            tb = sum((pm[n]['fetch_size_kb'] + pm[n]['write_size_kb']) * 1024.0 for n in names)
            res['roofline']['traffic'] = round(tb, 1)
            res['roofline']['traffic_note'] = (f'bytes per launch (FETCH_SIZE + WRITE_SIZE, rocprofv3 PMC, '
                                               f'profiles/traffic_{args.config}.json); algorithmic '
                                               f'{unit_bytes * batch:.0f}')
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        res['cpu_baseline'] = cpu_baseline(args.config, tile, offs, sizes, hs, ws, args.cpu_budget)
    if rank == 0:
        print(json.dumps(res), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
