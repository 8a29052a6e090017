"""Diagnostic: per-phase timing of jpeg_entropy_kernel<RRC> via in-kernel stamps.

Runs one batch with the debug stamp buffer enabled (diagnostic only: the
stamps are written to their own buffer and never read by the kernel).
"""
import ctypes, os, sys, time
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from ffcv_amd import libffcv as L
if len(sys.argv) > 2:
    L.LIB_PATH = os.path.abspath(sys.argv[2])  # a -DFFCV_K1_DIAG build (tools/build_variant.sh)
from bench import make_unique, IMAGENET_MEAN, IMAGENET_STD
from ffcv_amd.transforms.lut import make_lut

B = int(sys.argv[1]) if len(sys.argv) > 1 else 512
tile, offs, sizes, hs, ws = make_unique('jpg', 256, 4096, 0, 16)
dev = torch.device('cuda:0')
d_data = torch.from_numpy(tile).to(dev)
idx = np.resize(np.random.default_rng(1).permutation(len(offs)), B)  # (repeats past the unique count)
smp = np.zeros(B, L.SAMPLE_DTYPE)
smp['offset'] = offs[idx]; smp['size'] = sizes[idx]; smp['height'] = hs[idx]; smp['width'] = ws[idx]
d_smp = torch.from_numpy(smp.view(np.uint8)).to(dev)
d_ids = torch.from_numpy(idx.astype(np.int64)).to(dev)
crops = torch.empty((B, 4), dtype=torch.int32, device=dev)
cut = torch.empty((B, 2), dtype=torch.int32, device=dev)
dp = L.DrawParams(); dp.out_h = dp.out_w = 224; dp.cutout_size = 32
dp.scale[0], dp.scale[1] = 0.08, 1.0; dp.ratio[0], dp.ratio[1] = 0.75, 4/3
L.draw_batch(d_ids, d_smp, dp, crops, cut, None, None)
lut = torch.from_numpy(make_lut(IMAGENET_MEAN, IMAGENET_STD).view(np.int16)).to(dev)
rp = L.RRCParams(); rp.out_h = rp.out_w = 224; rp.cutout_size = 32; rp.lut = lut.data_ptr()
out = torch.empty((B, 224, 224, 3), dtype=torch.float16, device=dev)
status = torch.empty(B, dtype=torch.int32, device=dev)
dec = L.JpegDecoder(B, 256, 256, int(sizes.max()))
dbg = torch.zeros((B, 16), dtype=torch.int64, device=dev)
L.lib().ffcv_jpeg_set_debug.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
for it in range(3):
    L.lib().ffcv_jpeg_set_debug(dec.handle, ctypes.c_void_p(dbg.data_ptr() if it == 2 else 0))
    torch.cuda.synchronize(); t0 = time.perf_counter()
    dec.rrc(d_data, d_smp, B, crops, cut, None, rp, out, status)
    torch.cuda.synchronize(); print('iter', it, 'ms', (time.perf_counter() - t0) * 1e3)
d = dbg.cpu().numpy()
names = ['parse', 'tables', 'destuff', 'sync', 'scan', 'write', 'dcpred', 'info', 'idct']
print('phase means (us):')
for i, n in enumerate(names):
    dt = (d[:, i + 1] - d[:, i]) / 100.0
    print(f'  {n:12s} mean {dt.mean():8.1f}  p50 {np.median(dt):8.1f}  max {dt.max():8.1f}')
for n, (i0, i1) in (('  header load', (0, 10)), ('  parse+barrier', (10, 1))):
    dt = (d[:, i1] - d[:, i0]) / 100.0
    print(f'  {n:12s} mean {dt.mean():8.1f}  p50 {np.median(dt):8.1f}  max {dt.max():8.1f}')
tot = (d[:, 9] - d[:, 0]) / 100.0
print('  total        mean', tot.mean(), 'max', tot.max())
print('span of K1 us', (d[:, 9].max() - d[:, 0].min()) / 100.0)
print('rounds hist', np.bincount(d[:, 12].astype(int))[:20], 'nthr mean', d[:, 13].mean())
st = (d[:, 0] - d[:, 0].min()) / 100.0
print('start offsets us: p50', np.median(st), 'max', st.max())
print('sync wave-iterations mean', d[:, 14].mean(), 'max', d[:, 14].max(), '| write wave-iterations mean', d[:, 15].mean(), 'max', d[:, 15].max())
# workgroup hold: a K1 workgroup (JW images, one per wave) keeps its LDS until
# its slowest image is done; idle = the other waves' time between their own
# end and the workgroup's end
JW = int(os.environ.get('JW', '4'))
n = (B // JW) * JW
s0 = d[:n, 0].reshape(-1, JW).astype(np.float64); e = d[:n, 9].reshape(-1, JW).astype(np.float64)
wg_end = e.max(1, keepdims=True); wg_start = s0.min(1, keepdims=True)
busy = (e - s0).sum(); held = (wg_end - s0).sum()
print(f'workgroup hold: busy wave-time {busy / 100:.0f} us, held {held / 100:.0f} us, idle fraction {1 - busy / held:.3f}')
print(f'per-image busy us: mean {((e - s0) / 100).mean():.1f} cv {((e - s0).std() / (e - s0).mean()):.3f}')
# K2 bands on the general path (slot 11, counted by jpeg_color_resize_kernel)
nb = (224 + 15) // 16
g = d[:, 11]
print(f'K2 general-path bands: {g.sum()} of {B * nb} ({g.sum() / (B * nb):.3f}); images with any: {(g > 0).mean():.3f}')
