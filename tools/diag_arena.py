# Arena diagnosis: large fused launches, per-launch status and arena high
# water (ffcv_jpeg_arena_used).  GPU box:  python tools/diag_arena.py
import sys, os
sys.path.insert(0, os.getcwd())
import numpy as np, torch
from bench import make_unique
from ffcv_amd import libffcv as L
tile, offs, sizes, hs, ws = make_unique('jpg', 256, 4096, 0, 16)
dev = torch.device('cuda:0')
U = len(offs); N = 20480
tile_len = int(offs[-1] + (sizes[-1] + 7) // 8 * 8)
reps = (N + U - 1) // U
d_data = torch.empty(reps * tile_len + 64, dtype=torch.uint8, device=dev)
dt = torch.from_numpy(tile[:tile_len]).to(dev)
for r in range(reps): d_data[r*tile_len:(r+1)*tile_len].copy_(dt)
k = np.arange(N)
table = np.zeros(N, L.SAMPLE_DTYPE)
table['offset'] = (k // U).astype(np.uint64) * tile_len + offs[k % U]
table['size'] = sizes[k % U]; table['height'] = hs[k % U]; table['width'] = ws[k % U]
d_table = torch.from_numpy(table.view(np.uint8)).to(dev)
for cap, mult in ((10240, 1), (10240, 2), (10240, 0.5)):
    arena = int(L.arena_for(hs, ws, sizes, cap) * mult)
    dec = L.JpegDecoder(cap, int(hs.max()), int(ws.max()), int(sizes.max()), arena)
    ids = torch.from_numpy(np.random.default_rng(0).permutation(N)[:cap].astype(np.int64)).to(dev)
    dp = L.DrawParams(); dp.out_h = dp.out_w = 224; dp.scale[0], dp.scale[1] = 0.08, 1.0; dp.ratio[0], dp.ratio[1] = 0.75, 4/3
    rp = L.RRCParams(); rp.out_h = rp.out_w = 224
    crops = torch.empty((cap, 4), dtype=torch.int32, device=dev)
    out = torch.empty((cap, 224, 224, 3), dtype=torch.uint8, device=dev)
    st = torch.full((cap,), -1, dtype=torch.int32, device=dev)
    dec.rrc_fused(d_data, d_table, ids, dp, crops, None, None, rp, out, st)
    torch.cuda.synchronize()
    s = st.cpu().numpy()
    bad = np.nonzero(s)[0]
    need = L.scratch_bound(hs, ws, sizes)
    print('cap', cap, 'mult', mult, 'arena', arena, 'bad', bad.size, 'first bad k', bad[:5], 'codes', np.unique(s[bad]))
    del dec
# the failing ids alone, in a small launch
bad_ids = ids.cpu().numpy()[bad]
cap2 = min(1024, bad_ids.size)
if cap2 == 0:
    bad_ids, cap2 = ids.cpu().numpy()[:16], 16
dec = L.JpegDecoder(cap2, int(hs.max()), int(ws.max()), int(sizes.max()), L.arena_for(hs, ws, sizes, cap2))
ids2 = torch.from_numpy(bad_ids[:cap2]).to(dev)
crops = torch.empty((cap2, 4), dtype=torch.int32, device=dev)
out = torch.empty((cap2, 224, 224, 3), dtype=torch.uint8, device=dev)
st = torch.full((cap2,), -1, dtype=torch.int32, device=dev)
dec.rrc_fused(d_data, d_table, ids2, dp, crops, None, None, rp, out, st)
torch.cuda.synchronize()
print('failing ids alone: bad', int((st.cpu().numpy() != 0).sum()), 'of', cap2)
# growing launches: where does the first failure appear?
for cap3 in (9000, 9200, 9400, 9600):
    dec = L.JpegDecoder(cap3, int(hs.max()), int(ws.max()), int(sizes.max()), L.arena_for(hs, ws, sizes, cap3))
    ids3 = torch.from_numpy(np.arange(cap3, dtype=np.int64)).to(dev)
    crops = torch.empty((cap3, 4), dtype=torch.int32, device=dev)
    out = torch.empty((cap3, 224, 224, 3), dtype=torch.uint8, device=dev)
    st = torch.full((cap3,), -1, dtype=torch.int32, device=dev)
    dec.rrc_fused(d_data, d_table, ids3, dp, crops, None, None, rp, out, st)
    torch.cuda.synchronize()
    s = st.cpu().numpy()
    print('sequential ids cap', cap3, 'bad', int((s != 0).sum()), 'first', np.nonzero(s)[0][:3], 'arena used/cap', dec.arena_used())
