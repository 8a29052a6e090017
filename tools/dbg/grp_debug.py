"""Debug: which batches/images differ between launch-group settings."""
import os, sys, tempfile
import numpy as np
import torch as ch
sys.path.insert(0, os.getcwd())
sys.path.insert(0, os.path.join(os.getcwd(), 'tests'))
from test_loader_gpu import _c3_loader, write, NaturalDS
from ffcv_amd.fields import RGBImageField, IntField
d = tempfile.mkdtemp()
fn = os.path.join(d, 'grp.beton')
write(fn, NaturalDS(100, hw=(80, 96), var=True, seed=6), {'image': RGBImageField(write_mode='jpg'), 'label': IntField()})
for kw in [dict(batches_per_launch=1), dict(), dict(batches_per_launch=3), dict(batches_per_launch=1, entropy_index=False), dict(entropy_index=False)]:
    outs = []
    for rep in range(2):
        L = _c3_loader(fn, 7, drop_last=False, **kw)
        ep = []
        for e in range(2):
            ep.append(ch.cat([x[0].view(ch.int16).cpu() for x in L]))
        outs.append(ep)
    print(kw, 'rep-equal', [bool(ch.equal(outs[0][e], outs[1][e])) for e in range(2)], flush=True)
    if not kw:
        base = outs[0]
    globals().setdefault('ref', outs[0])
    diff = [(ref[e] != outs[0][e]).reshape(100, -1).any(1).nonzero().ravel().tolist() for e in range(2)]
    print('   vs batches_per_launch=1 differing images per epoch:', [x[:20] for x in diff], flush=True)
