"""Debug: the launch-groups test as written (three loaders zipped)."""
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
for extra in [dict(), dict(entropy_index=False)]:
    for trial in range(2):
        a = _c3_loader(fn, 7, drop_last=False, batches_per_launch=1, **extra)
        b = _c3_loader(fn, 7, drop_last=False, **extra)
        c = _c3_loader(fn, 7, drop_last=False, batches_per_launch=3, **extra)
        for epoch in range(2):
            bad = []
            for bi, ((ia, la), (ib, lb), (ic, lc)) in enumerate(zip(a, b, c)):
                for nm, x in (('b', ib), ('c', ic)):
                    dif = (ia.view(ch.int16) != x.view(ch.int16)).reshape(ia.shape[0], -1).any(1).nonzero().ravel().tolist()
                    if dif:
                        bad.append((nm, bi, dif[:6]))
            print(extra, 'trial', trial, 'epoch', epoch, 'bad', bad[:8], flush=True)
