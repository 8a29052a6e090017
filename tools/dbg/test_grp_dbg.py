"""Debug (not part of the suite): the launch-group test with per-loader oracle checks."""
import os
import tempfile
import numpy as np
import pytest
import torch as ch
from tests.helpers import NaturalDS, write, samples_of, expected_rrc
from tests.test_loader_gpu import _c3_loader, MEAN, STD
from ffcv_amd.fields import RGBImageField, IntField
from tests.conftest import oracle, hip_lib  # noqa: F401 (fixtures)

pytestmark = pytest.mark.gpu


def test_grp_debug(oracle):
    d = tempfile.mkdtemp()
    fn = os.path.join(d, 'grp.beton')
    write(fn, NaturalDS(100, hw=(80, 96), var=True, seed=6), {'image': RGBImageField(write_mode='jpg'), 'label': IntField()})
    samples = samples_of(fn)
    lut = oracle.normalize_lut(MEAN, STD)
    a = _c3_loader(fn, 7, drop_last=False, batches_per_launch=1)
    b = _c3_loader(fn, 7, drop_last=False)
    c = _c3_loader(fn, 7, drop_last=False, batches_per_launch=3)
    report = []
    for epoch in range(2):
        order = np.random.default_rng(7 + epoch).permutation(100)
        for bi, ((ia, la), (ib, lb), (ic, lc)) in enumerate(zip(a, b, c)):
            ids = order[bi * 16:(bi + 1) * 16]
            want = expected_rrc(oracle, samples, ids, 7, epoch, (64, 64), cutout=12, fill=(124, 116, 103), lut=lut)
            for nm, x in (('a', ia), ('b', ib), ('c', ic)):
                got = x.permute(0, 2, 3, 1).cpu().numpy()
                bad = np.nonzero((got.view(np.uint16) != want.view(np.uint16)).reshape(len(ids), -1).any(1))[0]
                if bad.size:
                    g, w = got.view(np.uint16)[bad[0]], want.view(np.uint16)[bad[0]]
                    nbad = int((g != w).sum())
                    report.append((epoch, bi, nm, bad.tolist(), ids[bad].tolist(), nbad))
    print('REPORT', report)
    assert not report, report
