"""Loader plumbing on a CPU-only Loader (the reference's C1 config:
raw RGBImageField + IntField, default pipelines, no GPU).  Mirrors the
assertion intent of test_image_pipeline.py (raw), test_partial_batches.py,
test_loader_filter.py and test_basic_pipeline.py."""
import os
import tempfile

import numpy as np
import pytest
import torch as ch

from ffcv_amd.loader import Loader, OrderOption
from ffcv_amd.fields import RGBImageField, IntField, BytesField
from ffcv_amd.fields.decoders import SimpleRGBImageDecoder, IntDecoder, RandomResizedCropRGBImageDecoder
from ffcv_amd.transforms import ToTensor, NormalizeImage, Cutout, RandomHorizontalFlip
from tests.helpers import ConstDS, NaturalDS, write


@pytest.fixture(scope='module')
def raw_beton(hip_lib):
    d = tempfile.mkdtemp()
    fn = write(os.path.join(d, 'raw.beton'), ConstDS(500, hw=(32, 32)),
               {'index': IntField(), 'value': RGBImageField(write_mode='raw')})
    return fn


def test_simple_raw_pipeline_cpu(raw_beton):
    loader = Loader(raw_beton, batch_size=7, num_workers=2, device='cpu')
    seen = 0
    for index, images in loader:
        assert isinstance(images, ch.Tensor) and images.device.type == 'cpu'
        assert images.shape[1:] == (32, 32, 3) and images.dtype == ch.uint8
        for i, image in zip(index, images):
            assert ch.all(image == (int(i) % 255))
            seen += 1
    assert seen == 500 // 7 * 7


@pytest.mark.parametrize('bs,drop_last,expected', [(7, True, 71), (7, False, 72), (60, True, 8),
                                                   (60, False, 9)])
def test_partial_batches(raw_beton, bs, drop_last, expected):
    loader = Loader(raw_beton, batch_size=bs, drop_last=drop_last, device='cpu')
    assert len(loader) == expected
    assert len(list(loader)) == expected


def test_random_order_matches_reference_semantics(raw_beton):
    loader = Loader(raw_beton, batch_size=10, order=OrderOption.RANDOM, seed=123, device='cpu',
                    drop_last=False)
    for epoch in range(2):
        got = np.concatenate([ix.numpy().reshape(-1).copy() for ix, _ in loader])
        want = np.random.default_rng(123 + epoch).permutation(np.arange(500, dtype='uint64'))
        assert np.array_equal(got, want)


def test_disabled_field_and_filter(raw_beton):
    loader = Loader(raw_beton, batch_size=8, device='cpu', pipelines={'value': None})
    batch = next(iter(loader))
    assert len(batch) == 1
    filtered = Loader(raw_beton, batch_size=8, device='cpu').filter('index', lambda x: int(x) % 3 == 0)
    idx = np.concatenate([ix.numpy().reshape(-1).copy() for ix, _ in filtered])
    assert (idx % 3 == 0).all() and len(idx) == len(filtered) * 8


def test_indices_subset(raw_beton):
    loader = Loader(raw_beton, batch_size=5, device='cpu', indices=[3, 10, 11, 400, 499])
    (ix, im), = list(loader)
    assert ix.reshape(-1).tolist() == [3, 10, 11, 400, 499]


def test_host_transforms_follow_contract(raw_beton):
    """Host Cutout/flip/normalize on numpy (no GPU) use the seeding contract."""
    from ffcv_amd.transforms.rng import contract_seed
    mean, std = np.array([0., 1., 2.]), np.array([1., 10., 20.])
    loader = Loader(raw_beton, batch_size=6, device='cpu', seed=5,
                    pipelines={'value': [SimpleRGBImageDecoder(), Cutout(8, (1, 2, 3)),
                                         NormalizeImage(mean, std, np.float16), ToTensor()]})
    ix, im = next(iter(loader))
    im = im.numpy().view(np.float16)
    for k, sid in enumerate(ix.reshape(-1).tolist()):
        rs = np.random.RandomState(contract_seed(5, 0, sid, 2))
        y, x = rs.randint(32 - 8 + 1), rs.randint(32 - 8 + 1)
        ref = np.full((32, 32, 3), sid % 255, np.uint8)
        ref[y:y + 8, x:x + 8] = (1, 2, 3)
        want = ((ref.astype(np.float64) - mean) / std).astype(np.float16)
        assert np.array_equal(im[k], want)


def test_cpu_device_rrc_raw_matches_oracle(tmp_path, oracle):
    """device='cpu' RRC on a raw .beton runs the reference's per-sample host
    loop (rgb_image.py:185-210) through the C ABI (ffcv_draw_batch_host +
    resize); with host Cutout / flip / NormalizeImage after it, bit-exact
    against the oracle under the seeding contract."""
    from tests.helpers import samples_of, expected_rrc
    fn = write(str(tmp_path / 'nat_raw.beton'), NaturalDS(40, hw=(90, 70), var=True, seed=3),
               {'image': RGBImageField(write_mode='raw'), 'label': IntField()})
    samples = samples_of(fn)
    mean, std = np.array([120., 110., 100.]), np.array([60., 55., 50.])
    lut = oracle.normalize_lut(mean, std)
    loader = Loader(fn, batch_size=8, seed=6, order=OrderOption.RANDOM, device='cpu', pipelines={
        'image': [RandomResizedCropRGBImageDecoder((48, 40)), Cutout(9, (1, 2, 3)), RandomHorizontalFlip(0.5),
                  NormalizeImage(mean, std, np.float16), ToTensor()]})
    for epoch in range(2):
        order = np.random.default_rng(6 + epoch).permutation(40)
        for b, (images, labels) in enumerate(loader):
            ids = order[b * 8:(b + 1) * 8]
            want = expected_rrc(oracle, samples, ids, 6, epoch, (48, 40), cutout=9, fill=(1, 2, 3),
                                flip_p=0.5, cut_before_flip=True, lut=lut)
            assert np.array_equal(images.numpy().view(np.uint16), want.view(np.uint16))
            assert (labels.numpy().reshape(-1) == ids % 10).all()


def test_host_draws_match_oracle(oracle):
    """ffcv_draw_batch_host (the device draw functions compiled for the host)
    equals the oracle's draws, crop / center crop / cutout."""
    from ffcv_amd import libffcv as L
    rng = np.random.default_rng(1)
    n = 3000
    ids = rng.integers(0, 2 ** 40, n).astype(np.uint64)
    hs = rng.integers(1, 700, n).astype(np.uint32)
    ws = rng.integers(1, 700, n).astype(np.uint32)
    for kind in (0, 1):
        p = L.DrawParams()
        p.crop_kind, p.out_h, p.out_w, p.cutout_size = kind, 224, 224, 32
        p.scale[0], p.scale[1] = 0.08, 1.0
        p.ratio[0], p.ratio[1] = 0.75, 4 / 3
        p.center_ratio = 224 / 256
        p.loader_seed, p.epoch = 12345, 7
        crops = np.zeros((n, 4), np.int32)
        cut = np.zeros((n, 2), np.int32)
        L.draw_batch_host(ids, hs, ws, p, crops, cut)
        oc, ocut = oracle.draw_batch(ids, hs, ws, 12345, 7, crop='random' if kind == 0 else 'center',
                                     cutout_size=32)
        assert np.array_equal(crops, oc) and np.array_equal(cut, ocut)


def test_cpu_device_loader_jpeg(tmp_path, oracle):
    """device='cpu' on a JPEG .beton, no GPU involved: the reference's host
    loop through the reference-signature C ABI -- imdecode on the CPU
    (ffcv_cpu_jpeg.hip), host draws and INTER_AREA resize -- host tensors
    out, bit-exact against the oracle (libjpeg-turbo decode + C restatement);
    and the default Simple pipeline on constant-size JPEGs."""
    from tests.helpers import samples_of, expected_rrc
    fn = str(tmp_path / 'cpu_jpg.beton')
    write(fn, NaturalDS(40, hw=(90, 110), var=True, seed=12),
          {'image': RGBImageField(write_mode='jpg'), 'label': IntField()})
    samples = samples_of(fn)
    loader = Loader(fn, batch_size=8, seed=5, order=OrderOption.RANDOM, device='cpu',
                    pipelines={'image': [RandomResizedCropRGBImageDecoder((56, 48)), Cutout(7, (9, 8, 7)),
                                         ToTensor()]})
    order = np.random.default_rng(5).permutation(40)
    for b, (images, labels) in enumerate(loader):
        assert images.device.type == 'cpu'
        ids = order[b * 8:(b + 1) * 8]
        want = expected_rrc(oracle, samples, ids, 5, 0, (56, 48), cutout=7, fill=(9, 8, 7), cut_before_flip=True)
        assert np.array_equal(images.numpy(), want)
    fn2 = str(tmp_path / 'cpu_jpg_const.beton')
    write(fn2, NaturalDS(12, hw=(40, 56), seed=13), {'image': RGBImageField(write_mode='jpg'), 'label': IntField()})
    s2 = samples_of(fn2)
    n = 0
    for images, labels in Loader(fn2, batch_size=4, device='cpu'):
        for k in range(4):
            i = int(np.nonzero([np.array_equal(oracle.ljt_decode(s[0]), images[k].numpy()) for s in s2])[0][0])
            assert int(labels[k]) == i % 10
            n += 1
    assert n == 12

