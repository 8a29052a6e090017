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


def test_decode_path_requires_gpu(tmp_path):
    fn = write(str(tmp_path / 'j.beton'), NaturalDS(8), {'image': RGBImageField(write_mode='jpg'),
                                                          'label': IntField()})
    with pytest.raises(RuntimeError, match='HIP device'):
        Loader(fn, batch_size=4, device='cpu')
    with pytest.raises(RuntimeError, match='HIP device'):
        Loader(fn, batch_size=4, device='cpu',
               pipelines={'image': [RandomResizedCropRGBImageDecoder((32, 32))]})
