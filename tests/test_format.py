""".beton format compatibility with the reference (CPU).

tests/golden/betons.npz holds files written by the REFERENCE's own
DatasetWriter (num_workers=1) under the stub harness.  Our Reader must parse
them and our DatasetWriter must reproduce them byte for byte.
"""
import os
import tempfile

import numpy as np
import pytest

from ffcv_amd.reader import Reader
from ffcv_amd.writer import DatasetWriter
from ffcv_amd.fields import RGBImageField, IntField, BytesField

GOLD = os.path.join(os.path.dirname(__file__), 'golden')


class RawDS:
    """Same generator as tests/golden/make_golden.py (_RawDS)."""

    def __init__(self, n, shapes, seed):
        self.n, self.shapes, self.seed = n, shapes, seed

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        r = np.random.default_rng(self.seed + i)
        h, w = self.shapes[i % len(self.shapes)]
        y = np.linspace(0, 1, h)[:, None, None]
        x = np.linspace(0, 1, w)[None, :, None]
        img = np.clip(128 + 100 * np.sin(7 * x + 5 * y + np.array([0, 1, 2])) +
                      r.normal(0, 20, (h, w, 3)), 0, 255).astype(np.uint8)
        return img, i * 7 - 3


def _spec(g, name):
    a = g['spec_' + name]
    n, seed = int(a[0]), int(a[1])
    shapes = [tuple(int(v) for v in a[2 + 2 * k:4 + 2 * k]) for k in range((len(a) - 2) // 2)]
    return n, seed, shapes


@pytest.mark.parametrize('name', ['raw32', 'rawvar', 'jpgvar', 'smart_maxres'])
def test_reader_parses_reference_files(name):
    g = np.load(os.path.join(GOLD, 'betons.npz'))
    with tempfile.NamedTemporaryFile(suffix='.beton') as f:
        f.write(g['beton_' + name].tobytes())
        f.flush()
        r = Reader(f.name)
        n, seed, shapes = _spec(g, name)
        assert r.num_samples == n and r.field_names == ['image', 'label']
        assert r.metadata.dtype.itemsize == 24
        assert (r.metadata['f1'] == np.arange(n) * 7 - 3).all()
        assert len(r.alloc_table) == n
        ds = RawDS(n, shapes, seed)
        mm = np.memmap(f.name, np.uint8, mode='r')
        ptrs = dict(zip(r.alloc_table['ptr'], r.alloc_table['size']))
        for i in range(n):
            md = r.metadata['f0'][i]
            img = ds[i][0]
            if name == 'smart_maxres':
                continue
            assert (md['height'], md['width']) == img.shape[:2]
            if md['mode'] == 1:
                size = ptrs[md['data_ptr']]
                assert np.array_equal(mm[md['data_ptr']:md['data_ptr'] + size], img.reshape(-1))


@pytest.mark.parametrize('name', ['raw32', 'rawvar', 'jpgvar', 'smart_maxres'])
def test_writer_reproduces_reference_bytes(name, hip_lib):
    """DatasetWriter output == the reference writer's file, byte for byte;
    smart_maxres runs the max_resolution INTER_AREA shrink (rgb_image.py:37-45)
    through the host C-ABI resize and the smart raw/jpg choice."""
    g = np.load(os.path.join(GOLD, 'betons.npz'))
    n, seed, shapes = _spec(g, name)
    kw = {'raw32': dict(write_mode='raw'), 'rawvar': dict(write_mode='raw'),
          'jpgvar': dict(write_mode='jpg', jpeg_quality=90),
          'smart_maxres': dict(write_mode='smart', max_resolution=48, smart_threshold=3000)}[name]
    with tempfile.TemporaryDirectory() as d:
        fn = os.path.join(d, 'x.beton')
        DatasetWriter(fn, {'image': RGBImageField(**kw), 'label': IntField()},
                      num_workers=1).from_indexed_dataset(RawDS(n, shapes, seed), chunksize=5)
        ours = np.fromfile(fn, np.uint8)
    assert np.array_equal(ours, g['beton_' + name])


def test_parallel_writer_same_bytes_as_serial():
    ds = RawDS(30, [(20, 30), (31, 17)], 5)
    with tempfile.TemporaryDirectory() as d:
        outs = []
        for nw in (1, 3):
            fn = os.path.join(d, f'{nw}.beton')
            DatasetWriter(fn, {'image': RGBImageField(write_mode='jpg'), 'label': IntField()},
                          num_workers=nw).from_indexed_dataset(ds)
            outs.append(np.fromfile(fn, np.uint8))
        assert np.array_equal(outs[0], outs[1])


def test_page_straddle_and_bytes_field():
    class DS:
        def __len__(self):
            return 9

        def __getitem__(self, i):
            return (i, np.full(900_000 + i, i % 251, np.uint8))
    with tempfile.TemporaryDirectory() as d:
        fn = os.path.join(d, 'b.beton')
        DatasetWriter(fn, {'index': IntField(), 'value': BytesField()}, page_size=1 << 21,
                      num_workers=1).from_indexed_dataset(DS())
        r = Reader(fn)
        mm = np.memmap(fn, np.uint8, mode='r')
        page = r.page_size
        for i in range(9):
            md = r.metadata['f1'][i]
            assert md['size'] == 900_000 + i
            assert md['ptr'] // page == (md['ptr'] + md['size'] - 1) // page  # no straddle
            assert (mm[md['ptr']:md['ptr'] + md['size']] == i % 251).all()
