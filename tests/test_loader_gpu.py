"""End-to-end Loader on the MI355X vs the oracle (bit-exact), through the
reference's own API: Loader + pipelines of Operations.

Ports the assertion intent of the reference suites (test_rrc.py,
test_image_pipeline.py, test_image_normalization.py, test_image_read.py)
and fixes the no-op ``is_true`` of test_rrc.py:65 into a real check; the
full-pixel parity tests compare every output against the CPU restatement
under the same (seed, epoch, sample index) contract.
"""
import os
import time
import tempfile

import numpy as np
import pytest
import torch as ch

from ffcv_amd.loader import Loader, OrderOption
from ffcv_amd.reader import Reader
from ffcv_amd.fields import RGBImageField, IntField
from ffcv_amd.fields.decoders import (RandomResizedCropRGBImageDecoder, CenterCropRGBImageDecoder,
                                      SimpleRGBImageDecoder, IntDecoder)
from ffcv_amd.transforms import (ToTensor, ToDevice, ToTorchImage, NormalizeImage, Cutout,
                                 RandomHorizontalFlip, Convert)
from ffcv_amd.loader.epoch_iterator import DecodeError
from tests.helpers import ConstDS, NaturalDS, write, samples_of as _samples, expected_rrc as _expected

pytestmark = pytest.mark.gpu
MEAN = np.array([0.485, 0.456, 0.406]) * 255
STD = np.array([0.229, 0.224, 0.225]) * 255


@pytest.fixture(scope='module', autouse=True)
def need_gpu(hip_lib):
    if not ch.cuda.is_available():
        pytest.skip('no HIP device')


@pytest.fixture(scope='module')
def tmpdir_m():
    return tempfile.mkdtemp()


@pytest.mark.parametrize('mode', ['raw', 'jpg'])
@pytest.mark.parametrize('decoder', ['rrc', 'cc'])
def test_crop_decoders_constant_images(tmpdir_m, mode, decoder):
    """test_rrc.py:52-110 (500 images 300-500 px, 160x160 output), with the
    jpg branch actually asserted (the reference's is a no-op)."""
    fn = os.path.join(tmpdir_m, f'const_{mode}.beton')
    if not os.path.exists(fn):
        write(fn, ConstDS(500, size_range=(300, 500)),
              {'index': IntField(), 'value': RGBImageField(write_mode=mode, jpeg_quality=95)})
    dec = RandomResizedCropRGBImageDecoder((160, 160)) if decoder == 'rrc' else \
        CenterCropRGBImageDecoder((160, 160), 224 / 256)
    loader = Loader(fn, batch_size=5, num_workers=2, pipelines={'value': [dec, ToTensor()]})
    n = 0
    for index, images in loader:
        assert images.device.type == 'cpu'  # no ToDevice -> host tensor, like the reference
        for i, image in zip(index, images):
            assert image.shape == (160, 160, 3)
            assert ch.all(image == (int(i) % 255)), int(i)
            n += 1
    assert n == 500


@pytest.mark.parametrize('mode', ['raw', 'jpg'])
def test_simple_pipeline_constant_images(tmpdir_m, mode):
    """test_image_pipeline.py: 500x300 constant images (jpg q95) decode exactly."""
    fn = os.path.join(tmpdir_m, f'simple_{mode}.beton')
    write(fn, ConstDS(60, hw=(500, 300)),
          {'index': IntField(), 'value': RGBImageField(write_mode=mode, jpeg_quality=95)})
    loader = Loader(fn, batch_size=5, pipelines={'value': [SimpleRGBImageDecoder(), ToTensor(),
                                                            ToDevice(ch.device('cuda:0'))]})
    for index, images in loader:
        assert images.device.type == 'cuda'
        for i, image in zip(index, images):
            assert ch.all(image == (int(i) % 255))


def test_simple_jpeg_natural_matches_oracle(tmpdir_m, oracle):
    fn = os.path.join(tmpdir_m, 'simple_nat.beton')
    write(fn, NaturalDS(40, hw=(77, 131)), {'image': RGBImageField(write_mode='jpg'), 'label': IntField()})
    samples = _samples(fn)
    loader = Loader(fn, batch_size=8, order=OrderOption.RANDOM, seed=3,
                    pipelines={'image': [SimpleRGBImageDecoder(), ToTensor(), ToDevice('cuda:0')],
                               'label': [IntDecoder(), ToTensor(), ToDevice('cuda:0')]})
    for images, labels in loader:
        assert labels.device.type == 'cuda'
        ids = None
        imgs = images.cpu().numpy()
        for k in range(imgs.shape[0]):
            matches = [i for i, s in enumerate(samples)
                       if np.array_equal(oracle.jpeg_decode(s[0]), imgs[k])]
            assert matches and int(labels[k]) == matches[0] % 10


@pytest.mark.parametrize('mode', ['raw', 'jpg'])
def test_c3_pipeline_matches_oracle(tmpdir_m, oracle, mode):
    """The north-star pipeline, fused into one launch, vs the oracle."""
    fn = os.path.join(tmpdir_m, f'nat_{mode}.beton')
    write(fn, NaturalDS(96, hw=(120, 160), var=True, seed=4),
          {'image': RGBImageField(write_mode=mode, jpeg_quality=90), 'label': IntField()})
    samples = _samples(fn)
    lut = oracle.normalize_lut(MEAN, STD)
    seed = 17
    loader = Loader(fn, batch_size=32, order=OrderOption.RANDOM, seed=seed, pipelines={
        'image': [RandomResizedCropRGBImageDecoder((64, 64)), Cutout(12, (124, 116, 103)), ToTensor(),
                  ToDevice(ch.device('cuda:0'), non_blocking=True), ToTorchImage(),
                  NormalizeImage(MEAN, STD, np.float16)],
        'label': [IntDecoder(), ToTensor(), ToDevice('cuda:0')]})
    for epoch in range(2):
        order = np.random.default_rng(seed + epoch).permutation(96)
        for b, (images, labels) in enumerate(loader):
            assert images.shape == (32, 3, 64, 64) and images.dtype == ch.float16
            assert images.is_contiguous(memory_format=ch.channels_last)
            ids = order[b * 32:(b + 1) * 32]
            want = _expected(oracle, samples, ids, seed, epoch, (64, 64), cutout=12,
                             fill=(124, 116, 103), lut=lut)
            got = images.permute(0, 2, 3, 1).cpu().numpy()
            assert np.array_equal(got.view(np.uint16), want.view(np.uint16))
            assert (labels.cpu().numpy().reshape(-1) == ids % 10).all()


def test_flip_cutout_center_and_staged_path(tmpdir_m, oracle):
    fn = os.path.join(tmpdir_m, 'nat_mix.beton')
    write(fn, NaturalDS(40, hw=(90, 70), var=True, seed=8),
          {'image': RGBImageField(write_mode='proportion', compress_probability=0.5), 'label': IntField()})
    samples = _samples(fn)
    assert {s[3] for s in samples} == {0, 1}
    for cache in (True, False):
        for cbf in (True, False):
            ops = [CenterCropRGBImageDecoder((48, 40), 0.8)]
            ops += [Cutout(9, (1, 2, 3)), RandomHorizontalFlip(0.5)] if cbf else \
                [RandomHorizontalFlip(0.5), Cutout(9, (1, 2, 3))]
            loader = Loader(fn, batch_size=8, seed=2, device_cache=cache,
                            pipelines={'image': ops + [ToTensor(), ToDevice('cuda:0')]})
            for b, (images, labels) in enumerate(loader):
                ids = np.arange(b * 8, (b + 1) * 8)
                want = _expected(oracle, samples, ids, 2, 0, (48, 40), crop='center', ratio=0.8,
                                 cutout=9, fill=(1, 2, 3), flip_p=0.5, cut_before_flip=cbf)
                assert np.array_equal(images.cpu().numpy(), want)


def test_unfused_device_transforms_and_user_op(tmpdir_m, oracle):
    """Operations the graph cannot fuse still run on the device (Cutout after
    a Simple decoder), and a user numpy Operation gets host arrays."""
    from dataclasses import replace
    from ffcv_amd.pipeline.operation import Operation
    from ffcv_amd.transforms.rng import contract_seed

    class AddOne(Operation):  # reference-style host op (jit_mode numpy)
        def generate_code(self):
            def f(images, dst):
                dst[:len(images)] = images + 1
                return dst[:len(images)]
            return f

        def declare_state_and_memory(self, previous_state):
            from ffcv_amd.pipeline.allocation_query import AllocationQuery
            return replace(previous_state, jit_mode=True), AllocationQuery(previous_state.shape,
                                                                           previous_state.dtype)
    fn = os.path.join(tmpdir_m, 'const_small.beton')
    write(fn, ConstDS(20, hw=(32, 32)), {'index': IntField(), 'value': RGBImageField()})
    loader = Loader(fn, batch_size=4, seed=9, pipelines={
        'value': [SimpleRGBImageDecoder(), Cutout(5, (200, 201, 202)), AddOne(), ToTensor()]})
    for index, images in loader:
        assert images.device.type == 'cpu'
        for k, sid in enumerate(index.reshape(-1).tolist()):
            rs = np.random.RandomState(contract_seed(9, 0, sid, 2))
            y, x = rs.randint(28), rs.randint(28)
            ref = np.full((32, 32, 3), sid % 255, np.uint8)
            ref[y:y + 5, x:x + 5] = (200, 201, 202)
            assert np.array_equal(images[k].numpy(), ref + 1)


def test_corrupt_jpeg_raises(tmpdir_m):
    fn = os.path.join(tmpdir_m, 'corrupt.beton')
    write(fn, NaturalDS(8, hw=(40, 40)), {'image': RGBImageField(write_mode='jpg'), 'label': IntField()})
    r = Reader(fn)
    p = int(r.metadata['f0'][3]['data_ptr'])
    with open(fn, 'r+b') as f:  # break sample 3's SOI marker
        f.seek(p)
        f.write(b'\x00\x00')
    loader = Loader(fn, batch_size=4, pipelines={'image': [RandomResizedCropRGBImageDecoder((32, 32))]})
    with pytest.raises(DecodeError, match='sample 3'):
        for _ in loader:
            pass


def test_distinct_epochs_and_determinism(tmpdir_m):
    fn = os.path.join(tmpdir_m, 'nat_det.beton')
    write(fn, NaturalDS(16, hw=(64, 64), seed=1), {'image': RGBImageField(write_mode='jpg'),
                                                   'label': IntField()})
    mk = lambda: Loader(fn, batch_size=16, seed=5, pipelines={
        'image': [RandomResizedCropRGBImageDecoder((32, 32)), ToTensor(), ToDevice('cuda:0')]})
    a, b = mk(), mk()
    e0a = next(iter(a))[0].cpu().clone()
    e1a = next(iter(a))[0].cpu().clone()
    e0b = next(iter(b))[0].cpu().clone()
    assert ch.equal(e0a, e0b) and not ch.equal(e0a, e1a)


@pytest.mark.parametrize('mode,n', [('raw', 200), ('jpg', 500)])
def test_process_cache_pcie_matches_device_cache(tmpdir_m, mode, n):
    """os_cache=False + device_cache=False (page scheduler, native gather out
    of the page slots, H2D per batch) gives the HBM-resident OS-cache result
    bit for bit, on a .beton spanning several 2 MiB pages."""
    from ffcv_amd.writer import DatasetWriter, MIN_PAGE_SIZE
    fn = os.path.join(tmpdir_m, f'paged_{mode}.beton')
    DatasetWriter(fn, {'image': RGBImageField(write_mode=mode, jpeg_quality=95), 'label': IntField()},
                  page_size=MIN_PAGE_SIZE, num_workers=1).from_indexed_dataset(
        NaturalDS(n, hw=(120, 160), var=True, seed=11), chunksize=25)
    mk = lambda **kw: Loader(fn, batch_size=64, order=OrderOption.RANDOM, seed=3, drop_last=False, pipelines={
        'image': [RandomResizedCropRGBImageDecoder((64, 64)), Cutout(12, (124, 116, 103)), ToTensor(),
                  ToDevice(ch.device('cuda:0'), non_blocking=True), ToTorchImage(),
                  NormalizeImage(MEAN, STD, np.float16)],
        'label': [IntDecoder(), ToTensor(), ToDevice('cuda:0')]}, **kw)  # noqa: E731
    a = mk(os_cache=True, device_cache=True)
    b = mk(os_cache=False, device_cache=False)
    assert len(b.memory_manager.page_to_samples) > 1
    for epoch in range(2):
        seen = 0
        for (ia, la), (ib, lb) in zip(a, b):
            assert ch.equal(la, lb)
            assert ch.equal(ia.view(ch.int16), ib.view(ch.int16))
            seen += len(lb)
        assert seen == n


@pytest.mark.parametrize('dtype', [np.float16, np.float32])
def test_gpu_normalization_standalone(tmpdir_m, dtype):
    """test_image_normalization.py:71-108 (test_gpu_normalization) ported:
    SimpleRGB -> ToTensor -> ToDevice -> ToTorchImage -> NormalizeImage ->
    View runs the standalone device LUT kernel (ffcv_lut_batch).  Checked
    exactly against the reference's LUT arithmetic (normalize.py:42-49) and
    with the reference's own np.allclose assertion; fp16 and fp32 tables."""
    from ffcv_amd.transforms import View
    fn = os.path.join(tmpdir_m, 'norm_raw.beton')
    if not os.path.exists(fn):
        write(fn, ConstDS(500, hw=(25, 30)), {'index': IntField(), 'value': RGBImageField(write_mode='raw')})
    mean, std = np.array([0, 1, 2]), np.array([1, 10, 20])
    tdt = ch.float16 if dtype == np.float16 else ch.float32
    loader = Loader(fn, batch_size=5, num_workers=2, pipelines={'value': [
        SimpleRGBImageDecoder(), ToTensor(), ToDevice(ch.device('cuda:0')), ToTorchImage(),
        NormalizeImage(mean, std, dtype), View(tdt)]})
    table = ((np.arange(256)[:, None] - mean[None, :]) / std[None, :]).astype(dtype)
    seen = 0
    for index, images in loader:
        assert images.dtype == tdt and images.shape[1:] == (3, 25, 30)
        got = images.cpu().numpy()
        for k, i in enumerate(index.reshape(-1).tolist()):
            v = i % 255
            want = np.broadcast_to(table[v][:, None, None], (3, 25, 30))
            assert np.array_equal(np.ascontiguousarray(got[k]).view(np.uint8), np.ascontiguousarray(want).view(np.uint8))
            ref = np.full((3, 25, 30), v, dtype)
            ref -= mean[:, None, None]
            ref /= std[:, None, None]
            assert np.allclose(ref, got[k])
            seen += 1
    assert seen == 500


def test_flip_unfused_device(tmpdir_m):
    """RandomHorizontalFlip after a Simple decoder runs the standalone device
    flip kernel (ffcv_flip_batch) with the contract's per-sample decisions."""
    from ffcv_amd.transforms.rng import contract_seed
    fn = os.path.join(tmpdir_m, 'flip_raw.beton')
    ds = NaturalDS(30, hw=(20, 26), seed=5)
    write(fn, ds, {'image': RGBImageField(write_mode='raw'), 'label': IntField()})
    loader = Loader(fn, batch_size=8, seed=4, drop_last=False, pipelines={
        'image': [SimpleRGBImageDecoder(), RandomHorizontalFlip(0.5), ToTensor(), ToDevice('cuda:0')]})
    flipped = 0
    for b, (images, labels) in enumerate(loader):
        got = images.cpu().numpy()
        for k in range(got.shape[0]):
            sid = b * 8 + k
            u = np.random.RandomState(contract_seed(4, 0, sid, 3)).uniform(0, 1)
            want = ds.imgs[sid][:, ::-1] if u < 0.5 else ds.imgs[sid]
            flipped += u < 0.5
            assert np.array_equal(got[k], want), sid
    assert 0 < flipped < 30


def _c3_loader(fn, seed, out=(64, 64), **kw):
    return Loader(fn, batch_size=16, order=OrderOption.RANDOM, seed=seed, pipelines={
        'image': [RandomResizedCropRGBImageDecoder(out), Cutout(12, (124, 116, 103)), ToTensor(),
                  ToDevice(ch.device('cuda:0'), non_blocking=True), ToTorchImage(),
                  NormalizeImage(MEAN, STD, np.float16)],
        'label': [IntDecoder(), ToTensor(), ToDevice('cuda:0')]}, **kw)


def test_launch_groups_match_single_batches(tmpdir_m):
    """Several batches per decode launch (the default) hand out exactly the
    batches one launch per batch gives, including a partial last batch."""
    fn = os.path.join(tmpdir_m, 'grp.beton')
    write(fn, NaturalDS(100, hw=(80, 96), var=True, seed=6),
          {'image': RGBImageField(write_mode='jpg'), 'label': IntField()})
    a = _c3_loader(fn, 7, drop_last=False, batches_per_launch=1)
    b = _c3_loader(fn, 7, drop_last=False)
    c = _c3_loader(fn, 7, drop_last=False, batches_per_launch=3)
    for epoch in range(2):
        n = 0
        for (ia, la), (ib, lb), (ic, lc) in zip(a, b, c):
            assert ch.equal(la, lb) and ch.equal(la, lc)
            assert ch.equal(ia.view(ch.int16), ib.view(ch.int16))
            assert ch.equal(ia.view(ch.int16), ic.view(ch.int16))
            n += len(la)
        assert n == 100


@pytest.mark.parametrize('recompile', [False, True])
def test_output_size_change_between_epochs(tmpdir_m, oracle, recompile):
    """Progressive resizing: a new decoder output_size between epochs takes
    effect (new buffers, new kernel target), with or without recompile
    (making_dataloaders.rst: a resolution change needs no recompile)."""
    fn = os.path.join(tmpdir_m, 'resz.beton')
    if not os.path.exists(fn):
        write(fn, NaturalDS(48, hw=(90, 110), var=True, seed=9),
              {'image': RGBImageField(write_mode='jpg'), 'label': IntField()})
    samples = _samples(fn)
    lut = oracle.normalize_lut(MEAN, STD)
    loader = _c3_loader(fn, 3, recompile=recompile)
    dec = loader.pipeline_specs['image'].decoder
    for epoch, size in enumerate([(64, 64), (48, 40), (72, 80)]):
        dec.output_size = size
        order = np.random.default_rng(3 + epoch).permutation(48)
        for b, (images, labels) in enumerate(loader):
            assert images.shape == (16, 3) + size
            ids = order[b * 16:(b + 1) * 16]
            want = _expected(oracle, samples, ids, 3, epoch, size, cutout=12, fill=(124, 116, 103), lut=lut)
            got = images.permute(0, 2, 3, 1).cpu().numpy()
            assert np.array_equal(got.view(np.uint16), want.view(np.uint16))


def test_early_break_then_next_epoch(tmpdir_m, oracle):
    """An iterator abandoned after one batch is stopped before the next
    epoch re-uses the buffer sets; the next epoch is exact."""
    fn = os.path.join(tmpdir_m, 'brk.beton')
    write(fn, NaturalDS(160, hw=(64, 80), var=True, seed=2),
          {'image': RGBImageField(write_mode='jpg'), 'label': IntField()})
    samples = _samples(fn)
    lut = oracle.normalize_lut(MEAN, STD)
    loader = _c3_loader(fn, 11, batches_per_launch=2)
    for _ in loader:
        break
    for epoch in (1, 2):
        order = np.random.default_rng(11 + epoch).permutation(160)
        n = 0
        for b, (images, labels) in enumerate(loader):
            ids = order[b * 16:(b + 1) * 16]
            want = _expected(oracle, samples, ids, 11, epoch, (64, 64), cutout=12, fill=(124, 116, 103), lut=lut)
            assert np.array_equal(images.permute(0, 2, 3, 1).cpu().numpy().view(np.uint16), want.view(np.uint16))
            assert (labels.cpu().numpy().reshape(-1) == ids % 10).all()
            n += 1
            if epoch == 1 and b == 4:
                break  # abandon again mid-epoch
        assert n == (5 if epoch == 1 else 10)


def test_entropy_index_epochs_match(tmpdir_m, oracle):
    """The entropy index (default on with device_cache) changes no output:
    three epochs with it equal three epochs without it, every sample's record
    is published after the first epoch, and large images use all 64 lane
    ranges; the last epoch is also checked against the oracle."""
    fn = os.path.join(tmpdir_m, 'eidx.beton')
    write(fn, NaturalDS(48, hw=(300, 380), var=True, seed=21),
          {'image': RGBImageField(write_mode='jpg', jpeg_quality=90), 'label': IntField()})
    samples = _samples(fn)
    lut = oracle.normalize_lut(MEAN, STD)
    a = _c3_loader(fn, 21, entropy_index=False)
    b = _c3_loader(fn, 21)
    assert a.device_dataset.entropy_index(0) is None
    for epoch in range(3):
        order = np.random.default_rng(21 + epoch).permutation(48)
        for bi, ((ia, la), (ib, lb)) in enumerate(zip(a, b)):
            assert ch.equal(la, lb)
            assert ch.equal(ia.view(ch.int16), ib.view(ch.int16))
            if epoch == 2:
                ids = order[bi * 16:(bi + 1) * 16]
                want = _expected(oracle, samples, ids, 21, epoch, (64, 64), cutout=12,
                                 fill=(124, 116, 103), lut=lut)
                assert np.array_equal(ib.permute(0, 2, 3, 1).cpu().numpy().view(np.uint16),
                                      want.view(np.uint16))
        if epoch == 0:
            head = b.device_dataset.entropy_index(0)[:, 0, 1].cpu().numpy().astype(np.uint32)
            assert (head & 0x80000000).all()
            nthr = (head >> 16) & 0xff
            assert nthr.max() == 64 and nthr.min() >= 1


def _dist_c3_worker(rank, world, port, fn, out, seed):
    """One rank of a world-size-2 job on the one GPU: the device-cache C3
    Loader with distributed=True (perm[rank::world], random.py:13-27)."""
    import torch.distributed as dist
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    loader = Loader(fn, batch_size=16, order=OrderOption.RANDOM, seed=seed, distributed=True, drop_last=False,
                    pipelines={'image': [RandomResizedCropRGBImageDecoder((224, 224)), Cutout(32, (124, 116, 103)),
                                         ToTensor(), ToDevice(ch.device('cuda:0'), non_blocking=True),
                                         ToTorchImage(), NormalizeImage(MEAN, STD, np.float16)],
                               'label': [IntDecoder(), ToTensor(), ToDevice('cuda:0')]})
    res = {}
    for epoch in range(2):
        imgs, ids = [], []
        for images, labels in loader:
            imgs.append(images.permute(0, 2, 3, 1).cpu().numpy().view(np.uint16))
            ids.append(labels.cpu().numpy().reshape(-1))
        res[f'img{epoch}'] = np.concatenate(imgs)
        res[f'ids{epoch}'] = np.concatenate(ids)
    np.savez(os.path.join(out, f'r{rank}.npz'), **res)
    dist.barrier()
    dist.destroy_process_group()


class _IdDS:
    def __init__(self, n, seed=12):
        from ffcv_amd.synthetic import natural_image, imagenet_like_shape
        rng = np.random.default_rng(seed)
        self.imgs = [natural_image(rng, *imagenet_like_shape(rng, 256)) for _ in range(n)]

    def __len__(self):
        return len(self.imgs)

    def __getitem__(self, i):
        return self.imgs[i], i


def test_distributed_device_loader_world2(tmpdir_m, oracle):
    """VERDICT r2 "next" 6: two processes on the one GPU (gloo process group),
    each a device-cache Loader(distributed=True) running the C3 pipeline on a
    JPEG .beton.  Each rank's batches equal the oracle bit for bit for its
    DistributedSampler slice (order included), and the two slices cover the
    epoch (padded like the sampler)."""
    import torch.multiprocessing as mp
    from torch.utils.data import DistributedSampler
    n, seed = 150, 21
    fn = os.path.join(tmpdir_m, 'dist_c3.beton')
    write(fn, _IdDS(n), {'image': RGBImageField(write_mode='jpg', jpeg_quality=90), 'label': IntField()})
    samples = _samples(fn)
    lut = oracle.normalize_lut(MEAN, STD)
    with tempfile.TemporaryDirectory() as d:
        port = 29300 + os.getpid() % 500
        mp.spawn(_dist_c3_worker, args=(2, port, fn, d, seed), nprocs=2, join=True)
        z = [np.load(os.path.join(d, f'r{r}.npz')) for r in range(2)]
    for epoch in range(2):
        both = []
        for r in range(2):
            smp = DistributedSampler(np.arange(n), num_replicas=2, rank=r, shuffle=True, seed=seed, drop_last=False)
            smp.set_epoch(epoch)
            want_ids = np.array(list(smp))
            ids = z[r][f'ids{epoch}']
            assert np.array_equal(ids, want_ids), (r, epoch)
            want = _expected(oracle, samples, ids, seed, epoch, (224, 224), cutout=32, fill=(124, 116, 103), lut=lut)
            assert np.array_equal(z[r][f'img{epoch}'], want.view(np.uint16)), (r, epoch)
            both.append(ids)
        both = np.concatenate(both)
        assert set(both.tolist()) == set(range(n)) and len(both) == 2 * ((n + 1) // 2)


def test_kept_batches_survive_set_boundaries(tmpdir_m):
    """A batch the training loop keeps stays intact while it takes
    batches_ahead more (the previous batch of a launch group was
    overwritten one batch later, at every set boundary)."""
    fn = os.path.join(tmpdir_m, 'keep.beton')
    write(fn, NaturalDS(120, hw=(60, 80), var=True, seed=5),
          {'image': RGBImageField(write_mode='jpg', jpeg_quality=90), 'label': IntField()})
    ahead = 2
    loader = Loader(fn, batch_size=8, order=OrderOption.RANDOM, seed=1, batches_ahead=ahead, batches_per_launch=3,
                    pipelines={'image': [RandomResizedCropRGBImageDecoder((48, 48)), ToTensor(),
                                         ToDevice(ch.device('cuda:0'))],
                               'label': [IntDecoder(), ToTensor(), ToDevice('cuda:0')]})
    for _ in range(2):
        kept = []
        for images, labels in loader:
            kept.append((images, images.clone(), labels, labels.clone()))
            kept = kept[-(ahead + 1):]
            ch.cuda.synchronize()
            time.sleep(0.002)  # let the producer run ahead as far as it may
            ch.cuda.synchronize()
            for k, (a, ac, b, bc) in enumerate(kept):
                assert ch.equal(a, ac) and ch.equal(b, bc), f'batch {k - len(kept) + 1} overwritten'


def test_bench_rccl_world1():
    """the N > 1 bench path's RCCL branch
    (init_process_group('nccl', device_id=...), barrier, max-over-ranks
    all-reduce of the timed region, per-rank all-gather) run once here, as a
    torchrun job of world size 1, so it is not first executed on the 8-GPU
    scaling node.  The line must carry process_group.backend == 'nccl' and a
    green parity check."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    port = 29800 + os.getpid() % 100
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node', '1',
           '--master-addr', '127.0.0.1', '--master-port', str(port), os.path.join(root, 'bench.py'),
           '--gpus', '1', '--steps', '6', '--warmup', '2', '--unique', '512', '--dataset-size', '40000',
           '--no-cpu-baseline', '--no-later-epochs', '--no-c5', '--parity-rows', '256']
    # the environment as the driver's run gets it (the box exports
    # HSA_ENABLE_IPC_MODE_LEGACY=0 itself; bench.py's self-launch keeps it)
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=110, cwd=root)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith('{')][-1])
    pg = line['process_group']
    assert pg['backend'] == 'nccl' and pg['world_size'] == 1, pg
    assert line['n_gpus'] == 1 and line['value'] > 0
    assert line['parity']['checked'] > 0 and line['parity']['mismatch'] == 0


def test_bench_gpus2_self_launch():
    """`bench.py --gpus 2` with no torchrun around it
    starts torchrun itself (a child process) with two ranks, each re-entering
    bench.py with RANK / WORLD_SIZE set; on this one-GPU box both ranks share
    cuda:0 over a gloo group (RCCL refuses two ranks on one device).  The line
    must report n_gpus 2, a world-2 process group with both ranks' timings,
    and green parity on every rank."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, os.path.join(root, 'bench.py'), '--gpus', '2', '--steps', '6', '--warmup', '2',
           '--unique', '512', '--dataset-size', '40000', '--no-cpu-baseline', '--no-later-epochs', '--no-c5',
           '--parity-rows', '256']
    env = dict(os.environ, FFCV_BENCH_BACKEND='gloo')
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=110, env=env, cwd=root)
    assert r.returncode == 0, r.stderr[-2000:]
    assert 'torch.distributed.run' in r.stderr
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith('{')][-1])
    pg = line['process_group']
    assert pg['backend'] == 'gloo' and pg['world_size'] == 2, pg
    assert [p['rank'] for p in pg['per_rank']] == [0, 1]
    assert line['n_gpus'] == 2 and line['config']['global_batch'] == 2 * 512
    assert abs(line['value'] - 2 * 512 * 6 / max(p['seconds'] for p in pg['per_rank'])) < 0.01 * line['value']
    par = line['parity']
    assert par['checked_all_ranks'] > par['checked'] > 0 and par['mismatch_all_ranks'] == 0
