import numpy as np

from ffcv_amd.writer import DatasetWriter
from ffcv_amd.fields import RGBImageField, IntField, BytesField


class ConstDS:
    """Reference test datasets (test_rrc.py:20-34, test_image_pipeline.py):
    constant images of value index % 255, random or fixed size."""

    def __init__(self, length, size_range=None, hw=None, seed=0):
        self.length, self.size_range, self.hw = length, size_range, hw
        self.rng = np.random.default_rng(seed)
        self.dims = [(int(self.rng.integers(size_range[0], size_range[1] + 1)),
                      int(self.rng.integers(size_range[0], size_range[1] + 1)))
                     if size_range else hw for _ in range(length)]

    def __len__(self):
        return self.length

    def __getitem__(self, index):
        h, w = self.dims[index]
        return index, ((np.ones((h, w, 3)) * index) % 255).astype('uint8')


class NaturalDS:
    def __init__(self, length, hw=(64, 48), seed=0, var=False):
        from ffcv_amd.synthetic import natural_image
        rng = np.random.default_rng(seed)
        self.imgs = []
        for i in range(length):
            h, w = (int(rng.integers(hw[0] // 2, hw[0] + 1)), int(rng.integers(hw[1] // 2, hw[1] + 1))) \
                if var else hw
            self.imgs.append(natural_image(rng, h, w))

    def __len__(self):
        return len(self.imgs)

    def __getitem__(self, i):
        return self.imgs[i], i % 10


def write(path, ds, fields, workers=1):
    DatasetWriter(path, fields, num_workers=workers).from_indexed_dataset(ds, chunksize=5)
    return path


def samples_of(fn):
    """(bytes, height, width, mode) of every sample of field f0."""
    from ffcv_amd.reader import Reader
    r = Reader(fn)
    mm = np.memmap(fn, np.uint8, mode='r')
    sizes = dict(zip(r.alloc_table['ptr'].tolist(), r.alloc_table['size'].tolist()))
    out = []
    for md in r.metadata['f0']:
        p = int(md['data_ptr'])
        out.append((np.array(mm[p:p + sizes[p]]), int(md['height']), int(md['width']), int(md['mode'])))
    return out


def expected_rrc(oracle, samples, ids, seed, epoch, out_hw, crop='random', ratio=224 / 256,
              cutout=0, fill=(0, 0, 0), flip_p=0.0, cut_before_flip=False, lut=None):
    ids = np.asarray(ids, np.uint64)
    hs = [samples[int(i)][1] for i in ids]
    ws = [samples[int(i)][2] for i in ids]
    crops, cyx = oracle.draw_batch(ids, hs, ws, seed, epoch, crop=crop, center_ratio=ratio,
                                   out_h=out_hw[0], out_w=out_hw[1], cutout_size=cutout)
    u8 = oracle.rrc_batch([samples[int(i)] for i in ids], crops, out_hw[0], out_hw[1])
    for k, sid in enumerate(ids):
        if cutout and cut_before_flip:
            y, x = cyx[k]
            u8[k, y:y + cutout, x:x + cutout] = fill
        if flip_p and oracle.MT(oracle.sample_seed(seed, epoch, int(sid), 3)).uniform(0, 1) < flip_p:
            u8[k] = u8[k, :, ::-1]
        if cutout and not cut_before_flip:
            y, x = cyx[k]
            u8[k, y:y + cutout, x:x + cutout] = fill
    if lut is not None:
        idx = u8.astype(np.int64)
        return np.stack([lut[idx[..., c], c] for c in range(3)], -1)
    return u8
