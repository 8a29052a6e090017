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
