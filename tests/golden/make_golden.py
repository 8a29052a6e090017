"""Generate golden vectors by running the REFERENCE's own Python (this
container only; /root/reference does not exist on the GPU box).

The reference package cannot import as-is here (numba / cv2 / its compiled
ffcv._libffcv are absent: an ordinary ModuleNotFoundError, not a permission
denial).  Following SURVEY.md Appendix E we insert stub modules:
  * numba     njit -> identity, prange -> range, typed.Dict -> dict, ...
              (so numba's np.random calls become numpy's legacy RandomState,
              whose MT19937/uniform/randint algorithms numba re-implements)
  * cv2       imencode via Pillow (RGB), cvtColor channel swap, INTER_AREA
              resize via the oracle restatement (only for max_resolution)
  * ffcv._libffcv  ctypes.CDLL shim whose resize/imdecode/my_memcpy are the
              oracle (memcpy = ctypes.memmove)
then import /root/reference/ffcv and call its functions.  Nothing from the
reference is copied into this repository; only the OUTPUTS are saved, as
tests/golden/*.npz.

Run:  python tests/golden/make_golden.py
"""
import ctypes
import importlib.abc
import importlib.machinery
import io
import os
import sys
import tempfile
import types

import numpy as np

REF = '/root/reference'
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from oracle import oracle as O  # noqa: E402


# ----------------------------------------------------------------- stubs ----
def _identity_decorator(*args, **kwargs):
    if len(args) == 1 and callable(args[0]) and not kwargs:
        return args[0]
    return lambda f: f


class _Permissive(types.SimpleNamespace):
    def __getattr__(self, name):
        return _Permissive()

    def __getitem__(self, item):
        return _Permissive()

    def __call__(self, *a, **k):
        return _Permissive()


def install_stubs():
    numba = types.ModuleType('numba')
    numba.njit = _identity_decorator
    numba.jit = _identity_decorator
    numba.prange = range
    numba.set_num_threads = lambda n: None
    numba.get_num_threads = lambda: 1
    numba.objmode = _Permissive()
    numba.warnings = types.SimpleNamespace(simplefilter=lambda *a, **k: None)
    numba.types = _Permissive()
    for t in ['uint8', 'uint16', 'uint32', 'uint64', 'int64', 'int32', 'float64']:
        setattr(numba, t, _Permissive())
    typed = types.ModuleType('numba.typed')
    typed.Dict = dict
    typed.List = list
    extending = types.ModuleType('numba.extending')
    extending.intrinsic = lambda f: f
    core = types.ModuleType('numba.core')
    errors = types.ModuleType('numba.core.errors')

    class NumbaPerformanceWarning(Warning):
        pass
    errors.NumbaPerformanceWarning = NumbaPerformanceWarning
    core.errors = errors
    numba.typed, numba.extending, numba.core = typed, extending, core
    sys.modules.update({'numba': numba, 'numba.typed': typed,
                        'numba.extending': extending, 'numba.core': core,
                        'numba.core.errors': errors})

    cv2 = types.ModuleType('cv2')
    cv2.COLOR_RGB2BGR = 4
    cv2.COLOR_BGR2RGB = 4
    cv2.IMREAD_COLOR = 1
    cv2.IMWRITE_JPEG_QUALITY = 1
    cv2.INTER_AREA = 3

    def cvtColor(img, code):
        return np.ascontiguousarray(img[..., ::-1])

    def imencode(ext, bgr, params):
        from PIL import Image
        q = int(params[1]) if params else 95
        b = io.BytesIO()
        Image.fromarray(np.ascontiguousarray(bgr[..., ::-1])).save(b, format='JPEG', quality=q)
        return True, np.frombuffer(b.getvalue(), np.uint8).copy()

    def resize(img, size, interpolation=None):
        w, h = int(size[0]), int(size[1])
        return O.resize_crop(img, 0, img.shape[0], 0, img.shape[1], h, w)
    cv2.cvtColor, cv2.imencode, cv2.resize = cvtColor, imencode, resize
    sys.modules['cv2'] = cv2

    class _FakeLib:
        def __init__(self):
            self.my_memcpy = self._wrap(lambda src, dst, n: ctypes.memmove(dst, src, n))
            self.resize = self._wrap(self._resize)
            self.imdecode = self._wrap(self._imdecode)
            self.resize_calls = []

        @staticmethod
        def _wrap(f):
            class F:
                argtypes = None
                restype = None

                def __call__(self, *a):
                    return f(*a)
            return F()

        def _resize(self, cres, src, sx, sy, r0, r1, c0, c1, dst, tx, ty):
            self.resize_calls.append((r0, r1, c0, c1))
            O.lib().orc_resize_crop(ctypes.c_void_p(src), sx, sy, r0, r1, c0, c1,
                                    ctypes.c_void_p(dst), tx, ty)

        def _imdecode(self, src, size, sh, sw, dst, ch, cw, ox, oy, sn, sd, crop, flip):
            data = np.ctypeslib.as_array((ctypes.c_uint8 * size).from_address(src))
            img = O.jpeg_decode(data.copy(), 'ifast')
            ctypes.memmove(dst, img.ctypes.data, img.nbytes)
            return 0

    fake = _FakeLib()
    real_cdll = ctypes.CDLL

    def cdll(name, *a, **k):
        if name == '/nonexistent':
            return fake
        return real_cdll(name, *a, **k)
    ctypes.CDLL = cdll

    class Finder(importlib.abc.MetaPathFinder, importlib.abc.Loader):
        def find_spec(self, fullname, path, target=None):
            if fullname == 'ffcv._libffcv':
                return importlib.machinery.ModuleSpec(fullname, self)
            return None

        def create_module(self, spec):
            m = types.ModuleType(spec.name)
            m.__file__ = '/nonexistent'
            return m

        def exec_module(self, module):
            pass
    sys.meta_path.insert(0, Finder())
    return fake


# --------------------------------------------------------------- goldens ----
def gen_crops(rgb):
    rng = np.random.default_rng(20261015)
    rows = []
    shapes = [(256, 256), (256, 192), (192, 256), (512, 512), (500, 333), (300, 500),
              (32, 32), (1, 1), (2, 7), (17, 400), (1000, 10), (10, 1000), (224, 224)]
    params = [((0.08, 1.0), (0.75, 4 / 3)), ((0.35, 1.0), (0.75, 4 / 3)),
              ((0.08, 0.5), (0.5, 2.0))]
    for k in range(24000):
        if k < len(shapes) * 40:
            H, W = shapes[k % len(shapes)]
        else:
            H, W = int(rng.integers(1, 1200)), int(rng.integers(1, 1200))
        sc, ra = params[k % len(params)] if k % 7 == 0 else params[0]
        seed = int(rng.integers(0, 2 ** 32))
        np.random.seed(seed)
        i, j, h, w = rgb.get_random_crop(np.uint32(H), np.uint32(W), np.array(sc), np.array(ra))
        rows.append((seed, H, W, sc[0], sc[1], ra[0], ra[1], i, j, h, w))
    arr = np.array(rows, dtype=np.float64)
    centers = []
    for k in range(2000):
        H, W = int(rng.integers(1, 1200)), int(rng.integers(1, 1200))
        ratio = [224 / 256, 0.875, 1.0, 0.5][k % 4]
        i, j, h, w = rgb.get_center_crop(H, W, None, ratio)
        centers.append((H, W, ratio, i, j, h, w))
    return arr, np.array(centers, np.float64)


def gen_cutout(Cutout):
    rng = np.random.default_rng(7)
    rows = []
    for k in range(4000):
        H = int(rng.integers(8, 500))
        W = int(rng.integers(8, 500))
        c = int(rng.integers(1, min(H, W) + 1))
        seed = int(rng.integers(0, 2 ** 32))
        op = Cutout(c, (1, 2, 3))
        fn = op.generate_code()
        img = np.zeros((1, H, W, 3), np.uint8)
        np.random.seed(seed)
        fn(img)
        ys, xs = np.nonzero(img[0, :, :, 0])
        rows.append((seed, H, W, c, ys.min(), xs.min()))
    return np.array(rows, np.int64)


def gen_lut(NormalizeImage):
    out = {}
    for name, mean, std in [('imagenet', np.array([0.485, 0.456, 0.406]) * 255,
                             np.array([0.229, 0.224, 0.225]) * 255),
                            ('test', np.array([0, 1, 2]), np.array([1, 10, 20]))]:
        op = NormalizeImage(mean, std, np.float16)
        out[f'lut_{name}'] = np.asarray(op.lookup_table).view(np.int16).copy()
        out[f'mean_{name}'] = mean
        out[f'std_{name}'] = std
    return out


def gen_orders(Random, Sequential):
    import torch.utils.data.distributed as tdd
    res = {}

    class FakeLoader:
        pass
    for N in [600, 1001]:
        for seed in [0, 1234]:
            for world in [1, 2, 4, 8]:
                for rank in range(world):
                    fl = FakeLoader()
                    fl.indices = np.arange(N, dtype='uint64')
                    fl.seed = seed
                    fl.distributed = world > 1
                    tdd.dist.get_world_size = lambda *a, w=world: w
                    tdd.dist.get_rank = lambda *a, r=rank: r
                    tdd.dist.is_available = lambda: True
                    for kind, Cls in [('random', Random), ('sequential', Sequential)]:
                        o = Cls(fl)
                        for epoch in [0, 1, 5]:
                            res[f'{kind}_N{N}_s{seed}_w{world}_r{rank}_e{epoch}'] = \
                                np.asarray(o.sample_order(epoch)).astype(np.int64)
    return res


class _RawDS:
    def __init__(self, n, shapes, seed):
        self.n = n
        self.shapes = shapes
        self.seed = seed

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


def gen_betons(ffcv):
    from ffcv.writer import DatasetWriter
    from ffcv.fields import RGBImageField, IntField
    out = {}
    with tempfile.TemporaryDirectory() as d:
        specs = {
            'raw32': (dict(write_mode='raw'), [(32, 32)], 40),
            'rawvar': (dict(write_mode='raw'), [(40, 30), (17, 64), (64, 64)], 12),
            'jpgvar': (dict(write_mode='jpg', jpeg_quality=90), [(50, 37), (64, 80), (33, 33)], 12),
            'smart_maxres': (dict(write_mode='smart', max_resolution=48, smart_threshold=3000),
                             [(100, 70), (30, 20)], 6),
        }
        for name, (kw, shapes, n) in specs.items():
            fn = os.path.join(d, name + '.beton')
            w = DatasetWriter(fn, {'image': RGBImageField(**kw), 'label': IntField()},
                              num_workers=1)
            w.from_indexed_dataset(_RawDS(n, shapes, 100), chunksize=5)
            out[f'beton_{name}'] = np.fromfile(fn, np.uint8)
            out[f'spec_{name}'] = np.array([n, 100] + [x for s in shapes for x in s], np.int64)
    return out


def gen_quasi():
    """QuasiRandom orders (quasi_random.py:14-85) on a multi-page .beton
    written by the reference writer: the allocation table (which defines the
    page -> sample sets) and the orders for several seeds / batch sizes /
    index subsets / epochs."""
    from ffcv.writer import DatasetWriter
    from ffcv.fields import RGBImageField, IntField
    from ffcv.reader import Reader
    from ffcv.memory_managers import OSCacheManager
    from ffcv.traversal_order.quasi_random import QuasiRandom
    out = {}

    class FakeLoader:
        pass
    with tempfile.TemporaryDirectory() as d:
        fn = os.path.join(d, 'quasi.beton')
        w = DatasetWriter(fn, {'image': RGBImageField(write_mode='raw'), 'label': IntField()},
                          page_size=1 << 21, num_workers=1)
        w.from_indexed_dataset(_RawDS(300, [(60, 80), (100, 120), (30, 40), (90, 70)], 7), chunksize=10)
        r = Reader(fn)
        at = r.alloc_table
        out['alloc'] = np.stack([at['sample_id'].astype(np.int64), at['ptr'].astype(np.int64),
                                 at['size'].astype(np.int64)], 1)
        out['page_size'] = np.array([r.page_size], np.int64)
        mm = OSCacheManager(r)
        for seed in [0, 7, 4000]:
            for bs in [4, 16]:
                for kind in ['all', 'third']:
                    fl = FakeLoader()
                    fl.memory_manager = mm
                    fl.indices = np.arange(300, dtype='uint64') if kind == 'all' else \
                        np.arange(0, 300, 3, dtype='uint64')
                    fl.seed = seed
                    fl.distributed = False
                    fl.batch_size = bs
                    q = QuasiRandom(fl)
                    for epoch in [0, 1, 3]:
                        out[f'order_s{seed}_b{bs}_{kind}_e{epoch}'] = np.asarray(q.sample_order(epoch), np.int64)
    return out


def main():
    install_stubs()
    sys.path.insert(0, REF)
    import ffcv  # noqa: F401
    from ffcv.fields import rgb_image
    from ffcv.transforms import Cutout, NormalizeImage
    from ffcv.traversal_order import Random, Sequential
    from ffcv.pipeline.compiler import Compiler
    Compiler.set_enabled(False)

    crops, centers = gen_crops(rgb_image)
    np.savez_compressed(os.path.join(HERE, 'crops.npz'), random=crops, center=centers)
    np.savez_compressed(os.path.join(HERE, 'cutout.npz'), rows=gen_cutout(Cutout))
    np.savez_compressed(os.path.join(HERE, 'normalize_lut.npz'), **gen_lut(NormalizeImage))
    np.savez_compressed(os.path.join(HERE, 'orders.npz'), **gen_orders(Random, Sequential))
    np.savez_compressed(os.path.join(HERE, 'betons.npz'), **gen_betons(ffcv))
    np.savez_compressed(os.path.join(HERE, 'quasi.npz'), **gen_quasi())
    print('golden vectors written to', HERE)


if __name__ == '__main__':
    main()
