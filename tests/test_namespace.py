"""The reference's import paths work unchanged (`ffcv.*` aliases `ffcv_amd.*`)."""
import sys


def test_ffcv_import_name():
    import ffcv
    from ffcv.loader import Loader, OrderOption
    from ffcv.fields import RGBImageField, IntField, FloatField, BytesField
    from ffcv.fields.decoders import (RandomResizedCropRGBImageDecoder, CenterCropRGBImageDecoder,
                                      SimpleRGBImageDecoder, IntDecoder)
    from ffcv.fields.ndarray import NDArrayField  # noqa: F401
    from ffcv.transforms import ToTensor, ToDevice, ToTorchImage, NormalizeImage, Cutout, RandomHorizontalFlip
    from ffcv.writer import DatasetWriter
    from ffcv.reader import Reader  # noqa: F401
    from ffcv.pipeline.operation import Operation
    from ffcv.pipeline.state import State  # noqa: F401
    from ffcv.pipeline.allocation_query import AllocationQuery  # noqa: F401
    from ffcv.pipeline.compiler import Compiler  # noqa: F401
    from ffcv.traversal_order import Random, Sequential, QuasiRandom  # noqa: F401
    from ffcv.memory_managers import OSCacheManager  # noqa: F401
    from ffcv.libffcv import imdecode, resize_crop, memcpy, read  # noqa: F401
    import ffcv_amd
    import ffcv_amd.loader
    import ffcv_amd.fields.rgb_image
    assert ffcv.Loader is ffcv_amd.Loader is Loader is ffcv_amd.loader.Loader
    assert ffcv.DatasetWriter is DatasetWriter
    assert RandomResizedCropRGBImageDecoder is ffcv_amd.fields.rgb_image.RandomResizedCropRGBImageDecoder
    import ffcv.fields.rgb_image
    assert sys.modules['ffcv.fields.rgb_image'] is sys.modules['ffcv_amd.fields.rgb_image']
    assert issubclass(Cutout, Operation) and OrderOption.RANDOM
