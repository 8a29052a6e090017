"""Graph lowering (CPU, no kernels launched): which operations the schedule
fuses into the crop/resize launch, and the implicit host transfers."""
import os
import tempfile

import numpy as np
import pytest
import torch as ch

from ffcv_amd.fields import RGBImageField, IntField
from ffcv_amd.fields.decoders import RandomResizedCropRGBImageDecoder, CenterCropRGBImageDecoder
from ffcv_amd.pipeline.graph import Graph
from ffcv_amd.pipeline import PipelineSpec
from ffcv_amd.reader import Reader
from ffcv_amd.memory_managers import OSCacheManager
from ffcv_amd.transforms import (Cutout, NormalizeImage, ToTensor, ToDevice, ToTorchImage,
                                 RandomHorizontalFlip, Convert)
from tests.helpers import NaturalDS, write

MEAN = np.array([0.485, 0.456, 0.406]) * 255
STD = np.array([0.229, 0.224, 0.225]) * 255


@pytest.fixture(scope='module')
def beton():
    d = tempfile.mkdtemp()
    return write(os.path.join(d, 'g.beton'), NaturalDS(6, var=True),
                 {'image': RGBImageField(write_mode='jpg'), 'label': IntField()})


def _graph(beton, ops):
    r = Reader(beton)
    specs = {'image': PipelineSpec('image', transforms=ops)}
    g = Graph(specs, r.handlers, {'image': 0, 'label': 1}, r.metadata,
              OSCacheManager(r).compile_reader(), device='cuda:0')
    return g, ops[0]


def test_c3_pipeline_fully_fused(beton):
    ops = [RandomResizedCropRGBImageDecoder((224, 224)), Cutout(32, (124, 116, 103)), ToTensor(),
           ToDevice(ch.device('cuda:0'), non_blocking=True), ToTorchImage(),
           NormalizeImage(MEAN, STD, np.float16)]
    g, dec = _graph(beton, ops)
    assert dec._fused_cutout is ops[1] and dec._fused_normalize is ops[5]
    assert ops[1]._absorbed and ops[5]._absorbed
    assert dec.output_dtype == ch.float16


def test_flip_cutout_order_recorded(beton):
    ops = [CenterCropRGBImageDecoder((64, 64), 0.875), RandomHorizontalFlip(), Cutout(8)]
    g, dec = _graph(beton, ops)
    assert dec._fused_flip is ops[1] and dec._fused_cutout is ops[2] and not dec._cutout_before_flip
    ops = [CenterCropRGBImageDecoder((64, 64), 0.875), Cutout(8), RandomHorizontalFlip()]
    g, dec = _graph(beton, ops)
    assert dec._cutout_before_flip


def test_fusion_stops_at_unknown_op(beton):
    ops = [RandomResizedCropRGBImageDecoder((64, 64)), Convert(ch.float32), Cutout(8)]
    g, dec = _graph(beton, ops)
    assert dec._fused_cutout is None and not ops[2]._absorbed
