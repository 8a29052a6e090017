from .basics import FloatDecoder, IntDecoder
from .rgb_image import (RandomResizedCropRGBImageDecoder, CenterCropRGBImageDecoder,
                        SimpleRGBImageDecoder)
from .bytes import BytesDecoder

__all__ = ['FloatDecoder', 'IntDecoder', 'RandomResizedCropRGBImageDecoder',
           'CenterCropRGBImageDecoder', 'SimpleRGBImageDecoder', 'BytesDecoder']
