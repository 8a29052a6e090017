from .base import Field
from .basics import FloatField, IntField
from .rgb_image import RGBImageField
from .bytes import BytesField
from .unsupported import NDArrayField, JSONField, TorchTensorField

__all__ = ['Field', 'BytesField', 'IntField', 'FloatField', 'RGBImageField', 'NDArrayField',
           'JSONField', 'TorchTensorField']
