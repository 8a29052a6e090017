"""Field types that exist in the reference's type table (ffcv/types.py:46-55)
but are not on this framework's decode path.  They
parse (so a .beton containing them opens and its other fields load) but
decoding them raises."""
import json
from typing import Type

import numpy as np

from .base import Field, ARG_TYPE
from ..pipeline.operation import Operation


class _Unsupported(Field):
    name = 'field'

    def __init__(self, *args, **kwargs):
        self.args = args

    @staticmethod
    def from_binary(binary: ARG_TYPE):
        raise NotImplementedError

    def to_binary(self) -> ARG_TYPE:
        return np.zeros(1, dtype=ARG_TYPE)[0]

    def encode(self, destination, field, malloc):
        raise NotImplementedError(f'{self.name} is not on the MI355X decode path')

    def get_decoder_class(self) -> Type[Operation]:
        raise NotImplementedError(f'{self.name} decoding is not on the MI355X decode path; '
                                  'disable the field with pipelines={name: None}')


class NDArrayField(_Unsupported):
    """ffcv/fields/ndarray.py:54-119 layout: metadata {ptr}, args = dtype+shape."""
    name = 'NDArrayField'

    def __init__(self, dtype=np.dtype('<f4'), shape=(1,)):
        self.dtype = np.dtype(dtype)
        self.shape = tuple(shape)
        self.element_size = self.dtype.itemsize * int(np.prod(self.shape))

    @property
    def metadata_type(self):
        return np.dtype('<u8')

    @staticmethod
    def from_binary(binary):
        header_size = np.dtype([('type_length', '<u8'), ('shape', ('<u8', 32))]).itemsize
        hdr = np.frombuffer(binary.tobytes()[:header_size],
                            np.dtype([('type_length', '<u8'), ('shape', ('<u8', 32))]))[0]
        shape = tuple(int(x) for x in hdr['shape'] if x)
        return NDArrayField(np.dtype('<f4'), shape or (1,))


class TorchTensorField(NDArrayField):
    name = 'TorchTensorField'


class JSONField(_Unsupported):
    """ffcv/fields/json.py: stored like BytesField ({ptr, size})."""
    name = 'JSONField'

    @property
    def metadata_type(self):
        return np.dtype([('ptr', '<u8'), ('size', '<u8')])

    @staticmethod
    def from_binary(binary):
        return JSONField()

    @staticmethod
    def unpack(array):
        return json.loads(bytes(array).decode('utf-8'))
