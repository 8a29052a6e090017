"""``.beton`` on-disk format, version 2 (ffcv/types.py:13-77).

Byte-compatible with files written by the reference (SURVEY.md Appendix A;
tests/test_format.py reads the reference writer's own output).
"""
from typing import List

import numpy as np

from .fields.base import Field
from .fields import (FloatField, IntField, RGBImageField, BytesField, NDArrayField,
                     JSONField, TorchTensorField)

CURRENT_VERSION = 2

HeaderType = np.dtype([
    ('version', '<u2'),
    ('num_fields', '<u2'),
    ('page_size', '<u4'),
    ('num_samples', '<u8'),
    ('alloc_table_ptr', '<u8')
], align=True)

ALLOC_TABLE_TYPE = np.dtype([
    ('sample_id', '<u8'),
    ('ptr', '<u8'),
    ('size', '<u8'),
])

FieldDescType = np.dtype([
    ('type_id', '<u1'),
    ('name', ('<u1', 16)),
    ('arguments', ('<u1', (1024,)))
], align=True)

TYPE_ID_HANDLER = {
    255: None,
    0: FloatField,
    1: IntField,
    2: RGBImageField,
    3: BytesField,
    4: NDArrayField,
    5: JSONField,
    6: TorchTensorField,
}


def get_handlers(field_descriptors):
    handlers = []
    for field_descriptor in field_descriptors:
        type_id = field_descriptor['type_id']
        Handler = TYPE_ID_HANDLER[type_id]
        if Handler is None:
            handlers.append(None)
        else:
            handlers.append(Handler.from_binary(field_descriptor['arguments']))
    return handlers


def get_metadata_type(handlers: List[Field]) -> np.dtype:
    return np.dtype([('', handler.metadata_type) for handler in handlers], align=True)
