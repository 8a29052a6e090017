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

# type id -> field class (255: a slot without a field)
_FIELD_CLASSES = (FloatField, IntField, RGBImageField, BytesField, NDArrayField,
                  JSONField, TorchTensorField)
TYPE_ID_HANDLER = {255: None, **dict(enumerate(_FIELD_CLASSES))}


def get_handlers(field_descriptors):
    """One decoded field handler per descriptor row (None for id 255)."""
    def handler(desc):
        cls = TYPE_ID_HANDLER[desc['type_id']]
        return None if cls is None else cls.from_binary(desc['arguments'])
    return [handler(d) for d in field_descriptors]


def get_metadata_type(handlers: List[Field]) -> np.dtype:
    """Per-sample metadata record: the fields' metadata types, C-aligned."""
    return np.dtype([('', h.metadata_type) for h in handlers], align=True)
