"""The Field interface of the .beton format.

A field type (reference ABC: ffcv/fields/base.py:8-45) must say four things:
the numpy dtype of its per-sample metadata record, how to serialise its
constructor arguments into the 1024-byte ``arguments`` blob of its field
descriptor (and back), how to encode one sample at write time, and which
Operation decodes it at load time.
"""
from __future__ import annotations

from abc import ABC, abstractmethod
from typing import Type

import numpy as np

from ..pipeline.operation import Operation

# ffcv/types.py FieldDescType 'arguments' slot: 1024 opaque bytes per field
ARG_TYPE = np.dtype([('', '<u1', 1024)])


def empty_arguments():
    """A zero-filled arguments blob (fields without constructor state)."""
    return np.zeros(1, dtype=ARG_TYPE)[0]


class Field(ABC):

    @property
    @abstractmethod
    def metadata_type(self) -> np.dtype:
        """dtype of the per-sample metadata record of this field."""

    @staticmethod
    @abstractmethod
    def from_binary(binary: ARG_TYPE) -> Field:
        """Rebuild the field from its descriptor's arguments blob."""

    @abstractmethod
    def to_binary(self) -> ARG_TYPE:
        """Serialise the constructor arguments into a blob."""

    @abstractmethod
    def encode(self, destination, field, malloc):
        """Write one sample: fill ``destination`` (its metadata record) and,
        for variable-size payloads, copy bytes into ``malloc(n)``'s buffer."""

    @abstractmethod
    def get_decoder_class(self) -> Type[Operation]:
        """Default decoder Operation for this field."""
