"""Scalar fields: IntField / FloatField and their decoders.

Reference behaviour (ffcv/fields/basics.py:14-93): the value lives entirely
in the sample's metadata record (no data region bytes), and decoding copies
``metadata[sample_id]`` into a ``(B, 1)`` host column that ToTensor /
ToDevice then move.  Labels ride alongside the images on the host; a batch
of them is a few KB, so there is nothing for the device to do here.
"""
from dataclasses import replace
from typing import Callable, Tuple, Type

import numpy as np

from .base import Field, ARG_TYPE, empty_arguments
from ..pipeline.operation import Operation
from ..pipeline.state import State
from ..pipeline.allocation_query import AllocationQuery


class _ScalarColumnDecoder(Operation):
    """Gathers one scalar per sample out of the metadata column."""
    per_sample = True
    column_dtype: np.dtype = None

    def declare_state_and_memory(self, previous_state: State) -> Tuple[State, AllocationQuery]:
        shape = (1,)
        state = replace(previous_state, jit_mode=True, shape=shape, dtype=self.column_dtype)
        return state, AllocationQuery(shape, dtype=self.column_dtype)

    def generate_code(self) -> Callable:
        def gather_column(indices, destination, column, storage_state):
            rows = np.asarray(indices, dtype=np.int64)
            out = destination[:rows.size]
            np.take(column, rows, out=out[:, 0])
            return out
        return gather_column


class IntDecoder(_ScalarColumnDecoder):
    """Decoder for an :class:`IntField` (signed 64-bit integers)."""
    column_dtype = np.dtype('<i8')
    dtype = column_dtype


class FloatDecoder(_ScalarColumnDecoder):
    """Decoder for a :class:`FloatField` (64-bit floats)."""
    column_dtype = np.dtype('<f8')
    dtype = column_dtype


class _ScalarField(Field):
    """A field stored as one metadata scalar per sample."""
    scalar_dtype: np.dtype = None
    decoder: Type[Operation] = None

    @property
    def metadata_type(self) -> np.dtype:
        return self.scalar_dtype

    @classmethod
    def from_binary(cls, binary: ARG_TYPE) -> Field:
        return cls()

    def to_binary(self) -> ARG_TYPE:
        return empty_arguments()

    def encode(self, destination, field, malloc):
        destination[0] = field

    def get_decoder_class(self) -> Type[Operation]:
        return self.decoder


class FloatField(_ScalarField):
    """A scalar float64 per sample (e.g. regression targets)."""
    scalar_dtype = np.dtype('<f8')
    decoder = FloatDecoder


class IntField(_ScalarField):
    """A scalar int64 per sample (e.g. class labels)."""
    scalar_dtype = np.dtype('<i8')
    decoder = IntDecoder
