"""Scalar fields (ffcv/fields/basics.py:14-93).  Labels ride alongside the
image on the host: ``destination[ix] = metadata[sample_id]`` then
ToTensor/ToDevice move them (a few bytes per sample)."""
from dataclasses import replace
from typing import Callable, Tuple, Type

import numpy as np

from .base import Field, ARG_TYPE
from ..pipeline.operation import Operation
from ..pipeline.state import State
from ..pipeline.allocation_query import AllocationQuery


class BasicDecoder(Operation):
    def declare_state_and_memory(self, previous_state: State) -> Tuple[State, AllocationQuery]:
        my_shape = (1,)
        return (replace(previous_state, jit_mode=True, shape=my_shape, dtype=self.dtype),
                AllocationQuery(my_shape, dtype=self.dtype))

    def generate_code(self) -> Callable:
        def decoder(indices, destination, metadata, storage_state):
            n = len(indices)
            destination[:n, 0] = metadata[np.asarray(indices, dtype=np.int64)]
            return destination[:n]
        return decoder


class IntDecoder(BasicDecoder):
    """Decoder for signed integer scalars (int64)."""
    dtype = np.dtype('<i8')


class FloatDecoder(BasicDecoder):
    """Decoder for floating point scalars (float64)."""
    dtype = np.dtype('<f8')


class FloatField(Field):
    def __init__(self):
        pass

    @property
    def metadata_type(self) -> np.dtype:
        return np.dtype('<f8')

    @staticmethod
    def from_binary(binary: ARG_TYPE) -> Field:
        return FloatField()

    def to_binary(self) -> ARG_TYPE:
        return np.zeros(1, dtype=ARG_TYPE)[0]

    def encode(self, destination, field, malloc):
        destination[0] = field

    def get_decoder_class(self) -> Type[Operation]:
        return FloatDecoder


class IntField(Field):
    @property
    def metadata_type(self) -> np.dtype:
        return np.dtype('<i8')

    @staticmethod
    def from_binary(binary: ARG_TYPE) -> Field:
        return IntField()

    def to_binary(self) -> ARG_TYPE:
        return np.zeros(1, dtype=ARG_TYPE)[0]

    def encode(self, destination, field, malloc):
        destination[0] = field

    def get_decoder_class(self) -> Type[Operation]:
        return IntDecoder
