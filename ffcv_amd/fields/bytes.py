"""Variable-length bytes field (ffcv/fields/bytes.py:14-74), host decode."""
from dataclasses import replace
from typing import Callable, Tuple, Type

import numpy as np

from .base import Field, ARG_TYPE
from ..pipeline.operation import Operation
from ..pipeline.state import State
from ..pipeline.allocation_query import AllocationQuery


class BytesDecoder(Operation):
    per_sample = True

    def declare_state_and_memory(self, previous_state: State) -> Tuple[State, AllocationQuery]:
        max_size = self.metadata['size'].max()
        my_shape = (max_size,)
        return (replace(previous_state, jit_mode=True, shape=my_shape, dtype='<u1'),
                AllocationQuery(my_shape, dtype='<u1'))

    def generate_code(self) -> Callable:
        mem_read = self.memory_read

        def decoder(batch_indices, destination, metadata, storage_state):
            for dest_ix, source_ix in enumerate(batch_indices):
                field = metadata[source_ix]
                data = mem_read(field['ptr'], storage_state)
                destination[dest_ix, :field['size']] = data
            return destination[:len(batch_indices)]
        return decoder


class BytesField(Field):
    """A field of variable-length uint8 arrays."""

    def __init__(self):
        pass

    @property
    def metadata_type(self) -> np.dtype:
        return np.dtype([('ptr', '<u8'), ('size', '<u8')])

    @staticmethod
    def from_binary(binary: ARG_TYPE) -> Field:
        return BytesField()

    def to_binary(self) -> ARG_TYPE:
        return np.zeros(1, dtype=ARG_TYPE)[0]

    def encode(self, destination, field, malloc):
        ptr, buffer = malloc(field.size)
        buffer[:] = field
        destination['ptr'] = ptr
        destination['size'] = field.size

    def get_decoder_class(self) -> Type[Operation]:
        return BytesDecoder
