"""Operator API (ffcv/pipeline/operation.py:14-41), unchanged for users.

``declare_state_and_memory(previous_state) -> (State, AllocationQuery|tuple|
None)`` and ``generate_code() -> callable``.  A decoder's callable is
``decode(batch_indices, destination, metadata, storage_state)``; a
transform's is ``fn(images, dst)`` or ``fn(images, dst, indices)`` when it
sets ``with_indices``.  User operations written for the reference run
unchanged as plain Python (the reference's ``Compiler.set_enabled(False)``
semantics; there is no numba here).

Operations that know how to run on a HIP device set the class attribute
``device_aware = True``; the graph inserts a device->host transfer in
front of any other operation that receives device-resident data.

``per_sample = True`` declares that the operation treats every sample of a
batch independently (no batch-level mixing such as ImageMixup): the
EpochIterator may then run several consecutive batches through the graph as
one launch (one decode launch fills the GPU) and hand them out one by one.
Unknown user operations default to False, which keeps one batch per run.
"""
from abc import ABC, abstractmethod
from typing import TYPE_CHECKING, Callable, Optional, Tuple

import numpy as np

from .allocation_query import AllocationQuery
from .state import State

if TYPE_CHECKING:
    from ..fields.base import Field


class Operation(ABC):
    device_aware = False
    per_sample = False

    def __init__(self):
        self.metadata: np.ndarray = None
        self.memory_read: Callable[[np.uint64], np.ndarray] = None

    def accept_field(self, field: 'Field'):
        self.field: 'Field' = field

    def accept_globals(self, metadata, memory_read):
        self.metadata = metadata
        self.memory_read = memory_read

    @abstractmethod
    def generate_code(self) -> Callable:
        raise NotImplementedError

    def declare_shared_memory(self, previous_state: State) -> Optional[AllocationQuery]:
        return None

    def generate_code_for_shared_state(self) -> Optional[Callable]:
        return None

    @abstractmethod
    def declare_state_and_memory(self, previous_state: State) -> Tuple[State, Optional[AllocationQuery]]:
        raise NotImplementedError
