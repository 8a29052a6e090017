"""Memory managers: how a sample's ``data_ptr`` becomes its bytes.

Reference: ffcv/memory_managers/base.py:32-82.  Every manager starts from the
.beton allocation table (``sample_id, ptr, size`` per allocation, written at
EOF in worker order) and derives:

* ``ptrs`` / ``sizes`` sorted by pointer, so a read is one ``searchsorted``;
* ``page_to_samples`` / ``sample_to_pages``: which ``page_size`` pages each
  sample occupies (a sample never straddles pages, memory_allocator.py), as
  sets filled in allocation-table order.  QuasiRandom iterates those sets,
  so their construction (and hence iteration order) follows the reference.

A manager hands out a per-epoch context (``schedule_epoch``) whose ``state``
is what decoders receive as ``storage_state`` and whose ``start_batch(b)``
may block until launch b's bytes are resident (process cache).
"""
from abc import ABC, abstractmethod
from collections import defaultdict
from contextlib import AbstractContextManager
from typing import Callable, Sequence

import numpy as np


class MemoryContext(AbstractContextManager):
    """Per-epoch view of the memory manager."""

    @property
    @abstractmethod
    def state(self):
        """Tuple handed to decoders as storage_state."""

    @abstractmethod
    def __enter__(self):
        return self

    def start_batch(self, batch: int):
        """Called before launch ``batch`` is built (no-op unless paged)."""

    @abstractmethod
    def __exit__(self, exc_type, exc_value, traceback):
        return None


class MemoryManager(ABC):

    def __init__(self, reader):
        self.reader = reader
        table = reader.alloc_table
        by_ptr = np.argsort(table['ptr'])
        self.ptrs = table['ptr'][by_ptr]
        self.sizes = table['size'][by_ptr]
        self.ptr_to_size = dict(zip(self.ptrs, self.sizes))
        shift = int(np.log2(reader.page_size))
        self.sample_to_pages = defaultdict(set)
        self.page_to_samples = defaultdict(set)
        for sample, page in zip(table['sample_id'], table['ptr'] >> shift):
            self.sample_to_pages[sample].add(page)
            self.page_to_samples[page].add(sample)

    @abstractmethod
    def schedule_epoch(self, batches: Sequence[Sequence[int]]) -> MemoryContext:
        """Context for one epoch that reads ``batches`` in order."""

    @abstractmethod
    def compile_reader(self) -> Callable:
        """``read(address, state) -> uint8 array`` of the sample at address."""

    @property
    @abstractmethod
    def state_type(self):
        """Type of the context's state."""
