"""Memory managers (ffcv/memory_managers/base.py:32-82): map a sample's
data_ptr to its bytes.  ptrs/sizes come from the allocation table sorted by
pointer (base.py:40-45)."""
from abc import ABC, abstractmethod
from collections import defaultdict
from contextlib import AbstractContextManager
from typing import Callable, Mapping, Sequence, Set

import numpy as np


class MemoryContext(AbstractContextManager):

    @property
    @abstractmethod
    def state(self):
        raise NotImplementedError()

    @abstractmethod
    def __enter__(self):
        return super().__enter__()

    def start_batch(self, batch: int):
        pass

    @abstractmethod
    def __exit__(self, __exc_type, __exc_value, __traceback):
        return super().__exit__(__exc_type, __exc_value, __traceback)


class MemoryManager(ABC):

    def __init__(self, reader):
        self.reader = reader
        alloc_table = self.reader.alloc_table
        self.ptrs = alloc_table['ptr']
        self.sizes = alloc_table['size']
        order = np.argsort(self.ptrs)
        self.ptrs = self.ptrs[order]
        self.sizes = self.sizes[order]
        self.ptr_to_size = dict(zip(self.ptrs, self.sizes))
        page_size_bit_location = int(np.log2(reader.page_size))
        page_locations = alloc_table['ptr'] >> page_size_bit_location
        sample_to_pages: Mapping[int, Set[int]] = defaultdict(set)
        page_to_samples: Mapping[int, Set[int]] = defaultdict(set)
        for sid, pid in zip(alloc_table['sample_id'], page_locations):
            sample_to_pages[sid].add(pid)
            page_to_samples[pid].add(sid)
        self.sample_to_pages = sample_to_pages
        self.page_to_samples = page_to_samples
        super().__init__()

    @abstractmethod
    def schedule_epoch(self, batches: Sequence[Sequence[int]]) -> MemoryContext:
        raise NotImplementedError()

    @abstractmethod
    def compile_reader(self) -> Callable:
        raise NotImplementedError()

    @property
    @abstractmethod
    def state_type(self):
        raise NotImplementedError()
