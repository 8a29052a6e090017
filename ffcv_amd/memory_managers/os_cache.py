"""OS page-cache manager (ffcv/memory_managers/os_cache.py:13-61).

The .beton is mapped read-only once per context; a sample's bytes are the
slice of the map that starts at its address and runs for the size of the
allocation-table entry found by binary search over the sorted pointers.
"""
import numpy as np

from .base import MemoryManager, MemoryContext


class OSCacheContext(MemoryContext):
    def __init__(self, manager: MemoryManager):
        self.manager = manager
        self.mmap = None

    @property
    def state(self):
        m = self.manager
        return (self.mmap, m.ptrs, m.sizes)

    def __enter__(self):
        entered = super().__enter__()
        if self.mmap is None:  # mapped lazily, kept across epochs
            self.mmap = np.memmap(self.manager.reader.file_name, dtype=np.uint8, mode='r')
        return entered

    def __exit__(self, *exc):
        return super().__exit__(*exc)


class OSCacheManager(MemoryManager):
    """Every epoch shares one context: the kernel's page cache does the work."""

    def __init__(self, reader):
        super().__init__(reader)
        self.context = OSCacheContext(self)

    def schedule_epoch(self, schedule):
        return self.context

    @property
    def state_type(self):
        return tuple

    def compile_reader(self):
        def read(address, mem_state):
            mapped, ptrs, sizes = mem_state
            entry = np.searchsorted(ptrs, address)
            return mapped[address:address + sizes[entry]]
        return read
