"""OS page-cache manager (ffcv/memory_managers/os_cache.py:13-61): the whole
file is np.memmap'd; ``read(address, state)`` returns
``mmap[address:address + sizes[searchsorted(ptrs, address)]]``."""
import numpy as np

from .base import MemoryManager, MemoryContext


class OSCacheContext(MemoryContext):
    def __init__(self, manager: MemoryManager):
        self.manager = manager
        self.mmap = None

    @property
    def state(self):
        return (self.mmap, self.manager.ptrs, self.manager.sizes)

    def __enter__(self):
        res = super().__enter__()
        if self.mmap is None:
            self.mmap = np.memmap(self.manager.reader.file_name, 'uint8', mode='r')
        return res

    def __exit__(self, __exc_type, __exc_value, __traceback):
        return super().__exit__(__exc_type, __exc_value, __traceback)


class OSCacheManager(MemoryManager):

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
            size = mem_state[2][np.searchsorted(mem_state[1], address)]
            return mem_state[0][address:address + size]
        return read
