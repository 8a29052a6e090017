from .base import MemoryManager, MemoryContext
from .os_cache import OSCacheManager


class ProcessCacheManager(OSCacheManager):
    """ffcv/memory_managers/process_cache: page scheduler for datasets larger
    than RAM.  Out of scope for this path: the OS-cache
    reader is used instead (same results)."""


__all__ = ['OSCacheManager', 'ProcessCacheManager', 'MemoryManager', 'MemoryContext']
