from .base import MemoryManager, MemoryContext
from .os_cache import OSCacheManager
from .process_cache import ProcessCacheManager


__all__ = ['OSCacheManager', 'ProcessCacheManager', 'MemoryManager', 'MemoryContext']
