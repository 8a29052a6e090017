"""Process-cache memory manager: the page scheduler used with ``os_cache=False``.

Behaviour follows ffcv/memory_managers/process_cache/ (manager.py:9-45,
context.py:10-59, schedule.py:23-131, page_reader.py:9-36):

* At the start of an epoch the batches are known, so the set of .beton pages
  each batch touches is known.  A page may be read up to ``prefetch_ahead``
  (3) batches before the first batch that needs it and is released after
  the last batch that needs it (schedule.py:23-79).
* Pages live in a fixed pool of ``num_slots`` page-sized slots.  Slots are
  handed out greedily in batch order, frees first, so the pool is as small as
  the largest number of pages alive at once (the prefetch windows are
  intervals, so greedy colouring is optimal).
* Worker threads read pages with ``pread`` into their slots
  (page_reader.py:22-36, libffcv.py:11-19 ``read``); ``start_batch(b)`` queues
  batch b's prefetches and blocks until every page batch b needs has landed
  (schedule.py:110-131).
* ``read(address, state)`` maps a sample pointer to its slot:
  ``memory[page_to_slot[address >> log2(page)], address & (page - 1):][:size]``
  (manager.py:34-45).  Samples never cross a page (the writer's allocator).

Results are the OS-cache results byte for byte; only where the bytes come from
differs.  The device PCIe path (``device_cache=False``) gathers each batch's
compressed samples out of the slot pool with the same native gather it uses
on the memory map (``BatchContext._stage``).
"""
import os
import threading
from dataclasses import dataclass, field
from queue import Queue
from typing import Dict, List, Sequence, Set

import numpy as np

from .base import MemoryManager, MemoryContext

PREFETCH_AHEAD = 3
NUM_READERS = 12


@dataclass
class PageSchedule:
    num_slots: int
    page_to_slot: Dict[int, int]
    prefetch_at: List[List[int]] = field(default_factory=list)  # per batch: pages to queue
    needed_at: List[List[int]] = field(default_factory=list)    # per batch: pages to wait for


def compute_schedule(pages_per_batch: Sequence[Set[int]], prefetch_ahead: int = PREFETCH_AHEAD) -> PageSchedule:
    """Slot assignment for one epoch (schedule.py:23-79 semantics)."""
    nb = len(pages_per_batch)
    first, last = {}, {}
    for b, pages in enumerate(pages_per_batch):
        for p in pages:
            first.setdefault(p, b)
            last[p] = b
    prefetch_at = [[] for _ in range(nb)]
    needed_at = [[] for _ in range(nb)]
    release_at = [[] for _ in range(nb + 1)]
    for p in sorted(first):
        prefetch_at[max(0, first[p] - prefetch_ahead)].append(p)
        needed_at[first[p]].append(p)
        release_at[last[p] + 1].append(p)
    page_to_slot = {}
    free: List[int] = []
    n_slots = 0
    for b in range(nb):
        for p in release_at[b]:
            free.append(page_to_slot[p])
        for p in prefetch_at[b]:
            if free:
                page_to_slot[p] = free.pop()
            else:
                page_to_slot[p] = n_slots
                n_slots += 1
    return PageSchedule(n_slots, page_to_slot, prefetch_at, needed_at)


def read(fileno: int, destination: np.ndarray, offset: int) -> int:
    """ffcv/libffcv.py:11-19 ``read``: pread into ``destination``; returns the
    bytes read (short at the end of the file)."""
    return os.preadv(fileno, [memoryview(destination).cast('B')], int(offset))


class _PageReaders:
    """Pool of reader threads: (page, slot) requests in, page numbers out."""

    def __init__(self, fname, memory, n):
        self.requests: Queue = Queue()
        self.landed: Queue = Queue()
        self.memory = memory
        self.error = None
        self.threads = [threading.Thread(target=self._run, args=(fname,), daemon=True) for _ in range(n)]
        for t in self.threads:
            t.start()

    def _run(self, fname):
        page_size = self.memory.shape[1]
        with open(fname, 'rb') as f:
            fd = f.fileno()
            while True:
                req = self.requests.get()
                if req is None:
                    return
                page, slot = req
                try:
                    read(fd, self.memory[slot], page * page_size)
                except BaseException as e:  # re-raised by start_batch
                    self.error = e
                self.landed.put(page)

    def close(self):
        for _ in self.threads:
            self.requests.put(None)


class ProcessCacheContext(MemoryContext):

    def __init__(self, manager: 'ProcessCacheManager', batches):
        self.manager = manager
        self.batches = batches
        self.page_size = manager.reader.page_size
        self.readers = None
        self.next_batch = 0
        self.landed: Set[int] = set()

    @property
    def state(self):
        return (self.memory, self.manager.ptrs, self.manager.sizes, self.page_to_slot)

    def __enter__(self):
        s2p = self.manager.sample_to_pages
        pages = [set().union(*(s2p[int(i)] for i in batch)) if len(batch) else set()
                 for batch in self.batches]
        self.schedule = compute_schedule(pages)
        self.memory = np.zeros((self.schedule.num_slots, self.page_size), dtype='<u1')
        max_page = max(self.schedule.page_to_slot, default=-1)
        self.page_to_slot = np.zeros(max_page + 1, dtype=np.uint32)
        for p, s in self.schedule.page_to_slot.items():
            self.page_to_slot[p] = s
        self.readers = _PageReaders(self.manager.reader.file_name, self.memory,
                                    min(NUM_READERS, max(1, self.schedule.num_slots)))
        self.next_batch = 0
        self.landed = set()
        return self

    def start_batch(self, batch: int):
        if batch != self.next_batch:  # schedule.py:111 (batches are read in order)
            raise RuntimeError(f'process cache: batch {batch} started, expected {self.next_batch}')
        sch = self.schedule
        for p in sch.prefetch_at[batch]:
            self.readers.requests.put((p, sch.page_to_slot[p]))
        for p in sch.needed_at[batch]:
            while p not in self.landed:
                self.landed.add(self.readers.landed.get())
        if self.readers.error is not None:
            raise self.readers.error
        self.next_batch = batch + 1

    def __exit__(self, *args):
        if self.readers is not None:
            self.readers.close()
            self.readers = None


class ProcessCacheManager(MemoryManager):

    def schedule_epoch(self, batches) -> MemoryContext:
        return ProcessCacheContext(self, batches)

    @property
    def state_type(self):
        return tuple

    def compile_reader(self):
        shift = int(np.log2(self.reader.page_size))
        mask = (1 << shift) - 1

        def read_sample(address, mem_state):
            size = int(mem_state[2][np.searchsorted(mem_state[1], address)])
            address = int(address)
            off = address & mask
            return mem_state[0][mem_state[3][address >> shift], off:off + size]

        return read_sample


def host_source(state, ptrs: np.ndarray):
    """(flat host buffer, byte offsets) of samples at file pointers ``ptrs``
    under a memory-manager state: the mmap and the pointers themselves for
    the OS cache, the slot pool and slot-relative offsets for this cache."""
    if len(state) == 4:
        memory, _, _, page_to_slot = state
        ps = memory.shape[1]
        shift = int(np.log2(ps))
        ptrs = np.asarray(ptrs, dtype=np.uint64)
        slots = page_to_slot[(ptrs >> np.uint64(shift)).astype(np.int64)].astype(np.uint64)
        return memory.reshape(-1), slots * np.uint64(ps) + (ptrs & np.uint64(ps - 1))
    return state[0], np.asarray(ptrs, dtype=np.uint64)
