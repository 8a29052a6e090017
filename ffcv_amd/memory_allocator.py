"""Page allocator of the ``.beton`` writer (behaviour of ffcv/memory_allocator.py:8-120).

The data region is a sequence of ``page_size`` pages starting at the first
page boundary after the metadata.  Every sample's regions live on ONE page:
a region that does not fit in what is left of the open page closes it and
opens the next one; if the same sample already placed a region on the page
just closed, its records are withdrawn and ``MemoryError`` tells the writer
the sample cannot be split (writer.py:42-59 then retries it from the fresh
page).  Closed pages are written at their file offset, zero padded.

This writer has one allocating process, so pages are opened in sample
order and written as they close -- no shared page counter and no
write-turn spin lock as in the multi-process reference, and the file is
deterministic.  ``allocations`` is the (sample id, file pointer, size) list
that becomes the allocation table.
"""
import numpy as np

from .utils import align_to_page


class MemoryAllocator:
    def __init__(self, fp, offset_start, page_size):
        self.fp = fp
        self.page_size = page_size
        self.data_start = align_to_page(offset_start, page_size)
        self.page = None            # index of the open page (None: none yet)
        self.fill = 0               # bytes used on the open page
        self.buf = np.zeros(page_size, '<u1')
        self.allocations = []       # (sample id, file pointer, size)
        self.current_sample_id = None
        self._pages_opened = 0

    def set_current_sample(self, current_sample_id):
        self.current_sample_id = current_sample_id

    @property
    def space_left_in_page(self):
        return 0 if self.page is None else self.page_size - self.fill

    def _page_pointer(self, page):
        return self.data_start + page * self.page_size

    def _open_next_page(self):
        """Close the open page and start a zeroed one; withdraw the current
        sample's records from the closed page (a sample never spans pages)."""
        self.flush_page()
        self.page = self._pages_opened
        self._pages_opened += 1
        self.fill = 0
        self.buf[:] = 0
        n_before = len(self.allocations)
        while self.allocations and self.allocations[-1][0] == self.current_sample_id:
            self.allocations.pop()
        if len(self.allocations) != n_before:
            raise MemoryError("Not enough memory to fit the whole sample")

    def malloc(self, size):
        """(file pointer, writable view) of ``size`` bytes for the current sample."""
        if size > self.page_size:
            raise ValueError(f"Tried allocating {size} but page size is {self.page_size}")
        if size > self.space_left_in_page:
            self._open_next_page()
        start, self.fill = self.fill, self.fill + size
        ptr = self._page_pointer(self.page) + start
        self.allocations.append((self.current_sample_id, ptr, size))
        return ptr, self.buf[start:self.fill]

    def flush_page(self):
        """Write the open page at its offset (zero-extending the file up to it)."""
        if self.page is None:
            return
        assert self.fill != 0, 'a page was opened and nothing was placed on it'
        at = self._page_pointer(self.page)
        end = self.fp.seek(0, 2)
        if end < at:
            self.fp.write(bytes(at - end))
        self.fp.seek(at)
        self.fp.write(self.buf.tobytes())
