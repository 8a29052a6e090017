"""Page allocator of the .beton writer (ffcv/memory_allocator.py:8-120).

Samples are appended to ``page_size`` pages; a sample never straddles a
page (if it does not fit, the sample restarts on a fresh page, writer.py:
42-59); pages are written in allocation order, zero padded.  Single-writer
version: allocation order = sample order, so the output is deterministic.
"""
import numpy as np

from .utils import align_to_page


class MemoryAllocator:
    def __init__(self, fp, offset_start, page_size):
        self.fp = fp
        self.offset = align_to_page(offset_start, page_size)
        self.page_size = page_size
        self.next_page = 0
        self.page_offset = 0
        self.my_page = -1
        self.page_data = np.zeros(self.page_size, '<u1')
        self.allocations = []
        self.current_sample_id = None

    def set_current_sample(self, current_sample_id):
        self.current_sample_id = current_sample_id

    @property
    def space_left_in_page(self):
        if self.my_page < 0:
            return 0
        return self.page_size - self.page_offset

    def malloc(self, size):
        if size > self.page_size:
            raise ValueError(f"Tried allocating {size} but page size is {self.page_size}")
        if size > self.space_left_in_page:
            self.flush_page()
            self.my_page = self.next_page
            self.next_page += 1
            self.page_offset = 0
            self.page_data.fill(0)
            region_in_previous_page = False
            while self.allocations and self.allocations[-1][0] == self.current_sample_id:
                self.allocations.pop()
                region_in_previous_page = True
            if region_in_previous_page:
                raise MemoryError("Not enough memory to fit the whole sample")
        previous_offset = self.page_offset
        self.page_offset += size
        buffer = self.page_data[previous_offset:self.page_offset]
        ptr = self.offset + self.my_page * self.page_size + previous_offset
        self.allocations.append((self.current_sample_id, ptr, size))
        return ptr, buffer

    def flush_page(self):
        if self.my_page < 0:
            return
        assert self.page_offset != 0
        expected_file_offset = self.offset + self.my_page * self.page_size
        current = self.fp.seek(0, 2)
        if current < expected_file_offset:
            self.fp.write(bytes(expected_file_offset - current))
        self.fp.seek(expected_file_offset)
        self.fp.write(self.page_data.tobytes())
