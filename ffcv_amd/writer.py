"""``.beton`` writer (ffcv/writer.py:122-347, ffcv/memory_allocator.py).

Same file layout as the reference (header, field descriptors, metadata,
page-aligned data pages, allocation table at EOF).  Encoding (JPEG, resize)
runs in a process pool; allocation and writing happen in sample order in the
parent, so ``num_workers`` does not change the bytes written (with one
worker the reference writes the same file: tests/test_format.py).
"""
from os import sched_getaffinity, SEEK_END
from typing import List, Mapping

import numpy as np

from .fields.base import Field
from .memory_allocator import MemoryAllocator
from .types import (TYPE_ID_HANDLER, get_metadata_type, HeaderType, FieldDescType,
                    CURRENT_VERSION, ALLOC_TABLE_TYPE)
from .utils import is_power_of_2

MIN_PAGE_SIZE = 1 << 21
MAX_PAGE_SIZE = 1 << 32


class _Recorder:
    """Records (size, bytes) mallocs of one sample in a worker."""

    def __init__(self):
        self.blobs = []

    def malloc(self, size):
        buf = np.zeros(size, np.uint8)
        self.blobs.append(buf)
        return len(self.blobs) - 1, buf


def _encode_sample(args):
    fields, metadata_type, sample = args
    rec = _Recorder()
    meta = np.zeros(1, dtype=metadata_type)
    for name, field, value in zip(metadata_type.names, fields.values(), sample):
        field.encode(meta[name][0:1], value, rec.malloc)
    return meta, rec.blobs


class DatasetWriter:
    """Writes given dataset into FFCV format (.beton).

    Parameters
    ----------
    fname: str
        File name to store dataset in FFCV format (.beton)
    fields : Mapping[str, Field]
        Map from keys to Field's (order matters!)
    page_size : int
        Page size used internally
    num_workers : int
        Number of processes used to encode samples
    """

    def __init__(self, fname: str, fields: Mapping[str, Field], page_size: int = 4 * MIN_PAGE_SIZE,
                 num_workers: int = -1):
        self.fields = fields
        self.fname = fname
        self.metadata_type = get_metadata_type(list(self.fields.values()))
        self.num_workers = num_workers
        if self.num_workers < 1:
            self.num_workers = len(sched_getaffinity(0))
        if not is_power_of_2(page_size):
            raise ValueError('page_size isnt a power of 2')
        if page_size < MIN_PAGE_SIZE:
            raise ValueError(f"page_size can't be lower than{MIN_PAGE_SIZE}")
        if page_size >= MAX_PAGE_SIZE:
            raise ValueError(f"page_size can't be bigger(or =) than{MAX_PAGE_SIZE}")
        self.page_size = page_size

    def _header(self, num_samples):
        header = np.zeros(1, dtype=HeaderType)[0]
        header['version'] = CURRENT_VERSION
        header['num_samples'] = num_samples
        header['num_fields'] = len(self.fields)
        header['page_size'] = self.page_size
        fields_descriptor = np.zeros(len(self.fields), dtype=FieldDescType)
        field_type_to_type_id = {v: k for (k, v) in TYPE_ID_HANDLER.items()}
        fieldname_max_len = fields_descriptor[0]['name'].shape[0]
        for i, (name, field) in enumerate(self.fields.items()):
            type_id = field_type_to_type_id.get(type(field), 255)
            encoded_name = np.frombuffer(name.encode('ascii'), dtype='<u1')
            actual_length = min(fieldname_max_len, len(encoded_name))
            fields_descriptor[i]['type_id'] = type_id
            fields_descriptor[i]['name'][:actual_length] = encoded_name[:actual_length]
            fields_descriptor[i]['arguments'][:] = field.to_binary()[0]
        return header, fields_descriptor

    def _write_direct(self, dataset, indices):
        """One process: fields encode straight into allocator storage, exactly
        like the reference's worker (writer.py:42-59, handle_sample)."""
        num_samples = len(indices)
        header, descriptors = self._header(num_samples)
        metadata = np.zeros(num_samples, dtype=self.metadata_type)
        metadata_start = HeaderType.itemsize + descriptors.nbytes
        data_region_start = metadata_start + metadata.nbytes
        names = self.metadata_type.names
        with open(self.fname, 'wb') as fp:
            fp.write(header.tobytes())
            fp.write(descriptors.tobytes())
            alloc = MemoryAllocator(fp, data_region_start, self.page_size)
            for dest_ix, source_ix in enumerate(indices):
                sample = dataset[int(source_ix)]
                for i in range(2):
                    try:
                        alloc.set_current_sample(dest_ix)
                        for name, field, value in zip(names, self.fields.values(), sample):
                            field.encode(metadata[name][dest_ix:dest_ix + 1], value, alloc.malloc)
                        break
                    except MemoryError:
                        if i == 1:
                            raise
            self._finish(fp, alloc, header, metadata, metadata_start)

    def _finish(self, fp, alloc, header, metadata, metadata_start):
        alloc.flush_page()
        fp.seek(metadata_start)
        fp.write(metadata.tobytes())
        fp.seek(0, SEEK_END)
        allocation_table_location = fp.tell()
        table = np.array(alloc.allocations, dtype=ALLOC_TABLE_TYPE) if alloc.allocations \
            else np.array([]).view(ALLOC_TABLE_TYPE)
        fp.write(table.tobytes())
        header['alloc_table_ptr'] = allocation_table_location
        fp.seek(0)
        fp.write(header.tobytes())

    def _write(self, samples_iter, num_samples):
        header, descriptors = self._header(num_samples)
        metadata = np.zeros(num_samples, dtype=self.metadata_type)
        metadata_start = HeaderType.itemsize + descriptors.nbytes
        data_region_start = metadata_start + metadata.nbytes
        with open(self.fname, 'wb') as fp:
            fp.write(header.tobytes())
            fp.write(descriptors.tobytes())
            alloc = MemoryAllocator(fp, data_region_start, self.page_size)
            for dest_ix, (meta, blobs) in samples_iter:
                for attempt in range(2):
                    try:
                        alloc.set_current_sample(dest_ix)
                        ptrs = []
                        for b in blobs:
                            ptr, storage = alloc.malloc(b.size)
                            storage[:] = b
                            ptrs.append(ptr)
                        break
                    except MemoryError:
                        if attempt == 1:
                            raise
                # patch recorded malloc handles with the real file pointers
                m = meta.copy()
                self._patch_pointers(m, ptrs)
                metadata[dest_ix] = m[0]
            self._finish(fp, alloc, header, metadata, metadata_start)

    def _patch_pointers(self, meta, ptrs):
        """Fields store the malloc handle (blob index) in their metadata; map
        it to the file pointer.  Pointer fields: 'data_ptr' (RGB), 'ptr'
        (bytes / ndarray / json)."""
        for name, field in zip(self.metadata_type.names, self.fields.values()):
            sub = meta[name]
            if sub.dtype.names is None:
                if type(field).__name__ in ('NDArrayField', 'TorchTensorField'):
                    sub[...] = ptrs[int(sub[0])]
                continue
            for key in ('data_ptr', 'ptr'):
                if key in sub.dtype.names:
                    sub[key] = ptrs[int(sub[key][0])]

    def from_indexed_dataset(self, dataset, indices: List[int] = None, chunksize=100,
                             shuffle_indices: bool = False):
        """Read dataset from an indexable dataset (writer.py:238-268)."""
        if indices is None:
            indices = np.arange(len(dataset))
        if shuffle_indices:
            indices = np.array(indices)
            np.random.shuffle(indices)
        n = len(indices)
        if self.num_workers <= 1:
            return self._write_direct(dataset, indices)
        jobs = ((self.fields, self.metadata_type, dataset[int(i)]) for i in indices)
        if self.num_workers > 1:
            import multiprocessing as mp
            with mp.get_context('fork').Pool(self.num_workers) as pool:
                results = pool.imap(_encode_sample, jobs, chunksize=max(1, chunksize))
                self._write(enumerate(results), n)
        else:
            self._write(enumerate(map(_encode_sample, jobs)), n)

    def from_webdataset(self, shards: List[str], pipeline):
        raise NotImplementedError('webdataset ingestion is outside the MI355X decode path')
