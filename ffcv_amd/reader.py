"""``.beton`` reader.

File layout (format version 2; reference parser
ffcv/reader.py:7-72):

    [ header: HeaderType, 24 B ]
    [ num_fields x FieldDescType (type id, name, 1024-byte argument blob) ]
    [ num_samples x metadata record (one struct member per field) ]
    [ data pages ... ]
    [ allocation table (sample_id, ptr, size) x n at header.alloc_table_ptr ]

Everything is parsed with ``np.fromfile`` into read-only structured arrays;
sample bytes themselves are left to the memory managers (mmap / page cache)
and, on the device path, to the HBM copy of the whole file.
"""
import numpy as np

from .utils import decode_null_terminated_string
from .types import (ALLOC_TABLE_TYPE, HeaderType, CURRENT_VERSION, FieldDescType,
                    get_handlers, get_metadata_type)


def _frozen(a):
    a.setflags(write=False)
    return a


class Reader:
    """Parsed header, field handlers, metadata and allocation table of one file.

    ``custom_handlers`` maps a field name to the Field class of a custom
    (type id 255) field, whose descriptor cannot name its own handler.
    """

    def __init__(self, fname, custom_handlers={}):
        self._fname = fname
        self._custom_handlers = dict(custom_handlers)
        self.read_header()
        self.read_field_descriptors()
        self.read_metadata()
        self.read_allocation_table()

    @property
    def file_name(self):
        return self._fname

    def read_header(self):
        self.header = _frozen(np.fromfile(self._fname, dtype=HeaderType, count=1))[0]
        if self.header['version'] != CURRENT_VERSION:
            raise AssertionError(f"file format mismatch: code={CURRENT_VERSION},"
                                 f"file={self.header['version']}")
        self.num_samples = self.header['num_samples']
        self.page_size = self.header['page_size']
        self.num_fields = self.header['num_fields']

    def read_field_descriptors(self):
        descs = _frozen(np.fromfile(self._fname, dtype=FieldDescType, count=self.num_fields,
                                    offset=HeaderType.itemsize))
        self.field_descriptors = descs
        self.field_names = [decode_null_terminated_string(d['name']) for d in descs]
        handlers = {}
        for name, desc, builtin in zip(self.field_names, descs, get_handlers(descs)):
            custom = self._custom_handlers.get(name)
            handler = custom.from_binary(desc['arguments']) if custom is not None else builtin
            if handler is None:
                raise ValueError(f"Must specify a custom_field entry for custom field {name}")
            handlers[name] = handler
        self.handlers = handlers
        self.metadata_type = get_metadata_type(list(handlers.values()))

    def read_metadata(self):
        start = HeaderType.itemsize + self.field_descriptors.nbytes
        self.metadata = _frozen(np.fromfile(self._fname, dtype=self.metadata_type,
                                            count=self.num_samples, offset=start))

    def read_allocation_table(self):
        self.alloc_table = _frozen(np.fromfile(self._fname, dtype=ALLOC_TABLE_TYPE,
                                               offset=self.header['alloc_table_ptr']))
