"""Per-batch execution context handed to decoders as ``storage_state``.

The reference passes the memory manager's state tuple (mmap, ptrs, sizes)
(memory_managers/os_cache.py:30-31) to decoders, which read bytes with
``memory_read(ptr, storage_state)``.  Here the same object also carries the
device side of the schedule: the HBM-resident bytes, the per-field
descriptor tables, the slot's HIP stream, the device copy of the batch
indices, the RNG contract inputs (loader seed, epoch) and a per-slot JPEG
decoder context.  Indexing it like the reference's tuple still works for
host readers.
"""
import threading

import numpy as np
import torch as ch

_tls = threading.local()


def current():
    """The BatchContext of the batch being built on this thread."""
    return getattr(_tls, 'ctx', None)


def set_current(ctx):
    _tls.ctx = ctx


class DeviceDataset:
    """Device-side view of one .beton: bytes in HBM + descriptor tables."""

    def __init__(self, reader, memory_manager, device, data=None, data_base=0, entropy_index=False):
        self.reader = reader
        self.use_entropy_index = entropy_index
        self._eidx = {}
        self.memory_manager = memory_manager
        self.device = device
        self.data = data              # torch uint8 tensor (file bytes) on device
        self.data_base = data_base    # file offset of data[0]
        self._tables = {}
        self._modes = {}
        self._limits = {}

    staged = False

    def host_table(self, f_ix):
        self.table(f_ix)
        return self._host_tables[f_ix]

    def table(self, f_ix):
        """ffcv_sample[N] for an RGBImageField, built once and kept in HBM."""
        if not hasattr(self, '_host_tables'):
            self._host_tables = {}
        if f_ix not in self._tables:
            from .. import libffcv as L
            md = self.reader.metadata[f'f{f_ix}']
            mm = self.memory_manager
            ptr = md['data_ptr'].astype(np.uint64)
            pos = np.searchsorted(mm.ptrs, ptr)
            pos = np.minimum(pos, len(mm.ptrs) - 1)
            sizes = np.where(mm.ptrs[pos] == ptr, mm.sizes[pos], 0).astype(np.uint64)
            t = np.zeros(len(md), L.SAMPLE_DTYPE)
            t['offset'] = ptr - np.uint64(self.data_base)
            t['size'] = sizes
            t['height'] = md['height']
            t['width'] = md['width']
            t['mode'] = md['mode']
            self._host_tables[f_ix] = t
            self._tables[f_ix] = ch.from_numpy(t.view(np.uint8)).to(self.device)
            self._modes[f_ix] = (bool((md['mode'] == 0).any()), bool((md['mode'] == 1).any()))
            jpg = md['mode'] == 0
            self._limits[f_ix] = (int(md['height'].max()), int(md['width'].max()),
                                  int(sizes[jpg].max()) if jpg.any() else 1)
        return self._tables[f_ix]

    def arena_bytes(self, f_ix, max_batch):
        """JPEG scratch arena for launches of max_batch samples of field
        f_ix: the sum of the largest max_batch per-image bounds (one huge image
        in a dataset costs its own size once, not x batch)."""
        key = (f_ix, int(max_batch))
        if not hasattr(self, '_arena'):
            self._arena = {}
        if key not in self._arena:
            from .. import libffcv as L
            t = self.host_table(f_ix)
            jpg = t['mode'] == 0
            self._arena[key] = L.arena_for(t['height'][jpg], t['width'][jpg], t['size'][jpg], max_batch) \
                if jpg.any() else 4096
        return self._arena[key]

    def entropy_index(self, f_ix):
        """Zeroed (N, 64, 3) uint32 records of field f_ix shared by every
        slot's decoder (ffcv_jpeg_set_entropy_index), or None."""
        if not self.use_entropy_index or self.data is None or not self.has_mode(f_ix, 0):
            return None
        if f_ix not in self._eidx:
            from .. import libffcv as L
            n = len(self.host_table(f_ix))
            self._eidx[f_ix] = ch.zeros((n, L.EIDX_LANES, L.EIDX_WORDS), dtype=ch.int32,
                                        device=self.device)
            ch.cuda.synchronize(self.device)  # zeroed before any slot stream reads it
        return self._eidx[f_ix]

    def has_mode(self, f_ix, mode):
        self.table(f_ix)
        return self._modes[f_ix][1 if mode == 1 else 0]

    def limits(self, f_ix):
        self.table(f_ix)
        return self._limits[f_ix]


class BatchContext:
    """storage_state for one batch slot."""

    def __init__(self, host_state, dataset: DeviceDataset, loader_seed, slot, batch_size):
        self.host_state = host_state
        self.dataset = dataset
        self.loader_seed = loader_seed
        self.slot = slot
        self.batch_size = batch_size
        self.epoch = 0
        self.stream = None
        self.batch_ids = None      # device int64[B]
        self.batch_indices = None  # host np array
        self._ids_buf = None
        self._ids_host = None
        self._decoders = {}
        self.pending_status = []
        self._h2d_done = None
        self._staging = {}
        self._staged_data = None
        self._status_host = {}

    # reference-compatible tuple access for host memory_read
    def __getitem__(self, i):
        return self.host_state[i]

    def __len__(self):
        return len(self.host_state)

    @property
    def data(self):
        if self.dataset.data is not None:
            return self.dataset.data
        return self._staged_data

    def begin_batch(self, batch_indices, epoch, stream):
        self.epoch = epoch
        self.stream = stream
        self.batch_indices = batch_indices
        self.pending_status = []
        if self.dataset is not None and self.dataset.device.type == 'cuda':
            B = len(batch_indices)
            from .. import libffcv as L
            if self._ids_buf is None:
                self._ids_buf = ch.empty(self.batch_size, dtype=ch.int64, device=self.dataset.device)
                self._ids_host = ch.empty(self.batch_size, dtype=ch.int64).pin_memory()
                self._ids_host_np = self._ids_host.numpy()
            self._wait_host_buffers()
            # host-side cost per batch matters here (the Loader's producer
            # thread runs close to the kernels' rate): a numpy fill of the
            # pinned ids and one library hipMemcpyAsync on the slot stream
            self._ids_host_np[:B] = batch_indices
            L.memcpy_h2d_async(self._ids_buf, self._ids_host, B * 8, stream)
            self.batch_ids = self._ids_buf[:B]

    def _wait_host_buffers(self):
        # pinned buffers of this slot are rewritten only after the copies that
        # read them (previous batch in this slot) have completed
        if self._h2d_done is not None:
            self._h2d_done.synchronize()
            self._h2d_done = None

    def end_batch(self, done_event=None):
        """``done_event``: an event already recorded on the slot stream after
        all of this batch's work (the status event), reused instead of a new one."""
        if self.stream is not None:
            if done_event is None:
                done_event = ch.cuda.Event()
                done_event.record(self.stream)
            self._h2d_done = done_event

    def status_host(self, i, like):
        buf = self._status_host.get(i)
        if buf is None or buf.numel() < like.numel():
            buf = ch.empty(self.batch_size, dtype=like.dtype).pin_memory()
            self._status_host[i] = buf
        return buf[:like.numel()].view(like.shape)

    def sample_table(self, f_ix):
        return self.dataset.table(f_ix)

    def batch_samples(self, f_ix, buf):
        """Gather this batch's ffcv_sample descriptors into buf (device)."""
        from .. import libffcv as L
        B = len(self.batch_indices)
        if self.dataset.data is not None:
            L.gather_samples(self.dataset.table(f_ix).view(-1, 32), self.batch_ids, buf[:B], self.stream)
            return buf[:B]
        return self._stage(f_ix, buf)

    def _stage(self, f_ix, buf):
        """PCIe path: gather this batch's compressed bytes from the mmap into
        pinned memory, copy them and their descriptors to the device."""
        from .. import libffcv as L
        idx = np.asarray(self.batch_indices, dtype=np.int64)
        B = len(idx)
        table = self.dataset.host_table(f_ix)[idx]
        sizes = table['size'].astype(np.int64)
        aligned = (sizes + 15) // 16 * 16
        offs = np.zeros(B, np.int64)
        offs[1:] = np.cumsum(aligned)[:-1]
        total = int(aligned.sum()) + 64
        st = self._staging.get(f_ix)
        if st is None or st[0].numel() < total:
            cap = max(total, int(self.dataset.limits(f_ix)[2] + 16) * self.batch_size + 64)
            st = (ch.empty(cap, dtype=ch.uint8).pin_memory(),
                  ch.empty(cap, dtype=ch.uint8, device=self.dataset.device),
                  ch.empty(self.batch_size * 32, dtype=ch.uint8).pin_memory())
            self._staging[f_ix] = st
        host, dev, desc_host = st
        # native multi-threaded gather out of the mmap, or out of the process
        # cache's page slots (os_cache=False), with ffcv_host_gather
        from ..memory_managers.process_cache import host_source
        src, src_off = host_source(self.host_state,
                                   table['offset'].astype(np.uint64) + np.uint64(self.dataset.data_base))
        L.host_gather(src, src_off, sizes, offs, host, nthreads=min(8, max(1, B // 32)))
        t = table.copy()
        t['offset'] = offs.astype(np.uint64)
        desc_host[:B * 32].copy_(ch.from_numpy(t.view(np.uint8)))
        dev[:total].copy_(host[:total], non_blocking=True)
        buf[:B].view(-1).copy_(desc_host[:B * 32], non_blocking=True)
        self._staged_data = dev
        return buf[:B]

    def any_mode(self, f_ix, mode):
        return self.dataset.has_mode(f_ix, mode)

    def jpeg_decoder(self, f_ix):
        if f_ix not in self._decoders:
            from .. import libffcv as L
            h, w, nbytes = self.dataset.limits(f_ix)
            dec = L.JpegDecoder(self.batch_size, h, w, nbytes,
                                self.dataset.arena_bytes(f_ix, self.batch_size))
            eidx = self.dataset.entropy_index(f_ix)
            if eidx is not None:
                dec.set_entropy_index(eidx)
            self._decoders[f_ix] = dec
        return self._decoders[f_ix]

    def raw_workspace(self, f_ix, out_h, out_w):
        """Device workspace of this slot for the raw decoder's per-image plans
        and tap tables (ffcv_rrc_raw_batch_ws), one per (field, output size)."""
        from .. import libffcv as L
        key = ('raw_ws', f_ix, out_h, out_w)
        ws = self._staging.get(key)
        if ws is None:
            ws = ch.empty(L.rrc_raw_workspace_bytes(self.batch_size, out_h, out_w), dtype=ch.uint8,
                          device=self.dataset.device)
            self._staging[key] = ws
        return ws

    def check_status(self, status, what):
        self.pending_status.append((status, what))
