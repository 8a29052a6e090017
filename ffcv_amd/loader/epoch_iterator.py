"""Epoch iterator (ffcv/loader/epoch_iterator.py:33-175).

Same structure as the reference: a background thread builds batches into a
ring of ``batches_ahead + 2`` slots, each slot owning a HIP stream; a
bounded queue hands (slot, result) to the consumer, whose ``__next__``
makes the current stream wait on the slot's stream; an event recorded on the
consumer stream keeps a slot from being overwritten while still in use.

What changed: the stages enqueue HIP kernels on the slot's stream instead of
running numba loops, so the thread only orchestrates; per-sample decode
status codes are copied back asynchronously and checked without stalling
the pipeline (a corrupt or unsupported JPEG raises FFCVError; the reference
silently returns garbage, rgb_image.py:131,196).
"""
import os
import time
from queue import Queue, Full
from threading import Thread, Event

import numpy as np
import torch as ch

from ..pipeline import runtime
from ..pipeline.compiler import Compiler
from ..utils import chunks


class DecodeError(RuntimeError):
    pass


def max_streams():
    """Slot streams the Loader may use: one hardware queue stays free for the
    consumer's stream.  10 concurrent batches measured fastest on 16 queues
    (device_cache Loader 1.92 M vs 1.73 M images/s at 8; bench.py C3 likewise)."""
    try:
        hwq = int(os.environ.get('GPU_MAX_HW_QUEUES', '4'))
        cap = int(os.environ.get('FFCV_LOADER_STREAMS', '10'))  # diagnostic override
    except ValueError:
        hwq, cap = 4, 10
    return max(1, min(cap, hwq - 1))


class EpochIterator(Thread):
    def __init__(self, loader, order):
        super().__init__(daemon=True)
        self.loader = loader
        self.order = order
        self.metadata = loader.reader.metadata
        self.current_batch_slot = 0
        batches = list(chunks(order, self.loader.batch_size))
        self.iter_ixes = iter(batches)
        self.closed = False
        self.output_queue = Queue(self.loader.batches_ahead)
        self.terminate_event = Event()
        self.memory_context = self.loader.memory_manager.schedule_epoch(batches)
        self.epoch = loader.next_epoch - 1
        self.error = None
        self.device = loader.device
        self.is_cuda = self.device.type == 'cuda'
        if self.is_cuda:
            self.current_stream = ch.cuda.current_stream(self.device)
        try:
            self.memory_context.__enter__()
        except MemoryError as e:
            raise e
        self.storage_state = self.memory_context.state
        # decode slots: at least batches_ahead + 2 (the reference's ring), and
        # at least max_streams() so that many batches can be decoding at once
        # (8 in flight measured fastest on MI355X); batches_ahead still bounds
        # how far the producer runs ahead of the consumer (the output queue)
        n_slots = max(self.loader.batches_ahead + 2, max_streams() if self.is_cuda else 0)
        self.n_slots = n_slots
        # Slot state lives on the loader across epochs: the device buffers and
        # the JPEG decoder scratch (hundreds of MB per slot) are allocated
        # once, not per epoch.  The slots share at most max_streams() HIP
        # streams (slot % n; two slots on one stream are simply ordered), so
        # the slot streams plus the consumer's fit the GPU's hardware queues
        # (GPU_MAX_HW_QUEUES, raised to 16 by ffcv_amd/__init__.py).
        key = (n_slots, self.loader.batch_size)
        cache = getattr(loader, '_slot_cache', None)
        if cache is None or cache['key'] != key:
            streams = [(ch.cuda.Stream(self.device) if self.is_cuda else None)
                       for _ in range(min(n_slots, max_streams()))]
            cache = {'key': key,
                     'streams': [streams[s % len(streams)] for s in range(n_slots)],
                     'memory': self.loader.graph.allocate_memory(self.loader.batch_size, n_slots),
                     'contexts': [runtime.BatchContext(None, loader.device_dataset, loader.seed, s,
                                                       loader.batch_size) for s in range(n_slots)]}
            loader._slot_cache = cache
        self.cuda_streams = cache['streams']
        self.memory_allocations = cache['memory']
        self.contexts = cache['contexts']
        for c in self.contexts:
            c.host_state = self.storage_state
            c.loader_seed = loader.seed
        if self.is_cuda:  # reused buffers: order this epoch after the consumer's queued work
            ev = ch.cuda.Event()
            ev.record(self.current_stream)
            for st in set(self.cuda_streams):
                st.wait_event(ev)
        self._status = [None] * n_slots
        self._t_pipeline = 0.0  # host seconds spent enqueueing batches (FFCV_LOADER_TIMING=1 prints it)
        self.start()

    # ------------------------------------------------------------- thread --
    def run(self):
        if os.environ.get('FFCV_LOADER_PROFILE'):  # diagnostics: cProfile of the producer thread
            import cProfile
            import pstats
            prof = cProfile.Profile()
            prof.enable()
            try:
                self._run()
            finally:
                prof.disable()
                pstats.Stats(prof).sort_stats('tottime').print_stats(25)
            return
        self._run()

    def _run(self):
        events = [None for _ in self.cuda_streams]
        try:
            b_ix = 0
            Compiler.set_num_threads(self.loader.num_workers)
            while True:
                ixes = next(self.iter_ixes)
                slot = self.current_batch_slot
                self.current_batch_slot = (slot + 1) % self.n_slots
                t0 = time.perf_counter()
                result = self.run_pipeline(b_ix, ixes, slot, events[slot])
                self._t_pipeline += time.perf_counter() - t0
                to_output = (slot, result)
                while True:
                    try:
                        self.output_queue.put(to_output, block=True, timeout=0.5)
                        break
                    except Full:
                        pass
                    if self.terminate_event.is_set():
                        return
                if self.is_cuda:
                    just_finished_slot = (slot - self.loader.batches_ahead - 1) % self.n_slots
                    event = ch.cuda.Event()
                    event.record(self.current_stream)
                    events[just_finished_slot] = event
                b_ix += 1
        except StopIteration:
            if os.environ.get('FFCV_LOADER_TIMING'):
                print(f'# epoch {self.epoch}: {b_ix} batches, host enqueue {self._t_pipeline * 1e3 / max(1, b_ix):.3f} '
                      f'ms/batch', flush=True)
            self.output_queue.put(None)
        except BaseException as e:  # surface worker errors to the consumer
            self.error = e
            self.output_queue.put(None)

    def run_pipeline(self, b_ix, batch_indices, batch_slot, cuda_event):
        self.memory_context.start_batch(b_ix)
        ctx = self.contexts[batch_slot]
        self._check_status(batch_slot, wait=True)
        if self.is_cuda:
            stream = self.cuda_streams[batch_slot]
            with ch.cuda.stream(stream):
                if cuda_event:
                    cuda_event.wait()
                runtime.set_current(ctx)
                ctx.begin_batch(batch_indices, self.epoch, stream)
                result = self.loader.graph.run(batch_indices, ctx, self.memory_allocations, batch_slot)
                ctx.end_batch(self._queue_status(batch_slot, ctx, stream))
        else:
            runtime.set_current(ctx)
            ctx.begin_batch(batch_indices, self.epoch, None)
            result = self.loader.graph.run(batch_indices, ctx, self.memory_allocations, batch_slot)
        runtime.set_current(None)
        return result

    # ------------------------------------------------- decode status check --
    def _queue_status(self, slot, ctx, stream):
        """Copy this batch's per-sample status words to pinned host memory
        and record an event after them; returns that event (None if no
        status is pending)."""
        if not ctx.pending_status:
            self._status[slot] = None
            return None
        from .. import libffcv as L
        recs = []
        for i, (status, what) in enumerate(ctx.pending_status):
            host = ctx.status_host(i, status)
            if status.is_contiguous():
                L.memcpy_d2h_async(host, status, status.numel() * status.element_size(), stream)
            else:
                host.copy_(status, non_blocking=True)
            recs.append((host, what))
        ev = ch.cuda.Event()
        ev.record(stream)
        self._status[slot] = (ev, recs, np.asarray(ctx.batch_indices).copy())
        return ev

    def _check_status(self, slot, wait=False):
        rec = self._status[slot]
        if rec is None:
            return
        ev, recs, ids = rec
        if not wait and not ev.query():
            return
        ev.synchronize()
        self._status[slot] = None
        from ..libffcv import SAMPLE_STATUS
        for host, what in recs:
            st = host.numpy()
            bad = np.nonzero(st)[0]
            if bad.size:
                k = int(bad[0])
                msg = (f'{what}: sample {int(ids[k])} failed to decode: '
                       f'{SAMPLE_STATUS.get(int(st[k]), st[k])} ({bad.size} bad in batch)')
                self.error = DecodeError(msg)

    # ----------------------------------------------------------- consumer --
    def __next__(self):
        result = self.output_queue.get()
        if result is None:
            if self.is_cuda:
                for s in range(len(self._status)):
                    self._check_status(s, wait=True)
            self.close()
            if self.error is not None:
                raise self.error
            raise StopIteration()
        slot, result = result
        if self.is_cuda:
            stream = self.cuda_streams[slot]
            self.current_stream.wait_stream(stream)
        if self.error is not None:
            self.close()
            raise self.error
        return result

    def __iter__(self):
        return self

    def close(self):
        self.terminate_event.set()
        if not self.closed:
            self.closed = True
            self.memory_context.__exit__(None, None, None)

    def __del__(self):
        self.close()
