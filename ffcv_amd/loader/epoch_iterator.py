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
from queue import Queue, Full
from threading import Thread, Event

import numpy as np
import torch as ch

from ..pipeline import runtime
from ..pipeline.compiler import Compiler
from ..utils import chunks


class DecodeError(RuntimeError):
    pass


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
        n_slots = self.loader.batches_ahead + 2
        self.cuda_streams = [(ch.cuda.Stream(self.device) if self.is_cuda else None)
                             for _ in range(n_slots)]
        self.memory_allocations = self.loader.graph.allocate_memory(self.loader.batch_size, n_slots)
        self.contexts = [runtime.BatchContext(self.storage_state, loader.device_dataset, loader.seed,
                                              s, loader.batch_size) for s in range(n_slots)]
        self._status = [None] * n_slots
        self.start()

    # ------------------------------------------------------------- thread --
    def run(self):
        events = [None for _ in self.cuda_streams]
        try:
            b_ix = 0
            Compiler.set_num_threads(self.loader.num_workers)
            while True:
                ixes = next(self.iter_ixes)
                slot = self.current_batch_slot
                self.current_batch_slot = (slot + 1) % (self.loader.batches_ahead + 2)
                result = self.run_pipeline(b_ix, ixes, slot, events[slot])
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
                    just_finished_slot = (slot - self.loader.batches_ahead - 1) % (self.loader.batches_ahead + 2)
                    event = ch.cuda.Event()
                    event.record(self.current_stream)
                    events[just_finished_slot] = event
                b_ix += 1
        except StopIteration:
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
                self._queue_status(batch_slot, ctx, stream)
                ctx.end_batch()
        else:
            runtime.set_current(ctx)
            ctx.begin_batch(batch_indices, self.epoch, None)
            result = self.loader.graph.run(batch_indices, ctx, self.memory_allocations, batch_slot)
        runtime.set_current(None)
        return result

    # ------------------------------------------------- decode status check --
    def _queue_status(self, slot, ctx, stream):
        if not ctx.pending_status:
            self._status[slot] = None
            return
        recs = []
        for i, (status, what) in enumerate(ctx.pending_status):
            host = ctx.status_host(i, status)
            host.copy_(status, non_blocking=True)
            recs.append((host, what))
        ev = ch.cuda.Event()
        ev.record(stream)
        self._status[slot] = (ev, recs, np.asarray(ctx.batch_indices).copy())

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
