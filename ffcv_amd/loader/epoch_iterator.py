"""Epoch iterator (ffcv/loader/epoch_iterator.py:33-175).

Same contract as the reference: a background thread builds batches ahead of
the training loop into a ring of buffers, each ring entry owning a HIP
stream; a bounded queue hands them to the consumer, whose ``__next__`` makes
the current stream wait on the batch's stream; an event recorded on the
consumer stream keeps a buffer from being overwritten while still in use.

What changed for MI355X:

* The stages enqueue HIP kernels instead of running numba loops, so the
  thread only orchestrates.
* **Launch groups.**  One batch of JPEG decode is 128 entropy workgroups,
  an eighth of what the GPU holds; the reference's one-batch-per-stream ring
  therefore needed 10 concurrent streams (and a raised GPU_MAX_HW_QUEUES) to
  fill the chip.  When every operation of the graph is ``per_sample`` (the
  north-star pipeline is), ``G`` consecutive batches run through the graph
  as ONE launch sequence of ``G * batch_size`` samples into one buffer set,
  and the consumer receives them one batch at a time (views of that set).
  Three sets rotate (two launches in flight while the consumer reads the
  third), on three streams, which HIP's default 4 hardware queues hold.
  Graphs with batch-level operations (mixup, user ops) keep G = 1.
* Buffer sets are released by the consumer: ``__next__`` records an event on
  the consumer stream once the previous set's last batch has been handed
  out; the producer waits (host side) for that release before re-using a
  set, and the set's stream waits (device side) on the event.
* Per-sample decode status is copied back asynchronously and checked before
  the set is reused and at the end of the epoch (a corrupt or unsupported
  JPEG raises DecodeError; the reference silently returns garbage,
  rgb_image.py:131,196).
"""
import os
import threading
import time
from queue import Queue, Full, Empty

import numpy as np
import torch as ch

from ..pipeline import runtime
from ..pipeline.compiler import Compiler
from ..utils import chunks

# samples per decode launch (bench.py GROUP: 24 x 512 measured best at 400
# steps; launches of 6,144 lost ~5% to per-launch tails)
TARGET_LAUNCH_SAMPLES = 12288
MAX_GROUP = 32
N_SETS = 3


class DecodeError(RuntimeError):
    pass


_HW_QUEUES = None


def hw_queues():
    """Hardware queues HIP gives this process: GPU_MAX_HW_QUEUES (HIP's
    default 4 when unset), read ONCE.  HIP reads the variable when its
    runtime initialises and never again; the first call here comes from an
    EpochIterator, after the Loader has initialised the device
    (``torch.cuda.set_device``), so the cached value is the one in force
    then, and a later change of the environment (which the runtime ignores)
    does not change the stream count either."""
    global _HW_QUEUES
    if _HW_QUEUES is None:
        try:
            _HW_QUEUES = max(1, int(os.environ.get('GPU_MAX_HW_QUEUES', '4')))
        except ValueError:
            _HW_QUEUES = 4
    return _HW_QUEUES


def max_streams():
    """Producer streams: one hardware queue stays free for the consumer's."""
    return max(1, hw_queues() - 1)


def launch_group(loader, n_batches):
    """Batches per launch for this loader (1 when the graph mixes samples)."""
    if loader.batches_per_launch is not None:
        g = int(loader.batches_per_launch)
    elif loader.device.type != 'cuda' or not loader.graph.groupable():
        g = 1
    else:
        g = -(-TARGET_LAUNCH_SAMPLES // loader.batch_size)
    return max(1, min(g, MAX_GROUP, max(1, n_batches)))


class EpochIterator(threading.Thread):
    def __init__(self, loader, order):
        super().__init__(daemon=True)
        self.loader = loader
        self.order = order
        self.metadata = loader.reader.metadata
        self.device = loader.device
        self.is_cuda = self.device.type == 'cuda'
        self.epoch = loader.next_epoch - 1
        self.error = None
        self.closed = False
        self.terminate_event = threading.Event()
        bs = loader.batch_size
        batches = list(chunks(order, bs))
        self.G = launch_group(loader, len(batches))
        # groups of G consecutive batches; the last group may be shorter and
        # its last batch partial (drop_last=False)
        self.groups = [batches[i:i + self.G] for i in range(0, len(batches), self.G)]
        self.output_queue = Queue(max(1, loader.batches_ahead))
        # the page scheduler (os_cache=False) sees one launch as one "batch"
        self.memory_context = loader.memory_manager.schedule_epoch(
            [np.concatenate(g) if len(g) else np.zeros(0, np.uint64) for g in self.groups])
        self.memory_context.__enter__()
        self.storage_state = self.memory_context.state
        if self.is_cuda:
            self.current_stream = ch.cuda.current_stream(self.device)
        self.n_sets = N_SETS if self.G > 1 else max(N_SETS, loader.batches_ahead + 2)
        self._bind_sets()
        # set release bookkeeping (consumer -> producer)
        self._cv = threading.Condition()
        self._released = [True] * self.n_sets      # set may be (re)filled
        self._release_event = [None] * self.n_sets  # consumer-stream event to wait on
        # [set, batches still to hand out before it is released]: the set of a
        # batch the consumer got is released when it asks for the hold-th
        # batch after it, so a batch the training loop keeps (logging,
        # lookahead) stays intact while it takes batches_ahead more, as with
        # the reference's ring.  Bound: the producer hands out launch m + 2's
        # batches only after it has re-acquired launch m's set for m + 3, so
        # the consumer can take (n_sets - 2) * G batches past a set before it
        # must have released it
        self._pending_release = []
        self._hold = max(1, min(loader.batches_ahead + 1, (self.n_sets - 2) * self.G + 1))
        self._status = [None] * self.n_sets
        self._t_pipeline = 0.0
        self.start()

    # -------------------------------------------------------------- buffers --
    def _bind_sets(self):
        """Per-set device buffers, batch contexts and streams, cached on the
        loader across epochs while the graph's allocations and the launch
        shape stay the same (the reference re-allocates every epoch,
        epoch_iterator.py:65; a resolution change between epochs therefore
        gets new buffers here too)."""
        loader = self.loader
        graph = loader.graph
        graph.collect_requirements()  # per epoch, like graph.py:356-358
        cap = self.G * loader.batch_size
        key = (self.n_sets, cap, graph.allocation_signature())
        cache = getattr(loader, '_slot_cache', None)
        if cache is None or cache['key'] != key:
            if cache is not None and self.is_cuda:
                ch.cuda.synchronize(self.device)  # old buffers may still be read
            n_streams = min(self.n_sets, max_streams())
            streams = [(ch.cuda.Stream(self.device) if self.is_cuda else None) for _ in range(n_streams)]
            cache = {'key': key,
                     'streams': [streams[s % n_streams] for s in range(self.n_sets)],
                     'memory': graph.allocate_memory(cap, self.n_sets),
                     'contexts': [runtime.BatchContext(None, loader.device_dataset, loader.seed, s, cap)
                                  for s in range(self.n_sets)]}
            loader._slot_cache = cache
        else:
            # same buffers, new node ids (recompile / per-epoch requirements)
            cache['memory'] = graph.rebind_memory(cache['memory'])
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

    # ------------------------------------------------------------- thread --
    def run(self):
        try:
            Compiler.set_num_threads(self.loader.num_workers)
            prev = None
            for m, group in enumerate(self.groups):
                s = m % self.n_sets
                if not self._acquire(s):
                    return
                t0 = time.perf_counter()
                results = self.run_pipeline(m, group, s)
                self._t_pipeline += time.perf_counter() - t0
                # hand out the previous launch while this one runs on the GPU
                if prev is not None and not self._put_group(*prev):
                    return
                prev = (s, group, results)
            if prev is not None and not self._put_group(*prev):
                return
            if os.environ.get('FFCV_LOADER_TIMING'):
                nb = sum(len(g) for g in self.groups)
                print(f'# epoch {self.epoch}: {nb} batches in {len(self.groups)} launches of <= {self.G}, '
                      f'host enqueue {self._t_pipeline * 1e3 / max(1, nb):.3f} ms/batch', flush=True)
            self._put(None)
        except BaseException as e:  # surface worker errors to the consumer
            self.error = e
            self._put(None, force=True)

    def _acquire(self, s):
        """Wait until the consumer released set s (host side)."""
        with self._cv:
            while not self._released[s]:
                if self.terminate_event.is_set():
                    return False
                self._cv.wait(0.1)
            self._released[s] = False
            return not self.terminate_event.is_set()

    def _put(self, item, force=False):
        while True:
            try:
                self.output_queue.put(item, block=True, timeout=0.5)
                return True
            except Full:
                if self.terminate_event.is_set():
                    if force:
                        try:
                            self.output_queue.get_nowait()
                        except Empty:
                            pass
                        continue
                    return False

    def _put_group(self, s, group, results):
        bs = self.loader.batch_size
        n = len(group)
        for j, batch in enumerate(group):
            lo, hi = j * bs, j * bs + len(batch)
            res = tuple(r[lo:hi] for r in results) if n > 1 else results
            if not self._put((s, res, j == n - 1)):
                return False
        return True

    def run_pipeline(self, m, group, s):
        self.memory_context.start_batch(m)
        ctx = self.contexts[s]
        self._check_status(s)
        indices = np.concatenate(group) if len(group) > 1 else group[0]
        if self.is_cuda:
            stream = self.cuda_streams[s]
            with ch.cuda.stream(stream):
                ev = self._release_event[s]
                if ev is not None:
                    stream.wait_event(ev)
                runtime.set_current(ctx)
                ctx.begin_batch(indices, self.epoch, stream)
                result = self.loader.graph.run(indices, ctx, self.memory_allocations, s)
                ctx.end_batch(self._queue_status(s, ctx, stream))
        else:
            runtime.set_current(ctx)
            ctx.begin_batch(indices, self.epoch, None)
            result = self.loader.graph.run(indices, ctx, self.memory_allocations, s)
        runtime.set_current(None)
        return result

    # ------------------------------------------------- decode status check --
    def _queue_status(self, s, ctx, stream):
        """Copy this launch's per-sample status words to pinned host memory
        and record an event after them; returns that event (None if no
        status is pending)."""
        if not ctx.pending_status:
            self._status[s] = None
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
        self._status[s] = (ev, recs, np.asarray(ctx.batch_indices).copy())
        return ev

    def _check_status(self, s):
        rec = self._status[s]
        if rec is None:
            return
        ev, recs, ids = rec
        ev.synchronize()
        self._status[s] = None
        from ..libffcv import SAMPLE_STATUS
        for host, what in recs:
            st = host.numpy().reshape(-1)
            bad = np.nonzero(st)[0]
            if bad.size:
                k = int(bad[0])
                code = int(st[k])
                msg = (f'{what}: sample {int(ids[k])} failed to decode: '
                       f'{SAMPLE_STATUS.get(code, code)} ({bad.size} bad in launch)')
                self.error = DecodeError(msg)

    # ----------------------------------------------------------- consumer --
    def _release_pending(self):
        """One more batch is being handed out: release every set whose hold
        ran out (the consumer is done enqueueing work on it)."""
        if not self._pending_release:
            return
        for p in self._pending_release:
            p[1] -= 1
        due = [p[0] for p in self._pending_release if p[1] <= 0]
        if not due:
            return
        self._pending_release = [p for p in self._pending_release if p[1] > 0]
        ev = None
        if self.is_cuda:
            ev = ch.cuda.Event()
            ev.record(self.current_stream)
        with self._cv:
            for s in due:
                self._release_event[s] = ev
                self._released[s] = True
            self._cv.notify_all()

    def __next__(self):
        self._release_pending()
        item = self.output_queue.get()
        if item is None:
            self.join()
            if self.is_cuda and self.error is None:
                for s in range(self.n_sets):
                    self._check_status(s)
            self.close()
            if self.error is not None:
                raise self.error
            raise StopIteration()
        s, result, last = item
        if self.is_cuda:
            self.current_stream.wait_stream(self.cuda_streams[s])
        if last:
            self._pending_release.append([s, self._hold])
        if self.error is not None:
            self.close()
            raise self.error
        return result

    def __iter__(self):
        return self

    def close(self):
        """Stop the producer (also for an iterator abandoned mid-epoch) and
        release the memory manager's epoch context."""
        self.terminate_event.set()
        with self._cv:
            self._cv.notify_all()
        if self.is_alive() and threading.current_thread() is not self:
            self.join()
        if not self.closed:
            self.closed = True
            self.memory_context.__exit__(None, None, None)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
