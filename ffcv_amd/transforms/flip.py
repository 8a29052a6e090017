"""RandomHorizontalFlip (ffcv/transforms/flip.py:12-46).

Flip decision per sample: one double from the sample's MT19937 (op id 3)
``< flip_prob`` (the reference draws ``rand(B) < flip_prob`` for the batch,
flip.py:35).  Fused into the crop/resize kernel when it follows the
decoder; otherwise a device kernel or host numpy.
"""
from dataclasses import replace
from typing import Callable, Optional, Tuple

import numpy as np
import torch as ch

from ..pipeline.allocation_query import AllocationQuery
from ..pipeline.operation import Operation
from ..pipeline.state import State
from ..pipeline import runtime
from .rng import contract_seed


class RandomHorizontalFlip(Operation):
    """Flip the image horizontally with probability flip_prob.

    Parameters
    ----------
    flip_prob : float
        The probability with which to flip each image in the batch horizontally.
    """
    device_aware = True
    per_sample = True

    def __init__(self, flip_prob: float = 0.5):
        super().__init__()
        self.flip_prob = flip_prob
        self._absorbed = False

    def generate_code(self) -> Callable:
        if self._absorbed:
            def fused(images, dst, *_):
                return images
            return fused
        flip_prob = float(self.flip_prob)

        def flip(images, dst, indices):
            ctx = runtime.current()
            if isinstance(images, ch.Tensor) and images.device.type == 'cuda':
                from .. import libffcv as L
                B = images.shape[0]
                flips = ch.empty(B, dtype=ch.uint8, device=images.device)
                p = L.DrawParams()
                p.flip_prob = flip_prob
                p.loader_seed, p.epoch = int(ctx.loader_seed), int(ctx.epoch)
                L.draw_batch(ctx.batch_ids, None, p, None, None, flips, None, ctx.stream)
                out = dst[:B]
                L.flip_batch(images, out, flips, ctx.stream)
                return out
            seed, epoch = (ctx.loader_seed, ctx.epoch) if ctx else (0, 0)
            for i, sid in enumerate(indices):
                u = np.random.RandomState(contract_seed(seed, epoch, int(sid), 3)).uniform(0, 1)
                dst[i] = images[i, :, ::-1] if u < flip_prob else images[i]
            return dst[:len(indices)]
        flip.is_parallel = True
        flip.with_indices = True
        return flip

    def declare_state_and_memory(self, previous_state: State) -> Tuple[State, Optional[AllocationQuery]]:
        if self._absorbed:
            return previous_state, None
        on_dev = previous_state.device.type == 'cuda'
        return (replace(previous_state, jit_mode=not on_dev and not isinstance(previous_state.dtype, ch.dtype)),
                AllocationQuery(previous_state.shape, previous_state.dtype,
                                previous_state.device if on_dev else None))
