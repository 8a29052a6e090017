"""Cutout (ffcv/transforms/cutout.py:13-52).

Fused into the crop/resize kernel when it directly follows a
RandomResizedCrop/CenterCrop decoder (the graph lowering does this);
otherwise runs as its own device kernel, or on host numpy arrays.  The
square origin is ``(randint(H-c+1), randint(W-c+1))`` drawn from the
sample's own MT19937 (op id 2) under the seeding contract.
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


class Cutout(Operation):
    """Cutout data augmentation (https://arxiv.org/abs/1708.04552).

    Parameters
    ----------
    crop_size : int
        Size of the random square to cut out.
    fill : Tuple[int, int, int], optional
        An RGB color ((0, 0, 0) by default) to fill the cutout square with.
    """
    device_aware = True
    per_sample = True

    def __init__(self, crop_size: int, fill: Tuple[int, int, int] = (0, 0, 0)):
        super().__init__()
        self.crop_size = crop_size
        self.fill = np.array(fill)
        self._absorbed = False

    def generate_code(self) -> Callable:
        if self._absorbed:
            def fused(images, *_):
                return images
            return fused
        crop_size = int(self.crop_size)
        fill = np.broadcast_to(np.asarray(self.fill).astype(np.uint8).reshape(-1), (3,)).copy()

        def cutout_square(images, dst, indices):
            ctx = runtime.current()
            if isinstance(images, ch.Tensor) and images.device.type == 'cuda':
                from .. import libffcv as L
                B = images.shape[0]
                yx = ch.empty((B, 2), dtype=ch.int32, device=images.device)
                p = L.DrawParams()
                p.out_h, p.out_w = int(images.shape[1]), int(images.shape[2])
                p.cutout_size = crop_size
                p.loader_seed, p.epoch = int(ctx.loader_seed), int(ctx.epoch)
                L.draw_batch(ctx.batch_ids, None, p, None, yx, None, None, ctx.stream)
                L.cutout_batch(images, yx, crop_size, fill, ctx.stream)
                return images
            seed, epoch = (ctx.loader_seed, ctx.epoch) if ctx else (0, 0)
            for i, sid in enumerate(indices):
                rs = np.random.RandomState(contract_seed(seed, epoch, int(sid), 2))
                y = rs.randint(images.shape[1] - crop_size + 1)
                x = rs.randint(images.shape[2] - crop_size + 1)
                images[i, y:y + crop_size, x:x + crop_size] = fill
            return images
        cutout_square.is_parallel = True
        cutout_square.with_indices = True
        return cutout_square

    def declare_state_and_memory(self, previous_state: State) -> Tuple[State, Optional[AllocationQuery]]:
        return replace(previous_state, jit_mode=previous_state.device.type == 'cpu'
                       and not isinstance(previous_state.dtype, ch.dtype)), None
