"""Memory declarations (ffcv/pipeline/allocation_query.py:8-41).

``AllocationQuery(shape, dtype, device)`` is allocated as ``[slots, batch,
*shape]``: host queries become one pinned buffer viewed as numpy (numpy
dtype) or a list of pinned tensors (torch dtype); device queries become one
tensor per slot on that device (HBM), exactly like the reference.
"""
from dataclasses import dataclass
from typing import Optional, Sequence, Tuple, Union

import numpy as np
import torch as ch


@dataclass(frozen=True)
class AllocationQuery:
    shape: Tuple[int, ...]
    dtype: Union[np.dtype, ch.dtype]
    device: Optional[ch.device] = None


Allocation = Union[AllocationQuery, Sequence[AllocationQuery]]


def _torch_dtype(dtype):
    if isinstance(dtype, ch.dtype):
        return dtype
    return ch.from_numpy(np.empty(0, dtype=dtype)).dtype


def allocate_query(memory_allocation: AllocationQuery, batch_size: int, batches_ahead: int):
    final_shape = [batches_ahead, batch_size, *[int(x) for x in memory_allocation.shape]]
    device = memory_allocation.device
    if device is not None and ch.device(device).type != 'cpu':
        return [ch.empty(*final_shape[1:], dtype=_torch_dtype(memory_allocation.dtype), device=device)
                for _ in range(final_shape[0])]
    if isinstance(memory_allocation.dtype, ch.dtype):
        result = []
        for _ in range(final_shape[0]):
            partial = ch.empty(*final_shape[1:], dtype=memory_allocation.dtype)
            if ch.cuda.is_available():
                partial = partial.pin_memory()
            result.append(partial)
        return result
    result = ch.empty(*final_shape, dtype=_torch_dtype(memory_allocation.dtype))
    if ch.cuda.is_available():
        result = result.pin_memory()
    return result.numpy()
