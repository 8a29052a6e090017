"""NormalizeImage (ffcv/transforms/normalize.py:21-138).

The 256x3 lookup table is built exactly as the reference builds it
(float64 arithmetic, cast to the target dtype; float16 carried as int16
bits), so the device output is bit-identical to the reference LUT.  When it
follows a crop/resize decoder (possibly through Cutout / flip / ToTensor /
ToDevice / ToTorchImage) the graph fuses the LUT into the resize kernel's
store; otherwise a standalone device kernel (normalize.py:65 cupy kernel
``output = table[input * 3 + i % 3]``) or host numpy.
"""
from dataclasses import replace
from typing import Callable, Optional, Tuple

import numpy as np
import torch as ch

from ..pipeline.allocation_query import AllocationQuery
from ..pipeline.operation import Operation
from ..pipeline.state import State
from ..pipeline import runtime
from .lut import make_lut


def ch_dtype_from_numpy(dtype):
    return ch.from_numpy(np.zeros((), dtype=dtype)).dtype


class NormalizeImage(Operation):
    """Normalization + type conversion of uint8 images (GPU or CPU tensors).

    Parameters
    ----------
    mean: np.ndarray
        The mean vector.
    std: np.ndarray
        The standard deviation vector.
    type: np.dtype
        The desired output type (numpy dtype).
    """
    device_aware = True
    per_sample = True

    def __init__(self, mean: np.ndarray, std: np.ndarray, type: np.dtype):
        super().__init__()
        table = make_lut(mean, std, type)
        self.original_dtype = type
        if type == np.float16:
            type = np.int16
        self.dtype = type
        self.lookup_table = table.view(type)
        self.previous_shape = None
        self.mode = 'cpu'
        self._absorbed = False
        self._dev_luts = {}

    def device_lut(self, device):
        key = str(device)
        if key not in self._dev_luts:
            self._dev_luts[key] = ch.from_numpy(np.ascontiguousarray(self.lookup_table)).to(device)
        return self._dev_luts[key]

    def generate_code(self) -> Callable:
        if self._absorbed:
            def fused(images, *_):
                return images
            return fused
        if self.mode == 'cpu':
            return self.generate_code_cpu()
        return self.generate_code_gpu()

    def generate_code_gpu(self) -> Callable:
        # any table dtype, like the reference's templated cupy kernel
        # (normalize.py:64-65): the kernel gathers element bit patterns
        final_type = ch_dtype_from_numpy(self.original_dtype)

        def normalize_convert(images, result):
            from .. import libffcv as L
            ctx = runtime.current()
            B, C, H, W = images.shape
            assert images.is_contiguous(memory_format=ch.channels_last), 'Images need to be in channel last'
            result = result[:B]
            flat = images.permute(0, 2, 3, 1)
            L.lut_batch(flat, self.device_lut(images.device), result, ctx.stream if ctx else None)
            final_result = result.reshape(B, H, W, C).permute(0, 3, 1, 2)
            return final_result.view(final_type)
        return normalize_convert

    def generate_code_cpu(self) -> Callable:
        table = self.lookup_table.view(dtype=self.dtype)

        def normalize_convert(images, result, indices):
            n = len(indices)
            imgs = images[:n].reshape(n, -1, 3)
            out = result[:n].reshape(n, -1, 3)
            for c in range(3):
                out[:, :, c] = table[imgs[:, :, c], c]
            return result[:n]
        normalize_convert.is_parallel = True
        normalize_convert.with_indices = True
        return normalize_convert

    def declare_state_and_memory(self, previous_state: State) -> Tuple[State, Optional[AllocationQuery]]:
        if self._absorbed:
            return replace(previous_state, dtype=ch_dtype_from_numpy(self.original_dtype)), None
        if previous_state.device == ch.device('cpu'):
            new_state = replace(previous_state, jit_mode=True, dtype=self.dtype)
            return new_state, AllocationQuery(shape=previous_state.shape, dtype=self.dtype,
                                              device=previous_state.device)
        self.mode = 'gpu'
        new_state = replace(previous_state, dtype=self.dtype)
        gpu_type = ch_dtype_from_numpy(self.dtype)
        return new_state, AllocationQuery(shape=previous_state.shape, device=previous_state.device,
                                          dtype=gpu_type)
