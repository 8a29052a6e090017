"""Layout / placement operations: ToTensor, ToDevice, ToTorchImage, Convert, View.

Semantics of the reference's ffcv/transforms/ops.py:17-160.  On the
device-resident path they are mostly free: the decode launch already wrote a
tensor on the Loader's device, so ToTensor / ToDevice pass it through and
ToTorchImage only re-labels the channels-last storage as NCHW.  On host data
they do what the reference does (``torch.from_numpy``, a non_blocking copy
into the slot's device buffer, an NCHW view or copy).
"""
from dataclasses import replace
from typing import Callable, Optional, Tuple

import numpy as np
import torch as ch

from ..pipeline.allocation_query import AllocationQuery
from ..pipeline.operation import Operation
from ..pipeline.state import State


def _as_torch_dtype(dtype):
    return dtype if isinstance(dtype, ch.dtype) else ch.from_numpy(np.empty((), dtype=dtype)).dtype


def _same_device(state_device, target):
    """True when data on ``state_device`` already satisfies ``ToDevice(target)``
    (an index-less 'cuda' target accepts any GPU)."""
    return state_device.type == target.type and (target.index is None or state_device == target)


class ToTensor(Operation):
    """numpy batch -> torch tensor (zero copy); tensors pass through."""
    device_aware = True
    per_sample = True

    def __init__(self):
        super().__init__()

    def generate_code(self) -> Callable:
        def to_tensor(inp, dst):
            return inp if isinstance(inp, ch.Tensor) else ch.from_numpy(inp)
        return to_tensor

    def declare_state_and_memory(self, previous_state: State) -> Tuple[State, Optional[AllocationQuery]]:
        return replace(previous_state, jit_mode=False, dtype=_as_torch_dtype(previous_state.dtype)), None


class ToDevice(Operation):
    """Move the batch to ``device`` (asynchronous when ``non_blocking``).

    Parameters
    ----------
    device: torch.device
        Device to move to.
    non_blocking: bool
        Asynchronous if copying from CPU to GPU.
    """
    device_aware = True
    per_sample = True

    def __init__(self, device, non_blocking=True):
        super().__init__()
        self.device = device
        self.non_blocking = non_blocking

    def generate_code(self) -> Callable:
        target = ch.device(self.device)
        non_blocking = self.non_blocking

        def to_device(inp, dst):
            if _same_device(inp.device, target):
                return inp
            n = inp.shape[0]
            if inp.dim() == 4 and inp.is_contiguous(memory_format=ch.channels_last):
                # keep the channels-last storage order of an NCHW view
                b, c, h, w = inp.shape
                dst = dst.reshape(dst.shape[0], h, w, c).permute(0, 3, 1, 2)
            out = dst[:n]
            out.copy_(inp, non_blocking=non_blocking)
            return out
        return to_device

    def declare_state_and_memory(self, previous_state: State) -> Tuple[State, Optional[AllocationQuery]]:
        target = ch.device(self.device)
        if _same_device(previous_state.device, target):
            return previous_state, None
        buffer = AllocationQuery(previous_state.shape, dtype=previous_state.dtype, device=target)
        return replace(previous_state, device=target), buffer


class ToTorchImage(Operation):
    """NHWC batch -> NCHW (B x C x H x W) as torch expects images.

    Parameters
    ----------
    channels_last : bool
        Use torch.channels_last (a permuted view, no copy).
    convert_back_int16 : bool
        Reinterpret int16 storage (NormalizeImage's fp16 bits) as float16.
    """
    device_aware = True
    per_sample = True

    def __init__(self, channels_last=True, convert_back_int16=True):
        super().__init__()
        self.channels_last = channels_last
        self.convert_int16 = convert_back_int16
        self.enable_int16conv = False

    def generate_code(self) -> Callable:
        as_fp16 = self.enable_int16conv
        keep_view = self.channels_last

        def to_torch_image(inp: ch.Tensor, dst):
            if as_fp16:
                inp = inp.view(dtype=ch.float16)
            nchw = inp.permute(0, 3, 1, 2)
            if keep_view:
                assert nchw.is_contiguous(memory_format=ch.channels_last)
                return nchw
            out = dst[:nchw.shape[0]]
            out[:] = nchw.contiguous()
            return out
        return to_torch_image

    def declare_state_and_memory(self, previous_state: State) -> Tuple[State, Optional[AllocationQuery]]:
        H, W, C = previous_state.shape
        dtype = previous_state.dtype
        if dtype is ch.int16 and self.convert_int16:
            dtype = ch.float16
            self.enable_int16conv = True
        buffer = None if self.channels_last else AllocationQuery((C, H, W), dtype=dtype,
                                                                 device=previous_state.device)
        return replace(previous_state, shape=(C, H, W), dtype=dtype), buffer


class Convert(Operation):
    """Cast to ``target_dtype`` (torch ``Tensor.type``)."""
    device_aware = True
    per_sample = True

    def __init__(self, target_dtype):
        super().__init__()
        self.target_dtype = target_dtype

    def generate_code(self) -> Callable:
        target = self.target_dtype

        def convert(inp, dst):
            return inp.type(target)
        convert.is_parallel = True
        return convert

    def declare_state_and_memory(self, previous_state: State) -> Tuple[State, Optional[AllocationQuery]]:
        return replace(previous_state, dtype=self.target_dtype), None


class View(Operation):
    """Reinterpret the batch's bytes as ``target_dtype`` (``.view``)."""
    device_aware = True
    per_sample = True

    def __init__(self, target_dtype):
        super().__init__()
        self.target_dtype = target_dtype

    def generate_code(self) -> Callable:
        target = self.target_dtype

        def view(inp, dst):
            return inp.view(target)
        view.is_parallel = True
        return view

    def declare_state_and_memory(self, previous_state: State) -> Tuple[State, Optional[AllocationQuery]]:
        return replace(previous_state, dtype=self.target_dtype, jit_mode=False), None
