"""General operations (ffcv/transforms/ops.py:17-160): ToTensor, ToDevice,
ToTorchImage, Convert, View.

Device stages hand tensors between kernels on the slot's HIP stream.
``ToTensor`` and ``ToDevice`` are free when the decoder already produced a
tensor on the target device (the device-resident path); otherwise they do
exactly what the reference does (from_numpy / non_blocking H2D copy).
"""
from dataclasses import replace
from typing import Callable, Optional, Tuple

import numpy as np
import torch as ch

from ..pipeline.allocation_query import AllocationQuery
from ..pipeline.operation import Operation
from ..pipeline.state import State


def _torch_dtype(dtype):
    if isinstance(dtype, ch.dtype):
        return dtype
    return ch.from_numpy(np.empty((), dtype=dtype)).dtype


class ToTensor(Operation):
    """Convert from Numpy array to PyTorch Tensor."""
    device_aware = True
    per_sample = True

    def __init__(self):
        super().__init__()

    def generate_code(self) -> Callable:
        def to_tensor(inp, dst):
            if isinstance(inp, ch.Tensor):
                return inp
            return ch.from_numpy(inp)
        return to_tensor

    def declare_state_and_memory(self, previous_state: State) -> Tuple[State, Optional[AllocationQuery]]:
        new_dtype = _torch_dtype(previous_state.dtype)
        return replace(previous_state, jit_mode=False, dtype=new_dtype), None


class ToDevice(Operation):
    """Move tensor to device (ops.py:32-62).

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

        def to_device(inp, dst):
            if inp.device == target or (target.type == inp.device.type == 'cuda' and
                                        target.index is None):
                return inp
            if len(inp.shape) == 4:
                if inp.is_contiguous(memory_format=ch.channels_last):
                    dst = dst.reshape(inp.shape[0], inp.shape[2], inp.shape[3], inp.shape[1])
                    dst = dst.permute(0, 3, 1, 2)
            dst = dst[:inp.shape[0]]
            dst.copy_(inp, non_blocking=self.non_blocking)
            return dst
        return to_device

    def declare_state_and_memory(self, previous_state: State) -> Tuple[State, Optional[AllocationQuery]]:
        target = ch.device(self.device)
        if previous_state.device.type == target.type and (target.index is None or
                                                          previous_state.device == target):
            return replace(previous_state, device=previous_state.device), None
        return replace(previous_state, device=target), AllocationQuery(previous_state.shape,
                                                                       dtype=previous_state.dtype,
                                                                       device=target)


class ToTorchImage(Operation):
    """Change tensor to PyTorch format for images (B x C x H x W).

    Parameters
    ----------
    channels_last : bool
        Use torch.channels_last.
    convert_back_int16 : bool
        Convert to float16.
    """
    device_aware = True
    per_sample = True

    def __init__(self, channels_last=True, convert_back_int16=True):
        super().__init__()
        self.channels_last = channels_last
        self.convert_int16 = convert_back_int16
        self.enable_int16conv = False

    def generate_code(self) -> Callable:
        do_conv = self.enable_int16conv
        channels_last = self.channels_last

        def to_torch_image(inp: ch.Tensor, dst):
            if do_conv:
                inp = inp.view(dtype=ch.float16)
            inp = inp.permute([0, 3, 1, 2])
            if channels_last:
                assert inp.is_contiguous(memory_format=ch.channels_last)
                return inp
            dst[:inp.shape[0]] = inp.contiguous()
            return dst[:inp.shape[0]]
        return to_torch_image

    def declare_state_and_memory(self, previous_state: State) -> Tuple[State, Optional[AllocationQuery]]:
        alloc = None
        H, W, C = previous_state.shape
        new_type = previous_state.dtype
        if new_type is ch.int16 and self.convert_int16:
            new_type = ch.float16
            self.enable_int16conv = True
        if not self.channels_last:
            alloc = AllocationQuery((C, H, W), dtype=new_type, device=previous_state.device)
        return replace(previous_state, shape=(C, H, W), dtype=new_type), alloc


class Convert(Operation):
    """Convert to target data type (ops.py:114-136)."""
    device_aware = True
    per_sample = True

    def __init__(self, target_dtype):
        super().__init__()
        self.target_dtype = target_dtype

    def generate_code(self) -> Callable:
        def convert(inp, dst):
            return inp.type(self.target_dtype)
        convert.is_parallel = True
        return convert

    def declare_state_and_memory(self, previous_state: State) -> Tuple[State, Optional[AllocationQuery]]:
        return replace(previous_state, dtype=self.target_dtype), None


class View(Operation):
    """View array using np.view or torch.view (ops.py:139-160)."""
    device_aware = True
    per_sample = True

    def __init__(self, target_dtype):
        super().__init__()
        self.target_dtype = target_dtype

    def generate_code(self) -> Callable:
        def convert(inp, dst):
            return inp.view(self.target_dtype)
        convert.is_parallel = True
        return convert

    def declare_state_and_memory(self, previous_state: State) -> Tuple[State, Optional[AllocationQuery]]:
        return replace(previous_state, dtype=self.target_dtype, jit_mode=False), None
