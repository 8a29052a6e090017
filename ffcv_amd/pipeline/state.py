"""Pipeline stage state (ffcv/pipeline/state.py:8-19).

Same fields and validity rules as the reference: ``jit_mode`` (host numpy
stage) implies a CPU device and a numpy dtype.  Device stages of this
framework run with ``jit_mode=False`` on a ``cuda`` (HIP) device.
"""
from dataclasses import dataclass
from typing import Any, Tuple

import torch as ch


@dataclass
class State:
    jit_mode: bool
    device: ch.device
    shape: Tuple[int, ...]
    dtype: Any

    def __post_init__(self):
        if self.jit_mode and self.device != ch.device('cpu'):
            raise AssertionError("Can't be in JIT mode and on the GPU")
        if self.jit_mode and isinstance(self.dtype, ch.dtype):
            raise AssertionError("Can't allocate a torch tensor in JIT mode")
