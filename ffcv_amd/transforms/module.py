"""Wrap a torch.nn.Module as an Operation (ffcv/transforms/module.py)."""
from dataclasses import replace
from typing import Callable, Optional, Tuple

import torch as ch

from ..pipeline.allocation_query import AllocationQuery
from ..pipeline.operation import Operation
from ..pipeline.state import State


class ModuleWrapper(Operation):
    """Transform using the given torch.nn.Module (on the tensor's device)."""
    device_aware = True

    def __init__(self, module: ch.nn.Module):
        super().__init__()
        self.module = module

    def generate_code(self) -> Callable:
        def apply_module(inp, _):
            return self.module(inp)
        return apply_module

    def declare_state_and_memory(self, previous_state: State) -> Tuple[State, Optional[AllocationQuery]]:
        return replace(previous_state, jit_mode=False), None
