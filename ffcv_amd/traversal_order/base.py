"""ffcv/traversal_order/base.py:10-20."""
from abc import ABC, abstractmethod
from typing import Sequence


class TraversalOrder(ABC):
    def __init__(self, loader):
        self.loader = loader
        self.indices = self.loader.indices
        self.seed = self.loader.seed
        self.distributed = loader.distributed
        self.sampler = None

    @abstractmethod
    def sample_order(self, epoch: int) -> Sequence[int]:
        raise NotImplementedError()
