"""Field ABC (ffcv/fields/base.py:8-45)."""
from __future__ import annotations

from abc import ABC, abstractmethod
from typing import Type

import numpy as np

from ..pipeline.operation import Operation

ARG_TYPE = np.dtype([('', '<u1', 1024)])


class Field(ABC):
    @property
    @abstractmethod
    def metadata_type(self) -> np.dtype:
        raise NotImplementedError

    @staticmethod
    @abstractmethod
    def from_binary(binary: ARG_TYPE) -> Field:
        raise NotImplementedError

    @abstractmethod
    def to_binary(self) -> ARG_TYPE:
        raise NotImplementedError

    @abstractmethod
    def encode(field, metadata_destination, malloc):
        raise NotImplementedError

    @abstractmethod
    def get_decoder_class(self) -> Type[Operation]:
        raise NotImplementedError
