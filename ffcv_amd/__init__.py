"""ffcv_amd: MI355X-native drop-in for ffcv's image decode-and-augment path.

``import ffcv_amd as ffcv`` gives the reference's public API surface for this
path: ``Loader``, ``DatasetWriter``, ``fields``, ``transforms``,
``pipeline`` (Operation / State / AllocationQuery), ``traversal_order``.
"""
__version__ = "0.1.0"

from .loader import Loader
from .writer import DatasetWriter

__all__ = ['Loader', 'DatasetWriter']
