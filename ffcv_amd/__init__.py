"""ffcv_amd: MI355X-native drop-in for ffcv's image decode-and-augment path.

``import ffcv_amd as ffcv`` gives the reference's public API surface for this
path: ``Loader``, ``DatasetWriter``, ``fields``, ``transforms``,
``pipeline`` (Operation / State / AllocationQuery), ``traversal_order``.
"""
__version__ = "0.1.0"

import os as _os

# Batches in flight each run on their own HIP stream; with HIP's default of 4
# hardware queues, streams beyond 3 share queues and serialise.  16 queues let
# the Loader keep 8 batches in flight (the measured optimum on MI355X,
# DESIGN.md section 6).  Raised to at least 16 -- environments commonly
# export HIP's default of 4 -- and only effective before the process's first
# HIP call.
try:
    _hwq = int(_os.environ.get('GPU_MAX_HW_QUEUES', '4'))
except ValueError:
    _hwq = 4
if _hwq < 16:
    _os.environ['GPU_MAX_HW_QUEUES'] = '16'

from .loader import Loader  # noqa: E402
from .writer import DatasetWriter  # noqa: E402

__all__ = ['Loader', 'DatasetWriter']
