"""Compatibility shim for ffcv/pipeline/compiler.py:9-42.

The reference JIT-compiles per-sample loops with numba.  Here the hot path
is precompiled HIP (libffcv_hip.so) and stages are scheduled on HIP streams,
so ``Compiler.compile`` returns the Python function unchanged (the
reference's ``set_enabled(False)`` behaviour) and ``get_iterator`` is
``range``.  ``set_num_threads`` still bounds torch's intra-op threads, as in
the reference.
"""
from os import sched_getaffinity

import torch as ch


class Compiler:
    is_enabled = False
    num_threads = 1

    @classmethod
    def set_enabled(cls, b):
        cls.is_enabled = bool(b)

    @classmethod
    def set_num_threads(cls, n):
        if n < 1:
            n = len(sched_getaffinity(0))
        cls.num_threads = n
        ch.set_num_threads(n)

    @classmethod
    def compile(cls, code, signature=None):
        return code

    @classmethod
    def get_iterator(cls):
        return range
