import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs a HIP device (MI355X); run with -m gpu')


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope='session')
def hip_lib():
    """The product library; building it is part of the check."""
    from ffcv_amd import _build
    _build.build()
    from ffcv_amd import libffcv
    return libffcv.lib()


@pytest.fixture(scope='session')
def oracle():
    from oracle import oracle as O
    O.build()
    return O
