"""Shared pytest setup.

Markers:
  gpu  — needs an MI355X (runs the HIP path through the C-ABI); the driver runs
         these with ``pytest -m gpu`` on a GPU box and ``-m "not gpu"`` here.
"""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD Instinct GPU (gfx950) and libof2d.so")


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as O
    O.lib().oracle_capture_output(1)
    return O


@pytest.fixture(scope="session")
def of2d_lib():
    """libof2d.so (built in-tree); fails loudly when missing."""
    from opticalflow2d_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        _lib.build()
    return _lib.lib()


@pytest.fixture(scope="session")
def gpu(of2d_lib):
    """Device presence for the gpu-marked tests: no silent CPU fallback."""
    import ctypes
    n = ctypes.c_int(0)
    of2d_lib.of2d_device_count(ctypes.byref(n))
    assert n.value > 0, "no HIP device visible: gpu tests need an MI355X"
    from opticalflow2d_amd import set_print_sink
    captured = []
    set_print_sink(captured.append)
    return captured


def golden(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)
