import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libpinot_hip.so)")


@pytest.fixture(scope="session")
def gpu_lib():
    """The product library on a GPU box; fails loudly (no CPU fallback) when it cannot load. Loaded after torch
    (one HIP runtime per process, _lib.load): the distributed tests drive RCCL on the library's buffers, and the
    test order must not decide which runtime the library binds to."""
    from pinot_amd import _lib
    lib = _lib.load(with_torch=True)
    import ctypes
    n = ctypes.c_int32(0)
    lib.phip_device_count(ctypes.byref(n))
    if n.value < 1:
        pytest.fail("no GPU visible to libpinot_hip.so")
    _lib.check(lib.phip_init(None, 0))
    return lib
