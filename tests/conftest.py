import os
import sys

import pytest

# torch (and its HIP runtime) before the in-tree libraries: with both HIP
# runtimes in one process, loading libaby3gpu.so first and torch later left
# hipSetDevice without devices on the GPU box (seen when CPU tests that call
# the host library ran before the first gpu-marked test of a session)
try:
    import torch  # noqa: F401
except ImportError:
    pass

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
TESTS = os.path.dirname(os.path.abspath(__file__))
if TESTS not in sys.path:
    sys.path.insert(0, TESTS)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels through the C-ABI)")


@pytest.fixture(scope="session")
def gpu():
    """The C-ABI library on cuda:0. Fails (never skips) when the GPU or the
    library is missing: a gpu-marked test must not pass on a fallback."""
    import torch

    assert torch.cuda.is_available(), "gpu tests need an MI355X"
    from aby3_amd import native

    lib = native.lib()
    lib.set_device(0)
    return lib


# The multi-process transport tests (three party processes per case) run
# after everything else: a transport fault there must not cut off the hot
# path's parity tests behind it under `pytest -x` (a fault in
# test_gpu_parties.py left every full-size C3/C4/C5 check unrun).
_LAST = ("test_gpu_parties.py",)


def pytest_collection_modifyitems(session, config, items):
    items.sort(key=lambda it: any(it.nodeid.split("::")[0].endswith(n) for n in _LAST))
