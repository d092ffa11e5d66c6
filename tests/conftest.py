import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")


@pytest.fixture(scope="session")
def gpu_node():
    """One shuffle node on cuda:0 for the whole GPU session (fails loudly without a GPU)."""
    import torch
    from sparkucx_amd.shuffle import Node

    assert torch.cuda.is_available(), "gpu tests need a GPU; run with -m 'not gpu' on CPU"
    node = Node(device=0)
    yield node
    node.close()


@pytest.fixture
def tuned(gpu_node):
    """Set fields of the session node's tuning table for one test; restored afterwards."""
    saved = gpu_node.tuning()

    def set_(**fields):
        gpu_node.set_tuning(**fields)
        return gpu_node

    yield set_
    gpu_node.set_tuning(**saved)
    gpu_node.check()  # no kernel recorded a failure under the test's tuning


@pytest.fixture(autouse=True)
def no_stale_hip_error(request):
    """After every GPU test: no HIP error may be left in this thread's last-error slot.  torch
    checks hipGetLastError() after its own kernel launches, so a stale error left by a library
    call (RCCL leaves "invalid device ordinal" behind some of its calls) would fail whatever
    torch launch comes next, in another test; this names the test that left it."""
    yield
    if request.node.get_closest_marker("gpu") is None:
        return
    import ctypes

    import torch
    # a test that ran the GPU only in child processes left nothing in this process; probing
    # here would load and initialise a HIP runtime before torch's own (the system library by
    # name, ahead of the one torch brings), after which torch found no GPU in this process
    if not torch.cuda.is_initialized():
        return
    try:
        hip = ctypes.CDLL("libamdhip64.so.7")
    except OSError:
        return
    hip.hipGetLastError.restype = ctypes.c_int
    err = hip.hipGetLastError()  # reads and clears
    assert err == 0, f"the test left HIP error {err} in the last-error slot"
