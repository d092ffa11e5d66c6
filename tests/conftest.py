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
