"""GPU: the C++ plugin mirror (include/sparkucx_amd/ucx_shuffle.hpp) end to end on cuda:0.

Runs tests/cpp/test_host_mirror (built in-tree by __graft_entry__.build() / `make -C tests/cpp`):
registerShuffle -> getWriter().write -> writeIndexFileAndCommit -> getReader().read /
UcxShuffleClient.fetchBlocks -> listener callbacks -> release, checked against the CPU oracle.
"""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "cpp", "test_host_mirror")


def test_cpp_host_mirror():
    assert os.path.exists(BIN), "build it first: make -C tests/cpp"
    r = subprocess.run([BIN], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
