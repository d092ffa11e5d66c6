"""GPU, multi-process: the one-sided IPC pull exchange with 2 and 3 ranks sharing cuda:0."""
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world", [2, 3])
def test_ipc_pull_exchange(world):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={world}", "--master-addr=127.0.0.1",
           f"--master-port={_free_port()}", os.path.join(HERE, "gpu_ipc_exchange_check.py")]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240,
                       env=dict(os.environ, OMP_NUM_THREADS="1"))
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-4000:]
    assert "ipc exchange ok" in r.stdout
