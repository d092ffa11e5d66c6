"""GPU, multi-process: the shuffle-level exchange at world sizes 2..8 on one GPU (bootstrap
transport: host all-gather over gloo + one-sided IPC pulls following the per-round all-to-all
plan), TeraSort and Zipf keys, whole-shuffle sux_exchange and windowed sux_exchange_maps
overlapped with the next window's writes, every fetched block bit-exact vs the oracle
(tests/gpu_shuffle_exchange_check.py)."""
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


@pytest.mark.parametrize("world,workload,maps,extra", [
    (2, "terasort", 5, []), (3, "zipf", 7, []), (8, "terasort", 12, []), (8, "zipf", 12, []),
    # windows exchanged while the next window's maps run; several batches -> several rounds
    (4, "terasort", 16, ["--windows", "3", "--batch-maps", "2"]),
    (3, "zipf", 13, ["--windows", "2", "--batch-maps", "1", "--loopback"]),
    (8, "terasort", 24, ["--windows", "4", "--batch-maps", "2"])])
def test_shuffle_exchange_bootstrap(world, workload, maps, extra):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={world}", "--master-addr=127.0.0.1",
           f"--master-port={_free_port()}", os.path.join(HERE, "gpu_shuffle_exchange_check.py"),
           "--workload", workload, "--maps", str(maps)] + extra
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, OMP_NUM_THREADS="1"))
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-4000:]
    assert "shuffle exchange ok" in r.stdout
