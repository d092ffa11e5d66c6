"""CPU, multi-process: the partition-aligned all-to-all exchange with world_size 2 and 3 (gloo)."""
import os
import socket
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(world, *args):
    env = dict(os.environ, OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={world}", "--master-addr=127.0.0.1",
           f"--master-port={_free_port()}", os.path.join(HERE, "dist_exchange_check.py"), *args]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "exchange ok" in r.stdout
    return r.stdout


def test_exchange_world2_matches_golden():
    _run(2, "--golden", os.path.join(HERE, "golden", "exchange_3maps_G2.json"))


@pytest.mark.parametrize("world,R,maps", [(2, 200, 2), (3, 10, 4)])
def test_exchange_world_sizes(world, R, maps):
    _run(world, "--R", str(R), "--maps", str(maps), "--rpm", "700")


@pytest.mark.parametrize("world", [2, 3])
def test_exchange_zipf_balanced_ownership(world):
    """Zipf keys (C4), ownership balanced from the all-reduced partition bytes;
    every block bit-exact through the owned plan, and the busiest owner's ingress closer to the
    mean than under the equal split."""
    bal = _run(world, "--zipf", "--balanced", "--R", "200", "--maps", "2", "--rpm", "5000")
    eq = _run(world, "--zipf", "--R", "200", "--maps", "2", "--rpm", "5000")
    ratio = lambda out: float(out.split("ingress max/mean=")[1].split()[0])  # noqa: E731
    assert ratio(bal) <= ratio(eq) + 1e-9
