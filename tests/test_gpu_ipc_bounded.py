"""GPU: an IPC import that does not return is bounded.

The round-5 W = 8 probe stalled inside hipIpcOpenMemHandle (profiles/r06_ipc/: the runtime's
import of a torch-allocated 2048 / 3072 MiB buffer into a process holding one of its own never
returns).  sux_ipc_open now waits at most SUX_IPC_OPEN_TIMEOUT_S seconds and fails with SUX_ECOMM
naming the exporter.  Driven here with a handle the runtime cannot resolve (round 4 measured such
an open to spend ~10.5 s inside the runtime before it fails): with a 2 s bound the call returns
ECOMM after ~2 s, in a child process (the abandoned helper thread dies with it)."""
import os
import subprocess
import sys
import textwrap

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = textwrap.dedent("""
    import sys, time
    sys.path.insert(0, %r)
    import torch
    from sparkucx_amd import native as N
    from sparkucx_amd.shuffle import Node
    node = Node(device=0)
    buf = torch.zeros(1 << 20, dtype=torch.uint8, device="cuda")
    desc = bytearray(node.ipc_handle(buf))
    desc[0:8] = (0x7fff00000000).to_bytes(8, "little")  # an address no allocation has
    desc[8:12] = (1).to_bytes(4, "little")              # exported by pid 1
    t0 = time.perf_counter()
    try:
        node.ipc_open(bytes(desc))
        print("OPENED")
    except N.SuxError as e:
        print("CODE", e.code, round(time.perf_counter() - t0, 2), str(e)[:300])
    sys.stdout.flush()
    node.close()
""") % ROOT


def test_stuck_ipc_open_returns_ecomm_with_the_exporter_named():
    env = dict(os.environ, SUX_IPC_OPEN_TIMEOUT_S="2")
    r = subprocess.run([sys.executable, "-c", CHILD], capture_output=True, text=True,
                       timeout=120, env=env)
    out = r.stdout
    assert "CODE" in out, out + r.stderr[-2000:]
    code, secs = out.split("CODE", 1)[1].split()[:2]
    if int(code) == -4:  # SUX_ECOMM: the bound fired
        assert 1.5 <= float(secs) < 10 and "pid 1" in out and "did not return" in out, out
    else:  # the runtime rejected the handle within the bound: a prompt error, no hang either
        assert int(code) == -3 and float(secs) < 2.5, out
