"""GPU, two processes: an IPC mapping must never outlive the allocation it was opened for.

Process A exports an allocation, B opens it through the library (sux_ipc_open); A frees it and
allocates again — HIP hands the same address back — and exports the new allocation; B opens that
one too and must read the NEW bytes.  The HIP runtime keys its imported mappings by the
exporter's address, so it returns B's still-open mapping of the old, freed memory for the new
handle; the library detects a returned base it already holds under another handle, drops the
stale mapping and opens the handle again (sux_api.cpp, ipc_open_fresh)."""
import ctypes as C
import multiprocessing as mp
import os
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MB = 1 << 20
SIZE = 100 * MB


def _hip():
    h = C.CDLL("libamdhip64.so")
    h.hipMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t]
    h.hipFree.argtypes = [C.c_void_p]
    h.hipMemset.argtypes = [C.c_void_p, C.c_int, C.c_size_t]
    h.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
    h.hipDeviceSynchronize.argtypes = []
    return h


def _exporter(conn):
    sys.path.insert(0, ROOT)
    from sparkucx_amd.shuffle import Node
    hip = _hip()
    node = Node(device=0)
    p = C.c_void_p()
    assert hip.hipMalloc(C.byref(p), SIZE) == 0
    hip.hipMemset(p, 0x11, SIZE)
    hip.hipDeviceSynchronize()
    conn.send((p.value, _export(node, p.value)))
    assert conn.recv() == "opened"
    hip.hipFree(p)
    q = C.c_void_p()
    assert hip.hipMalloc(C.byref(q), SIZE) == 0
    hip.hipMemset(q, 0x22, SIZE)
    hip.hipDeviceSynchronize()
    conn.send((q.value, _export(node, q.value)))
    assert conn.recv() == "done"
    hip.hipFree(q)
    node.close()


def _export(node, ptr):
    buf = (C.c_uint8 * 72)()
    rc = node.lib.sux_ipc_export(node.h, C.c_void_p(ptr), buf)
    assert rc == 0
    return bytes(buf)


def _read_byte(hip, ptr):
    b = (C.c_uint8 * 1)()
    assert hip.hipMemcpy(C.addressof(b), C.c_void_p(ptr), 1, 2) == 0  # D2H
    return b[0]


def test_reopened_address_maps_the_new_allocation():
    sys.path.insert(0, ROOT)
    from sparkucx_amd.shuffle import Node
    # this process's runtime first (torch, then the library), then the exporter child: a parent
    # whose first HIP initialisation raced its freshly spawned child's once found no GPU
    hip = _hip()
    node = Node(device=0)
    ctx = mp.get_context("spawn")
    a, b = ctx.Pipe()
    proc = ctx.Process(target=_exporter, args=(b,))
    proc.start()
    try:
        va1, h1 = a.recv()
        p1 = node.ipc_open(h1)
        assert _read_byte(hip, p1) == 0x11
        a.send("opened")
        va2, h2 = a.recv()
        p2 = node.ipc_open(h2)
        got = _read_byte(hip, p2)
        a.send("done")
        assert got == 0x22, (f"the second handle (exporter address {va2:#x}, first was {va1:#x}) "
                             f"mapped the freed allocation: read {got:#x}")
        node.ipc_close(p2)
        node.close()
    finally:
        proc.join(60)
        if proc.is_alive():  # never leave the exporter waiting on the pipe
            proc.kill()
            proc.join()
        assert proc.exitcode == 0


def test_unresolvable_handle_fails_once_with_a_diagnosis():
    """A handle the runtime cannot resolve (here: a live handle with its exporter pid field
    pointing at a process that exported nothing) fails at once — no retry loop (round 3 had
    one) — with the exporter pid / address and this process's descriptor count in the message
    (DESIGN.md §5).  The runtime itself spends ~10 s on it before it gives up."""
    sys.path.insert(0, ROOT)
    from sparkucx_amd import native as N
    from sparkucx_amd.shuffle import Node
    node = Node(device=0)
    try:
        desc = bytearray(72)
        desc[0:8] = (0x7f0000000000).to_bytes(8, "little")
        desc[8:12] = (1).to_bytes(4, "little")  # pid 1 exported nothing
        with pytest.raises(N.SuxError) as e:
            node.ipc_open(bytes(desc))
        assert e.value.code == N.SUX_EHIP
        assert "exporter pid 1" in str(e.value) and "open descriptors" in str(e.value)
    finally:
        node.close()
