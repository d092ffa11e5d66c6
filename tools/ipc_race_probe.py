"""What the HIP runtime does when ONE allocation is exported more than once (GPU box diagnostic).

The W = 8 one-GPU rehearsal failed once with `hipIpcOpenMemHandle: invalid device pointer`
(profiles/r03_v6/ipc_open_flake.txt).  Its send buffers were 4 MB torch tensors: the caching
allocator carves blocks of 1-10 MB out of one 20 MB segment, so the three send buffers of a rank
share ONE hipMalloc allocation and sux_ipc_export (hipMemGetAddressRange -> hipIpcGetMemHandle
of the base) exported that allocation three times, one all-gather apart.  This probe asks the
runtime directly, with raw hip calls (no library code):

  1. do repeated hipIpcGetMemHandle calls on one live allocation return the same 64 bytes?
  2. can an importer still open the FIRST handle after the exporter created later ones?
  3. does a second handle of the same allocation open to the same base in the importer?

usage: python tools/ipc_race_probe.py    (two processes on cuda:0)
"""
import ctypes as C
import multiprocessing as mp
import struct
import time

MB = 1 << 20


class IpcHandle(C.Structure):  # hipIpcMemHandle_t, passed BY VALUE to hipIpcOpenMemHandle
    _fields_ = [("reserved", C.c_char * 64)]


def _hip():
    h = C.CDLL("libamdhip64.so")
    h.hipMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t]
    h.hipFree.argtypes = [C.c_void_p]
    h.hipMemset.argtypes = [C.c_void_p, C.c_int, C.c_size_t]
    h.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
    h.hipIpcGetMemHandle.argtypes = [C.c_void_p, C.c_void_p]
    h.hipIpcOpenMemHandle.argtypes = [C.POINTER(C.c_void_p), IpcHandle, C.c_uint]
    h.hipIpcCloseMemHandle.argtypes = [C.c_void_p]
    h.hipSetDevice(0)
    return h


def handle(hip, p):
    h = (C.c_char * 64)()
    rc = hip.hipIpcGetMemHandle(h, p)
    return rc, bytes(h)


def fields(h):
    return " ".join(f"{w:08x}" for w in struct.unpack("<16I", h))


def exporter(conn, n_exports):
    hip = _hip()
    p = C.c_void_p()
    assert hip.hipMalloc(C.byref(p), 20 * MB) == 0
    hip.hipMemset(p, 0x5A, 20 * MB)
    hip.hipDeviceSynchronize()
    hs = []
    for k in range(n_exports):
        rc, h = handle(hip, p)
        hs.append((rc, h))
        if k == 0:
            conn.send(("first", p.value, rc, h))
            conn.recv()  # the importer opened the first handle
    conn.send(("all", p.value, hs))
    conn.recv()  # importer done
    hip.hipFree(p)
    conn.send("freed")


def open_h(hip, h):
    base = C.c_void_p()
    hh = IpcHandle()
    C.memmove(C.addressof(hh), h, 64)
    rc = hip.hipIpcOpenMemHandle(C.byref(base), hh, 1)
    return rc, base.value


def torch_layout():
    """The rehearsal's send ring: three 4 MB torch tensors -> their allocation bases."""
    import torch
    hip = _hip()
    hip.hipMemGetAddressRange.argtypes = [C.POINTER(C.c_void_p), C.POINTER(C.c_size_t), C.c_void_p]
    ts = [torch.empty(40000 * 100, dtype=torch.uint8, device="cuda:0") for _ in range(3)]
    for k, t in enumerate(ts):
        base, size = C.c_void_p(), C.c_size_t()
        hip.hipMemGetAddressRange(C.byref(base), C.byref(size), C.c_void_p(t.data_ptr()))
        print(f"torch send[{k}] {t.data_ptr():#x}: allocation base {base.value:#x} "
              f"size {size.value >> 20} MB offset {t.data_ptr() - base.value}")


def buffer_ids():
    """HIP_POINTER_ATTRIBUTE_BUFFER_ID of allocations, and of a new one at a freed address."""
    hip = _hip()
    hip.hipPointerGetAttribute.argtypes = [C.c_void_p, C.c_int, C.c_void_p]
    attr = 7  # HIP_POINTER_ATTRIBUTE_BUFFER_ID (driver_types.h: CONTEXT = 1, ... BUFFER_ID = 7)

    def bid(p):
        v = C.c_ulonglong(0)
        rc = hip.hipPointerGetAttribute(C.byref(v), attr, p)
        return rc, v.value

    a, b = C.c_void_p(), C.c_void_p()
    hip.hipMalloc(C.byref(a), 20 * MB)
    hip.hipMalloc(C.byref(b), 20 * MB)
    print("buffer id a", hex(a.value), bid(a), "b", hex(b.value), bid(b))
    print("buffer id a+4MB (inside a)", bid(C.c_void_p(a.value + 4 * MB)))
    old = a.value
    hip.hipFree(a)
    c = C.c_void_p()
    hip.hipMalloc(C.byref(c), 20 * MB)
    print("after free: new allocation at", hex(c.value), "same address:", c.value == old,
          "buffer id", bid(c))


def main():
    ctx = mp.get_context("spawn")
    p = ctx.Process(target=buffer_ids)
    p.start()
    p.join()
    p = ctx.Process(target=torch_layout)
    p.start()
    p.join()
    for delayed in (False, True):
        a, b = ctx.Pipe()
        proc = ctx.Process(target=exporter, args=(b, 4))
        proc.start()
        hip = _hip()
        _, va, rc0, h0 = a.recv()
        print(f"--- importer opens the first handle {'AFTER' if delayed else 'BEFORE'} "
              f"the exporter created three more")
        print(f"exporter base {va:#x}; first export rc {rc0}: {fields(h0)}")
        opened = []
        if not delayed:
            opened.append(("first", open_h(hip, h0)))
        a.send("go")
        _, _, hs = a.recv()
        for k, (rc, h) in enumerate(hs):
            print(f"export {k}: rc {rc} same bytes as export 0: {h == h0}  {fields(h)}")
        if delayed:
            time.sleep(0.05)
            opened.append(("first (late)", open_h(hip, h0)))
        for k, (rc, h) in enumerate(hs[1:], 1):
            opened.append((f"export {k}", open_h(hip, h)))
        for name, (rc, base) in opened:
            print(f"open {name}: rc {rc} base {base if base is None else hex(base)}")
            if rc == 0:
                v = (C.c_uint8 * 1)()
                hip.hipMemcpy(C.addressof(v), C.c_void_p(base), 1, 2)
                print(f"   reads {v[0]:#x} (exporter wrote 0x5a)")
        for name, (rc, base) in opened:
            if rc == 0:
                print(f"close {name}: rc {hip.hipIpcCloseMemHandle(C.c_void_p(base))}")
        a.send("done")
        print(a.recv())
        proc.join()


if __name__ == "__main__":
    main()
