"""Concurrent IPC imports on one GPU (GPU box diagnostic for the round-3 open failure).

The W = 8 one-GPU rehearsal once failed with `hipIpcOpenMemHandle: invalid device pointer` on a
live, just-exported buffer (profiles/r03_v6/ipc_open_flake.txt).  tools/ipc_race_probe.py showed
that re-exporting one allocation returns the SAME 64 handle bytes (so the library never held two
handles of one allocation), that HIP_POINTER_ATTRIBUTE_BUFFER_ID is unique per allocation, and
that torch's caching allocator carves the rehearsal's three 4 MB send buffers out of ONE 20 MB
allocation.  This probe asks whether the failure is a runtime limit on CONCURRENT imports:
W processes each export one allocation (memset to its rank), all-gather the handles, then open
each other's handles in five patterns (below), all opens of a pattern at the same moment; each
opened mapping is read (one byte) and closed; every failed open is counted with its error code
and the slowest open is timed.
usage: python tools/ipc_stress_probe.py [W=8] [rounds=1]
"""
import ctypes as C
import multiprocessing as mp
import sys
import time

MB = 1 << 20


class IpcHandle(C.Structure):
    _fields_ = [("reserved", C.c_char * 64)]


def _hip():
    h = C.CDLL("libamdhip64.so")
    h.hipMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t]
    h.hipMemset.argtypes = [C.c_void_p, C.c_int, C.c_size_t]
    h.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
    h.hipIpcGetMemHandle.argtypes = [C.POINTER(IpcHandle), C.c_void_p]
    h.hipIpcOpenMemHandle.argtypes = [C.POINTER(C.c_void_p), IpcHandle, C.c_uint]
    h.hipIpcCloseMemHandle.argtypes = [C.c_void_p]
    h.hipGetErrorString.restype = C.c_char_p
    h.hipSetDevice(0)
    return h


def worker(rank, W, rounds, handles, bar, q, ptracer_any=False, plans_only=None):
    if ptracer_any:  # let any process of this user read this one's fds (Yama ptrace_scope 1)
        libc = C.CDLL(None)
        libc.prctl.argtypes = [C.c_int, C.c_ulong, C.c_ulong, C.c_ulong, C.c_ulong]
        print(f"rank {rank} prctl(PR_SET_PTRACER, ANY) = {libc.prctl(0x59616d61, C.c_ulong(-1).value, 0, 0, 0)}",
              flush=True)
    hip = _hip()
    p = C.c_void_p()
    assert hip.hipMalloc(C.byref(p), 20 * MB) == 0
    hip.hipMemset(p, rank + 1, 20 * MB)
    hip.hipDeviceSynchronize()
    h = IpcHandle()
    assert hip.hipIpcGetMemHandle(C.byref(h), p) == 0
    # all 64 bytes (a c_char-array FIELD reads back cut at its first NUL byte: the first version of
    # this probe shipped truncated handles and every open failed after ~10.5 s with error 17)
    handles[rank] = C.string_at(C.addressof(h), 64)
    bar.wait()
    slowest = [0.0]

    def one(g):
        hh = IpcHandle()
        C.memmove(C.addressof(hh), handles[g], 64)
        base = C.c_void_p()
        t0 = time.perf_counter()
        rc = hip.hipIpcOpenMemHandle(C.byref(base), hh, 1)
        slowest[0] = max(slowest[0], time.perf_counter() - t0)
        if rc != 0:
            hip.hipGetLastError()
            return rc, None
        v = (C.c_uint8 * 1)()
        hip.hipMemcpy(C.addressof(v), base, 1, 2)
        ok = v[0] == g + 1
        hip.hipIpcCloseMemHandle(base)
        return (0 if ok else -1000), base

    print(f"rank {rank} exported, {time.strftime('%X')}", flush=True)
    # who opens whom, all at the same moment (a barrier before each pattern):
    #   fanin  - every other rank opens rank 0's handle; rank 0 opens nothing
    #   mutual - ranks 0 and 1 open each other's handle; the rest open nothing
    #   chain  - rank r opens r + 1 (the last opens nothing): no cycle
    #   ring   - rank r opens (r + 1) % W: one cycle through every rank
    # (every rank opening every peer at once — the rehearsal's pattern — failed every open after
    # ~10.5 s in this probe's first version: profiles/r04/ipc_stress_burst.txt)
    plans = {
        "fanin": [0] if rank else [],
        "mutual": [1 - rank] if rank < 2 else [],
        "chain": [rank + 1] if rank + 1 < W else [],
        "ring": [(rank + 1) % W],
        "burst": [g for g in range(W) if g != rank],
    }
    if plans_only:
        plans = {m: t for m, t in plans.items() if m in plans_only}
    stats = {m: [0, 0, {}, 0.0] for m in plans}
    for mode, targets in plans.items():
        st = stats[mode]
        for rd in range(rounds):
            bar.wait()
            slowest[0] = 0.0
            for g in targets:
                rc, _ = one(g)
                st[0] += 1
                if rc:
                    st[1] += 1
                    st[2][rc] = st[2].get(rc, 0) + 1
            st[3] = max(st[3], slowest[0])
        print(f"rank {rank} {mode}: {st[1]} of {st[0]} opens failed {st[2]}, slowest "
              f"{1e3 * st[3]:.1f} ms", flush=True)
    bar.wait()
    q.put((rank, stats))


def run(W, rounds, method, ptracer_any, modes):
    ctx = mp.get_context(method)
    mgr = ctx.Manager()
    handles = mgr.list([b""] * W)
    bar = ctx.Barrier(W)
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(r, W, rounds, handles, bar, q, ptracer_any, modes))
          for r in range(W)]
    t0 = time.time()
    for p in ps:
        p.start()
    res = [q.get(timeout=300) for _ in ps]
    for p in ps:
        p.join()
    for mode in modes:
        opens = sum(st[mode][0] for _, st in res)
        fails = sum(st[mode][1] for _, st in res)
        codes = {}
        for _, st in res:
            for c, n in st[mode][2].items():
                codes[c] = codes.get(c, 0) + n
        slow = max(st[mode][3] for _, st in res)
        print(f"== start={method} ptracer_any={ptracer_any} W={W} {mode}: {fails} of {opens} opens "
              f"failed {codes}, slowest {1e3 * slow:.1f} ms  (17 = hipErrorInvalidDevicePointer)",
              flush=True)
    print(f"   ({time.time() - t0:.1f} s)", flush=True)


def main():
    W = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    try:
        with open("/proc/sys/kernel/yama/ptrace_scope") as f:
            print("kernel.yama.ptrace_scope =", f.read().strip(), flush=True)
    except OSError as e:
        print("no yama:", e, flush=True)
    # siblings started by spawn, with and without PR_SET_PTRACER_ANY, then by fork
    run(W, rounds, "spawn", False, ["fanin", "mutual", "chain", "ring", "burst"])

if __name__ == "__main__":
    main()
