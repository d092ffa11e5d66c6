"""Concurrent IPC imports on one GPU (GPU box diagnostic for the round-3 open failure).

The W = 8 one-GPU rehearsal once failed with `hipIpcOpenMemHandle: invalid device pointer` on a
live, just-exported buffer (profiles/r03_v6/ipc_open_flake.txt).  tools/ipc_race_probe.py showed
that re-exporting one allocation returns the SAME 64 handle bytes (so the library never held two
handles of one allocation), that HIP_POINTER_ATTRIBUTE_BUFFER_ID is unique per allocation, and
that torch's caching allocator carves the rehearsal's three 4 MB send buffers out of ONE 20 MB
allocation.  This probe asks whether the failure is a runtime limit on CONCURRENT imports:
W processes each export one allocation (memset to its rank), all-gather the handles, then
  - mode "burst": every process opens all W - 1 peers' handles at the same moment (a barrier
    before), reads one byte of each, closes them — the rehearsal's pattern;
  - mode "staggered": step k, process r opens only peer (r + k) % W, so every exporter serves
    exactly one importer at a time;
repeated for `rounds` rounds; every failed open is counted with its error code.
usage: python tools/ipc_stress_probe.py [W=8] [rounds=30]
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


def worker(rank, W, rounds, handles, bar, q):
    hip = _hip()
    p = C.c_void_p()
    assert hip.hipMalloc(C.byref(p), 20 * MB) == 0
    hip.hipMemset(p, rank + 1, 20 * MB)
    hip.hipDeviceSynchronize()
    h = IpcHandle()
    assert hip.hipIpcGetMemHandle(C.byref(h), p) == 0
    handles[rank] = bytes(h.reserved)
    bar.wait()
    stats = {"burst": [0, 0, {}], "staggered": [0, 0, {}]}  # opens, failures, codes

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
    for mode in ("burst", "staggered"):
        st = stats[mode]
        for rd in range(rounds):
            print(f"rank {rank} {mode} round {rd}: {st[1]} failed of {st[0]}, slowest open "
                  f"{1e3 * slowest[0]:.1f} ms", flush=True)
            bar.wait()
            if mode == "burst":
                for g in range(W):
                    if g == rank:
                        continue
                    rc, _ = one(g)
                    st[0] += 1
                    if rc:
                        st[1] += 1
                        st[2][rc] = st[2].get(rc, 0) + 1
            else:
                for k in range(1, W):
                    bar.wait()
                    rc, _ = one((rank + k) % W)
                    st[0] += 1
                    if rc:
                        st[1] += 1
                        st[2][rc] = st[2].get(rc, 0) + 1
    bar.wait()
    q.put((rank, stats))


def main():
    W = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    ctx = mp.get_context("spawn")
    mgr = ctx.Manager()
    handles = mgr.list([b""] * W)
    bar = ctx.Barrier(W)
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(r, W, rounds, handles, bar, q)) for r in range(W)]
    t0 = time.time()
    for p in ps:
        p.start()
    res = [q.get(timeout=300) for _ in ps]
    for p in ps:
        p.join()
    tot = {"burst": [0, 0, {}], "staggered": [0, 0, {}]}
    for rank, st in sorted(res):
        for m in tot:
            tot[m][0] += st[m][0]
            tot[m][1] += st[m][1]
            for c, n in st[m][2].items():
                tot[m][2][c] = tot[m][2].get(c, 0) + n
        print(f"rank {rank}: burst {st['burst'][1]}/{st['burst'][0]} failed {st['burst'][2]}, "
              f"staggered {st['staggered'][1]}/{st['staggered'][0]} failed {st['staggered'][2]}")
    print(f"W={W} rounds={rounds} ({time.time() - t0:.1f} s): burst {tot['burst'][1]} of "
          f"{tot['burst'][0]} opens failed {tot['burst'][2]}; staggered {tot['staggered'][1]} of "
          f"{tot['staggered'][0]} failed {tot['staggered'][2]} (1 = invalid value, "
          f"17 = invalid device pointer, -1000 = wrong bytes)")


if __name__ == "__main__":
    main()
