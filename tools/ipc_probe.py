"""Do two live allocations ever export identical hipIpcMemHandle bytes?  (GPU box diagnostic)

Allocates buffers of the plugin leg's slab sizes with hipMalloc, exports their IPC handles,
frees one and allocates again, and prints which handles coincide.
usage: python tools/ipc_probe.py
"""
import ctypes as C

hip = C.CDLL("libamdhip64.so")


def malloc(n):
    p = C.c_void_p()
    assert hip.hipMalloc(C.byref(p), C.c_size_t(n)) == 0
    return p


def handle(p):
    h = (C.c_char * 64)()
    rc = hip.hipIpcGetMemHandle(h, p)
    assert rc == 0, rc
    return bytes(h)


def main():
    MB = 1 << 20
    live = {}
    for name, size in [("a100", 100 * MB), ("b100", 100 * MB), ("c52", 52 * MB), ("d52", 52 * MB),
                       ("e200", 200 * MB), ("f12", 12 * MB), ("g12", 12 * MB)]:
        live[name] = malloc(size)
    hs = {k: handle(v) for k, v in live.items()}
    for k, h in hs.items():
        print(k, hex(live[k].value), h[:40].hex())
    print("again a100 equal:", handle(live["a100"]) == hs["a100"])
    dup = [(a, b) for a in hs for b in hs if a < b and hs[a] == hs[b]]
    print("identical handles among live allocations:", dup)
    hip.hipFree(live["a100"])
    live["h100"] = malloc(100 * MB)
    hh = handle(live["h100"])
    print("h100 (after freeing a100)", hex(live["h100"].value), hh[:40].hex(),
          "== old a100:", hh == hs["a100"], "== any live:", [k for k in hs if k != "a100" and hs[k] == hh])


if __name__ == "__main__":
    main()
