"""Host cost of the bench's in-step block resolve, piece by piece (GPU box).

954 maps x 1024 TeraSort records (the headline's map count, tiny maps: the resolve's cost does
not depend on record counts), R = 200, one block per (map, reduce task) as bench.py resolves.
usage: python tools/resolve_probe.py
"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sparkucx_amd import native as N  # noqa: E402
from sparkucx_amd.shuffle import Node  # noqa: E402


def t(f, reps=5):
    best = 1e9
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        f()
        best = min(best, time.perf_counter() - t0)
    return best * 1e3


def lex_sorted(b):
    return b[np.lexsort(b.T[::-1])]


def main(maps=954, rpm=1024, R=200, rs=100):
    n = maps * rpm
    with Node(device=0) as node:
        if rs == 100:
            part = node.partitioner(N.PART_RANGE_BYTES, R, key_offset=0, key_len=10,
                                    bounds=lex_sorted(np.random.default_rng(1).integers(
                                        0, 256, (R - 1, 10), dtype=np.uint8)).tobytes())
            recs = node.generate(N.GEN_TERASORT, 1, 0, n, rs)
        else:
            part = node.partitioner(N.PART_MURMUR3_LONG, R, key_offset=0, key_len=8)
            recs = node.generate(N.GEN_SMALL, 1, 0, n, rs)
        out, index, _ = node.partition_maps(part, recs, rs, rpm)
        torch.cuda.synchronize()
        tasks = min(R, 200)
        lo_t = (np.arange(tasks) * R) // tasks
        hi_t = (np.arange(1, tasks + 1) * R) // tasks
        blocks = np.stack([np.repeat(np.arange(maps), tasks), np.tile(lo_t, maps),
                           np.tile(hi_t, maps)], 1).astype(np.int32)
        arr = Node._blocks(blocks)
        res = {"blocks": len(blocks)}
        res["convert_ms"] = t(lambda: Node._blocks(blocks))
        sid = [100]

        def reg():
            sid[0] += 1
            node.register_shuffle(sid[0], maps, R, rs)
            node.adopt_map_outputs(sid[0], 0, out, rpm, n, index)

        def full():
            reg()
            node.resolve_blocks(sid[0], blocks)
            node.unregister_shuffle(sid[0])
        res["register_adopt_ms"] = t(lambda: (reg(), node.unregister_shuffle(sid[0])))
        res["full_ms"] = t(full)
        import ctypes as C
        addrs = (C.c_uint64 * len(blocks))()
        sizes = (C.c_int64 * len(blocks))()

        def raw_first():
            reg()
            t0 = time.perf_counter()
            N.check(node.lib.sux_resolve_blocks(node.h, sid[0], arr.ctypes.data, len(blocks), addrs, sizes), "r")
            t1 = time.perf_counter()
            N.check(node.lib.sux_resolve_blocks(node.h, sid[0], arr.ctypes.data, len(blocks), addrs, sizes), "r")
            t2 = time.perf_counter()
            node.unregister_shuffle(sid[0])
            return (t1 - t0) * 1e3, (t2 - t1) * 1e3
        r = [raw_first() for _ in range(5)]
        res["c_resolve_first_ms"] = min(x[0] for x in r)
        res["c_resolve_again_ms"] = min(x[1] for x in r)
        print(res)
        part.close()


if __name__ == "__main__":
    main()
    main(maps=1024, rpm=1024, R=10000, rs=16)
    main(maps=16384, rpm=64, R=10000, rs=16)
