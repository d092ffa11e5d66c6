"""LZ4 compressor A/B on the bench's compress leg: 32 TeraSort map outputs (2^20 records, R = 200)
compressed under tuning lz4_queue A and B, alternating, `reps` times each (the leg decodes and
checks every stream).  usage: python tools/lz4_ab.py [A=1] [B=3] [reps=2] [block_size=32768]
Prints one JSON line per run."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from sparkucx_amd import native as N  # noqa: E402
from sparkucx_amd.shuffle import Node  # noqa: E402


def main():
    a = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    b = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    bs = int(sys.argv[4]) if len(sys.argv) > 4 else 32768
    dev = torch.device("cuda", 0)
    node = Node(device=0)
    maps, rpm, rs, R = 32, 1 << 20, 100, 200
    n = maps * rpm
    recs = node.generate(N.GEN_TERASORT, 0x5EED0007, 0, n, rs)
    bounds = b"".join(((k + 1) * (1 << 80) // R).to_bytes(10, "big") for k in range(R - 1))
    part = node.partitioner(N.PART_RANGE_BYTES, R, key_offset=0, key_len=10, bounds=bounds)
    out, index, _ = node.partition_maps(part, recs, rs, rpm)
    torch.cuda.synchronize()
    for _ in range(reps):
        for q in (a, b):
            node.set_tuning(lz4_queue=q)
            r = bench.compress_leg(node, out, index, maps, R, dev, bs)
            print(json.dumps({"lz4_queue": q, "block_size": bs, "GB/s": r["GB/s"], "ms": r["ms"],
                              "ratio": r["ratio"], "decompress_GB/s": r["decompress"]["GB/s"]}),
                  flush=True)
    part.close()
    node.close()


if __name__ == "__main__":
    main()
