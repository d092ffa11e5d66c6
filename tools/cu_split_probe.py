"""K1 (k_hist4) and K3 (k_scatter8) of one TeraSort launch group (32 maps x 2^20 records, R = 200)
on CU-masked streams of 256..32 CUs: do the two kernels scale with CUs (CU-bound) or hold their
rate on fewer CUs (HBM-bound)?  Decides whether K1 and K3 of consecutive groups could run side by
side on disjoint CU sets."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sparkucx_amd import native as N  # noqa: E402
from sparkucx_amd.shuffle import Node  # noqa: E402
from bench import uniform_bounds  # noqa: E402


def main():
    node = Node(device=0)
    R, rs, rpm, maps = 200, 100, 1 << 20, 32
    n = rpm * maps
    part = node.partitioner(N.PART_RANGE_BYTES, R, key_offset=0, key_len=10, bounds=uniform_bounds(R))
    data = node.generate(N.GEN_TERASORT, 0x5EED0002, 0, n, rs)
    out = torch.empty(n * rs, dtype=torch.uint8, device="cuda")
    index = torch.empty(maps * (R + 1), dtype=torch.int64, device="cuda")
    ws = torch.empty(node.workspace_size(part, rs, rpm, n), dtype=torch.uint8, device="cuda")
    node.set_kernel_timing(True)
    res = {}
    for cus in (256, 224, 192, 128, 96, 64, 32):
        if cus == 256:
            st = torch.cuda.current_stream()
        else:
            st = torch.cuda.ExternalStream(node.cu_stream(256 - cus, complement=True))
        for rep in range(4):
            if rep == 1:
                torch.cuda.synchronize()
                node.kernel_times()  # (reading resets nothing; take differences)
                t0 = node.kernel_times()
            node.partition_maps(part, data, rs, rpm, num_records=n, out=out, index=index,
                                workspace=ws, want_be=False, stream=st)
        torch.cuda.synchronize()
        t1 = node.kernel_times()
        d = {k: (t1[k][1] - t0[k][1]) / max(1, t1[k][0] - t0[k][0]) for k in ("hist", "scatter")}
        res[cus] = {"k1_ms": round(d["hist"], 4), "k3_ms": round(d["scatter"], 4),
                    "k1_TBps": round(n * rs / d["hist"] / 1e9, 2),
                    "k3_TBps": round(2 * n * rs / d["scatter"] / 1e9, 2)}
        print(cus, res[cus], flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
