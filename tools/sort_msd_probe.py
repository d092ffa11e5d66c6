"""What would a record-moving MSD sort of a reduce partition cost?

The reduce sort's first pass, done the record-moving way, is exactly a range partition of the
partition's records into R buckets over its key span: this probe times the library's own map-side
kernels (K1 histogram + scan + K3 line-image scatter, sux_partition_maps) doing that on a reduce
partition's worth of TeraSort records (5 M x 100 B, keys of one reduce partition: a fixed top
byte), for R = 1024 .. 8192 buckets, beside today's sux_sort_records on the same records.  The
second pass (each bucket sorted in LDS and written out) would move the records once more, so the
first pass alone must beat ~half of today's sort for the design to pay.

usage: python tools/sort_msd_probe.py [records=5000000]
Prints one JSON line per measurement.
"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sparkucx_amd import native as N  # noqa: E402
from sparkucx_amd.shuffle import Node  # noqa: E402


def timed(fn, reps=5):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 5_000_000
    rs = 100
    node = Node(device=0)
    recs = node.generate(N.GEN_TERASORT, 0x5EED0002, 0, n, rs)
    recs.view(n, rs)[:, 0] = 0x80  # one reduce partition's keys: a narrow span
    keys = recs.view(n, rs)[:, :10].cpu().numpy()
    kint = [int.from_bytes(k.tobytes(), "big") for k in (keys.min(0), keys.max(0))]
    # (the min / max rows above are per byte, a loose span: enough for uniform buckets)
    lo, hi = kint
    out = torch.empty(n * rs, dtype=torch.uint8, device="cuda")
    ws = torch.empty(node.sort_workspace_size(n, rs), dtype=torch.uint8, device="cuda")
    ms = timed(lambda: node.sort_records(recs, rs, N.SORT_BYTES, 0, 10, num_records=n, out=out,
                                         workspace=ws))
    print(json.dumps({"what": "sux_sort_records", "records": n, "ms": round(ms, 4),
                      "GB/s": round(n * rs / ms / 1e6, 1)}), flush=True)
    for R in (1024, 2048, 4096, 8192):
        bounds = b"".join((lo + (hi - lo) * (k + 1) // R).to_bytes(10, "big") for k in range(R - 1))
        part = node.partitioner(N.PART_RANGE_BYTES, R, key_offset=0, key_len=10, bounds=bounds)
        for rpm in (n, 1 << 20):
            maps = -(-n // rpm)
            idx = torch.empty(maps * (R + 1), dtype=torch.int64, device="cuda")
            wsp = torch.empty(node.workspace_size(part, rs, rpm, n), dtype=torch.uint8,
                              device="cuda")
            node.set_kernel_timing(True)
            node.kernel_times()
            ms = timed(lambda: node.partition_maps(part, recs, rs, rpm, num_records=n, out=out,
                                                   index=idx, want_be=False, workspace=wsp))
            kt = node.kernel_times()
            node.set_kernel_timing(False)
            names = [node.kernel_variant(i) for i in range(3)]
            sizes = np.diff(idx.view(maps, R + 1).cpu().numpy(), axis=1).sum(0) // rs
            print(json.dumps({"what": "range partition over the key span", "R": R,
                              "records_per_map": rpm, "ms": round(ms, 4),
                              "kernels": names,
                              "kernel_ms_per_call": {k: round(v[1] / max(1, v[0]), 4)
                                                     for k, v in kt.items()},
                              "bucket_records_max": int(sizes.max()),
                              "bucket_records_mean": round(float(sizes.mean()), 1)}),
                  flush=True)
        part.close()
    node.close()


if __name__ == "__main__":
    main()
