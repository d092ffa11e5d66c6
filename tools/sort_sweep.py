"""Reduce-side sort timing for the digit-width sweep (run once per SUX_SORT_MAX_DIGIT_BITS value:
the library reads it once per process).  TeraSort 10-byte keys (5 M x 100 B, one reduce
partition of the bench) and int64 keys (32 Mi x 16 B, full range and [0, 2^31))."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sparkucx_amd import native as N  # noqa: E402
from sparkucx_amd.shuffle import Node  # noqa: E402


def timed(node, recs, n, rs, kind, off, klen, reps=10):
    out = torch.empty(n * rs, dtype=torch.uint8, device="cuda")
    ws = torch.empty(node.sort_workspace_size(n, rs), dtype=torch.uint8, device="cuda")
    for _ in range(2):
        node.sort_records(recs, rs, kind, off, klen, num_records=n, out=out, workspace=ws)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        node.sort_records(recs, rs, kind, off, klen, num_records=n, out=out, workspace=ws)
    e1.record()
    torch.cuda.synchronize()
    return round(e0.elapsed_time(e1) / reps, 3)


def main():
    node = Node(device=0)
    res = {"max_digit_bits": os.environ.get("SUX_SORT_MAX_DIGIT_BITS", "default")}
    n = 5_000_000
    d = node.generate(N.GEN_TERASORT, 25, 0, n, 100)
    res["terasort_5M_ms"] = timed(node, d, n, 100, N.SORT_BYTES, 0, 10)
    del d
    ns = 32 << 20
    g = torch.Generator(device="cuda")
    g.manual_seed(5)
    for name, hi in [("long_full_32M_ms", None), ("long_2e31_32M_ms", 1 << 31)]:
        rows = torch.empty((ns, 2), dtype=torch.int64, device="cuda")
        if hi is None:
            rows[:, 0] = torch.randint(-(1 << 62), 1 << 62, (ns,), generator=g, device="cuda")
        else:
            rows[:, 0] = torch.randint(0, hi, (ns,), generator=g, device="cuda")
        rows[:, 1] = torch.arange(ns, device="cuda")
        res[name] = timed(node, rows.view(torch.uint8).view(-1), ns, 16, N.SORT_LONG, 0, 8)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
