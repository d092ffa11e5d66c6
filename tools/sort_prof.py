"""The reduce-side sort alone, for a kernel-trace profile: 5 M TeraSort records (one reduce
partition of the bench), `reps` timed calls after two warm-ups; prints the HIP-event mean.
With SORT_PROF_INPUT=partition the keys are those of one range partition of 200 (TeraSort's
uniform bounds, partition 100: the first key byte 0x80 or, for 22 % of the keys, 0x81 with the
second byte below 0x47), the shape of the bench's reduce_sort leg.
SORT_PROF_N=<records> changes the record count (TeraSort inputs).
usage: python tools/sort_prof.py [reps=20] [tuning field=value,...] [library path (A/B builds)]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sparkucx_amd import native as N  # noqa: E402
from sparkucx_amd.shuffle import Node  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    if len(sys.argv) > 3:
        N.LIB_PATH = os.path.abspath(sys.argv[3])
    node = Node(device=0)
    if len(sys.argv) > 2 and sys.argv[2]:
        node.set_tuning(**{k: int(v) for k, v in (kv.split("=") for kv in sys.argv[2].split(","))})
    n, rs = int(os.environ.get("SORT_PROF_N", 5_000_000)), 100
    kind, klen = N.SORT_BYTES, 10
    if os.environ.get("SORT_PROF_INPUT") == "long":  # bench.py reduce_sort_long's 32 Mi rows
        n, rs, kind, klen = 32 << 20, 16, N.SORT_LONG, 8
        g = torch.Generator(device="cuda")
        g.manual_seed(5)
        rows = torch.empty((n, 2), dtype=torch.int64, device="cuda")
        rows[:, 0] = torch.randint(0, 1 << 31, (n,), generator=g, device="cuda")
        rows[:, 1] = torch.arange(n, device="cuda")
        d = rows.view(torch.uint8).view(-1)
    else:
        d = node.generate(N.GEN_TERASORT, 25, 0, n, rs)
    if os.environ.get("SORT_PROF_INPUT") == "partition":
        v = d.view(n, rs)
        g = torch.Generator(device="cuda")
        g.manual_seed(5)
        hi = torch.rand(n, device="cuda", generator=g) < 0.22
        v[:, 0] = torch.where(hi, 0x81, 0x80).to(torch.uint8)
        b1 = torch.randint(0, 0x47, (n,), device="cuda", generator=g, dtype=torch.int32)
        v[:, 1] = torch.where(hi, b1.to(torch.uint8), v[:, 1])  # uniform, no modulo bias
    out = torch.empty(n * rs, dtype=torch.uint8, device="cuda")
    ws = torch.empty(node.sort_workspace_size(n, rs), dtype=torch.uint8, device="cuda")
    for _ in range(2):
        node.sort_records(d, rs, kind, 0, klen, num_records=n, out=out, workspace=ws)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        node.sort_records(d, rs, kind, 0, klen, num_records=n, out=out, workspace=ws)
    e1.record()
    torch.cuda.synchronize()
    node.check()
    print(f"sort {n} x {rs} B ({os.environ.get('SORT_PROF_INPUT', 'random')} keys): "
          f"{e0.elapsed_time(e1) / reps:.4f} ms per call ({N.LIB_PATH})", flush=True)


if __name__ == "__main__":
    main()
