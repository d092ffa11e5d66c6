"""Reduce-side sort A/B over the record-gather variants (tuning gather_kernel 1 = own launch,
16-byte units; 3 = fused into the LDS bucket sort): 5 M TeraSort records (one reduce partition of
the bench), plus key sets that exercise the fused sort's leftovers (a heavy hitter above the LDS
cap; keys varying only in the top digit).  Outputs of every variant must be byte-equal."""
import json
import os
import sys

import torch

sys.path.insert(0, os.environ.get("SUX_PKG_ROOT") or os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sparkucx_amd import native as N  # noqa: E402
from sparkucx_amd.shuffle import Node  # noqa: E402


def run(node, recs, n, rs, kind, off, klen, reps):
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
    node.check()
    return round(e0.elapsed_time(e1) / reps, 4), out


def main():
    node = Node(device=0)
    reps = int(os.environ.get("REPS", "20"))
    n = 5_000_000
    cases = {}
    d = node.generate(N.GEN_TERASORT, 25, 0, n, 100)
    cases["terasort_5M"] = (d, n, 100, N.SORT_BYTES, 0, 10)
    hh = node.generate(N.GEN_TERASORT, 26, 0, n, 100).view(n, 100).clone()
    hh[: n // 10, :10] = hh[0, :10]  # 500 000 equal keys: one bucket far above the LDS cap
    cases["heavy_hitter_5M"] = (hh.view(-1), n, 100, N.SORT_BYTES, 0, 10)
    lc = node.generate(N.GEN_TERASORT, 28, 0, n, 100).view(n, 100).clone()
    pick = torch.randint(0, 100, (n,), device="cuda", generator=torch.Generator(device="cuda").manual_seed(3))
    lc[:, :10] = lc[:100, :10][pick]  # 100 distinct keys: buckets of ~50 000 equal keys each
    cases["distinct100_5M"] = (lc.view(-1), n, 100, N.SORT_BYTES, 0, 10)
    tk = node.generate(N.GEN_TERASORT, 27, 0, n, 100).view(n, 100).clone()
    tk[:, 1:10] = 0  # keys vary in their first byte only: the top pass finishes the sort
    cases["top_digit_only_5M"] = (tk.view(-1), n, 100, N.SORT_BYTES, 0, 10)
    ns = 32 << 20  # the bench's reduce_sort_long: int64 keys in [0, 2^31) + int64 values
    g = torch.Generator(device="cuda")
    g.manual_seed(5)
    rows = torch.empty((ns, 2), dtype=torch.int64, device="cuda")
    rows[:, 0] = torch.randint(0, 1 << 31, (ns,), generator=g, device="cuda")
    rows[:, 1] = torch.arange(ns, device="cuda")
    cases["long_2e31_32M"] = (rows.view(torch.uint8).view(-1), ns, 16, N.SORT_LONG, 0, 8)
    res = {}
    only = os.environ.get("CASES")
    for name, (recs, nn, rs, kind, off, klen) in cases.items():
        if only and name not in only.split(","):
            continue
        outs = {}
        for gk in [int(g) for g in os.environ.get("GK", "1,3").split(",")]:
            node.set_tuning(gather_kernel=gk)
            ms, out = run(node, recs, nn, rs, kind, off, klen, reps)
            res[f"{name}_gk{gk}_ms"] = ms
            outs[gk] = out
        if 1 in outs and 3 in outs:
            res[f"{name}_equal"] = bool(torch.equal(outs[1], outs[3]))
        for gk in outs:  # records moved per ms, the bench's reduce_sort GB/s
            res[f"{name}_GB/s_gk{gk}"] = round(nn * rs / res[f"{name}_gk{gk}_ms"] / 1e6, 1)
        del outs
    node.set_tuning(gather_kernel=0)
    print(json.dumps(res))
    if not all(v for k, v in res.items() if k.endswith("_equal")):
        sys.exit(1)


if __name__ == "__main__":
    main()
