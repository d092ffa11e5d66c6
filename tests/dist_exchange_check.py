"""Multi-process exchange check (CPU, gloo).  Launched by tests/test_exchange_gloo.py as

    python -m torch.distributed.run --nproc-per-node W --master-addr 127.0.0.1 \
        --master-port P tests/dist_exchange_check.py [--maps M --rpm N --R R]

Every rank plays one GPU of the node: it lays out its map outputs peer-major (the oracle of
sux_partition_maps_peer_major), all-gathers the index tables, plans the all-to-all with the
library's host planner (sux_plan_group — the code sux_exchange_group runs before
ncclAllToAllv), exchanges with all_to_all_single, and checks every received (source, map,
partition) block against the oracle's map output, located with sux_plan_block_offset.
Exit code 0 = all blocks bit-exact.
"""
import argparse
import ctypes as C
import hashlib
import json
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import oracle as O  # noqa: E402
from sparkucx_amd import native as N  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--maps", type=int, default=3)
    ap.add_argument("--rpm", type=int, default=500)
    ap.add_argument("--R", type=int, default=8)
    ap.add_argument("--golden", default="")
    ap.add_argument("--zipf", action="store_true",
                    help="Zipf(1.1) int64 keys, Spark SQL murmur3 partitioner (C4's shape)")
    ap.add_argument("--balanced", action="store_true",
                    help="ownership balanced by the all-reduced partition bytes "
                         "(sux_plan_ownership) instead of the equal split")
    a = ap.parse_args()
    dist.init_process_group("gloo")
    rank, W = dist.get_rank(), dist.get_world_size()
    R, M, rpm = a.R, a.maps, a.rpm
    if a.zipf:
        part = O.Partitioner(O.MURMUR3_LONG, R, 0, 8, 42)
        gen = lambda g: O.gen_zipf(11, g * M * rpm, M * rpm)  # noqa: E731
    else:
        part = O.terasort_partitioner(R)
        gen = lambda g: O.gen_terasort(11 + g, 0, M * rpm)  # noqa: E731
    recs = gen(rank)
    own = np.array([(h * R) // W for h in range(W + 1)], np.int32)
    if a.balanced:
        # partition bytes of every rank's maps, summed over ranks -> the balanced ownership
        lens = np.zeros(R, np.int64)
        for m0 in range(0, M * rpm, rpm):
            lens += np.asarray(O.write_map(part, recs[m0 * 100:(m0 + rpm) * 100], 100)[1])
        t = torch.from_numpy(lens * 100)
        dist.all_reduce(t)
        own = N.plan_ownership(W, t.numpy())
        assert own.tolist() == O.plan_ownership(W, t.numpy())
    send, index, peer_bytes = O.peer_major(part, recs, 100, rpm, W, own=own)

    # 1. all-gather the index tables (replaces the driver metadata table + phase-1 GETs)
    idx = torch.from_numpy(index.astype(np.int64))
    gathered = [torch.empty_like(idx) for _ in range(W)]
    dist.all_gather(gathered, idx)
    gi = np.ascontiguousarray(torch.stack(gathered).numpy().reshape(W, M, R + 1))

    # 2. plan with the library's host planner
    lib = N.load()
    sc, sd, rc, rd = [(C.c_uint64 * W)() for _ in range(4)]
    assert lib.sux_plan_group_owned(W, rank, M, R, gi.ctypes.data, own.ctypes.data,
                                    sc, sd, rc, rd) == 0, N.last_error()
    assert list(sc) == peer_bytes.tolist(), (list(sc), peer_bytes.tolist())
    assert list(sd) == np.concatenate([[0], np.cumsum(peer_bytes)[:-1]]).tolist()

    # 3. the exchange itself (gloo here; ncclAllToAllv over xGMI on the GPUs)
    recv = torch.empty(int(sum(rc)), dtype=torch.uint8)
    dist.all_to_all_single(recv, torch.from_numpy(send.copy()), list(rc), list(sc))
    rbuf = recv.numpy()

    # 4. every block this rank owns, from every source map, bit-exact
    lo, hi = int(own[rank]), int(own[rank + 1])
    blocks = {}
    for g in range(W):
        grecs = gen(g)
        for m in range(M):
            d, _, ix, _ = O.write_map(part, grecs[m * rpm * 100:(m + 1) * rpm * 100], 100)
            for p in range(lo, hi):
                off = lib.sux_plan_block_offset_owned(W, rank, M, R, gi.ctypes.data,
                                                      own.ctypes.data, g, m, p)
                assert off >= 0
                want = d[ix[p]:ix[p + 1]]
                got = rbuf[off:off + len(want)]
                assert got.tobytes() == want.tobytes(), (rank, g, m, p)
                blocks[f"{m}_{p}"] = blocks.get(f"{m}_{p}", []) + [
                    hashlib.sha256(want.tobytes()).hexdigest()]
    if a.golden:
        with open(a.golden) as f:
            gold = json.load(f)
        for g in range(W):
            for m in range(M):
                for p in range(lo, hi):
                    assert blocks[f"{m}_{p}"][g] == gold["ranks"][g]["blocks"][f"{m}_{p}"]
    dist.barrier()
    # received bytes per rank: max over mean (what the exchange's busiest owner carries)
    ing = torch.tensor([float(sum(rc))])
    mx, tot = ing.clone(), ing.clone()
    dist.all_reduce(mx, op=dist.ReduceOp.MAX)
    dist.all_reduce(tot)
    if rank == 0:
        print(f"exchange ok: world={W} maps={M} R={R} ownership={own.tolist()} "
              f"ingress max/mean={float(mx) / (float(tot) / W):.3f}", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
