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
    a = ap.parse_args()
    dist.init_process_group("gloo")
    rank, W = dist.get_rank(), dist.get_world_size()
    R, M, rpm = a.R, a.maps, a.rpm
    part = O.terasort_partitioner(R)
    seed = 11 + rank
    recs = O.gen_terasort(seed, 0, M * rpm)
    send, index, peer_bytes = O.peer_major(part, recs, 100, rpm, W)

    # 1. all-gather the index tables (replaces the driver metadata table + phase-1 GETs)
    idx = torch.from_numpy(index.astype(np.int64))
    gathered = [torch.empty_like(idx) for _ in range(W)]
    dist.all_gather(gathered, idx)
    gi = np.ascontiguousarray(torch.stack(gathered).numpy().reshape(W, M, R + 1))

    # 2. plan with the library's host planner
    lib = N.load()
    sc, sd, rc, rd = [(C.c_uint64 * W)() for _ in range(4)]
    assert lib.sux_plan_group(W, rank, M, R, gi.ctypes.data, sc, sd, rc, rd) == 0, N.last_error()
    assert list(sc) == peer_bytes.tolist(), (list(sc), peer_bytes.tolist())
    assert list(sd) == np.concatenate([[0], np.cumsum(peer_bytes)[:-1]]).tolist()

    # 3. the exchange itself (gloo here; ncclAllToAllv over xGMI on the GPUs)
    recv = torch.empty(int(sum(rc)), dtype=torch.uint8)
    dist.all_to_all_single(recv, torch.from_numpy(send.copy()), list(rc), list(sc))
    rbuf = recv.numpy()

    # 4. every block this rank owns, from every source map, bit-exact
    lo, hi = (rank * R) // W, ((rank + 1) * R) // W
    blocks = {}
    for g in range(W):
        grecs = O.gen_terasort(11 + g, 0, M * rpm)
        for m in range(M):
            d, _, ix, _ = O.write_map(part, grecs[m * rpm * 100:(m + 1) * rpm * 100], 100)
            for p in range(lo, hi):
                off = lib.sux_plan_block_offset(W, rank, M, R, gi.ctypes.data, g, m, p)
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
    if rank == 0:
        print(f"exchange ok: world={W} maps={M} R={R}", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
