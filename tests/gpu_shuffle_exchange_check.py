"""Multi-process GPU check of the shuffle-level exchange (run by tests/test_gpu_shuffle_exchange.py):

    python -m torch.distributed.run --nproc-per-node W --master-addr 127.0.0.1 \
        --master-port P tests/gpu_shuffle_exchange_check.py --workload terasort|zipf \
        [--windows K] [--batch-maps B] [--loopback]

W executors share cuda:0 (RCCL refuses two ranks on one device), so the node gets no RCCL
communicator and the exchange runs over the bootstrap transport: the directory of committed maps
travels through a host all-gather (gloo here; Spark RPC in a JVM) and every rank PULLS its
partitions from the owners' IPC-mapped batch slabs, following the same per-round plan the RCCL
transport feeds to ncclAllToAllv.  The flow is the plugin's: registerShuffle -> getWriter(...).write
for this executor's map tasks (sux_write_map_outputs batches: at W > 1 each batch slab is
peer-major) -> the exchange -> UcxShuffleClient.fetchBlocks.

--windows K: the maps form K windows (every window holds maps of every rank); window k+1's
writes are enqueued BEFORE window k's sux_exchange_maps, so the exchange of one window overlaps
the next window's map kernels (the bounded in-flight window of UcxShuffleReader.scala:56-70);
one sux_exchange_wait at the end.  --batch-maps B: an executor writes its maps of a window in
batches of B (several pieces -> several all-to-all rounds).  --loopback: own maps also travel
through the transport (tuning exchange_self).  Every fetched block is compared with the CPU
oracle's map output, regenerated on every rank from the counter-based generator: this rank's
partitions of every map (ShuffleBlockBatchId per map), single ShuffleBlockIds of its OWN maps in
other ranks' ranges (served from the peer-major slab segments), and another rank's whole range of
a few maps (a peer read from where that rank serves it: a reduce task scheduled off its owner).
"""
import argparse
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import oracle as O  # noqa: E402  (test infrastructure: the checker)
from sparkucx_amd import native as N  # noqa: E402
from sparkucx_amd.shuffle import Node  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="terasort", choices=["terasort", "zipf"])
    ap.add_argument("--maps", type=int, default=12)
    ap.add_argument("--rpm", type=int, default=20000)
    ap.add_argument("--R", type=int, default=200)
    ap.add_argument("--windows", type=int, default=1)
    ap.add_argument("--batch-maps", type=int, default=0)
    ap.add_argument("--loopback", action="store_true")
    a = ap.parse_args()
    dist.init_process_group("gloo")
    rank, W = dist.get_rank(), dist.get_world_size()
    R, M, rpm, seed = a.R, a.maps, a.rpm, 0x5EED0007

    node = Node(device=0, rank=rank, world_size=W)
    if a.loopback:
        node.set_tuning(exchange_self=1)

    def allgather(b: bytes):
        out = [None] * W
        dist.all_gather_object(out, b)
        return out

    node.set_bootstrap(allgather)
    if a.workload == "terasort":
        opart = O.terasort_partitioner(R)
        part = node.partitioner(N.PART_RANGE_BYTES, R, key_offset=0, key_len=10, bounds=opart.bounds)
        gen_kind, ogen = N.GEN_TERASORT, O.gen_terasort
    else:  # Spark SQL hash of a Zipf(1.1) int64 key: a hot partition far above the mean
        opart = O.Partitioner(O.MURMUR3_LONG, R, 0, 8, 42)
        part = node.partitioner(N.PART_MURMUR3_LONG, R, key_offset=0, key_len=8, seed=42)
        gen_kind, ogen = N.GEN_ZIPF, O.gen_zipf

    sid = 3
    node.register_shuffle(sid, M, R, 100)
    K = max(1, a.windows)
    win = [((k * M) // K, ((k + 1) * M) // K) for k in range(K)]
    keep = []  # generated inputs stay alive until their writes ran

    def write_window(k):
        w0, w1 = win[k]
        # this executor runs map tasks [m0, m1) of the window (uneven when W does not divide it)
        m0, m1 = w0 + (rank * (w1 - w0)) // W, w0 + ((rank + 1) * (w1 - w0)) // W
        B = a.batch_maps if a.batch_maps > 0 else max(1, m1 - m0)
        for b0 in range(m0, m1, B):
            b1 = min(m1, b0 + B)
            recs = node.generate(gen_kind, seed, b0 * rpm, (b1 - b0) * rpm, 100)
            keep.append(recs)
            node.write_map_outputs(sid, b0, part, recs, rpm, (b1 - b0) * rpm)
        return list(range(m0, m1))

    mine = write_window(0)
    for k in range(K):
        if k + 1 < K:
            mine += write_window(k + 1)  # next window's kernels run under this window's exchange
        node.exchange_maps(sid, win[k][0], win[k][1] - win[k][0])
    node.exchange_wait(sid)

    lo, hi = node.owned_partitions(sid)
    blocks = [(m, lo, hi) for m in range(M)]  # ShuffleBlockBatchId per map
    rng = np.random.default_rng(rank)
    others = [p for p in range(R) if not lo <= p < hi]
    own_single = [(m, int(rng.choice(others))) for m in mine] if others else []
    # another rank's whole range of a few maps it does not own either: read from where that
    # rank serves it (its receive buffer or batch slab, IPC-mapped: a peer read)
    h2 = (rank + 1) % W
    lo2, hi2 = node.owned_partitions(sid, h2)
    remote = [(m, lo2, hi2) for m in rng.choice(M, size=min(3, M), replace=False).tolist()] \
        if W > 1 else []
    req = blocks + [(m, p, p + 1) for m, p in own_single] + remote
    buf, sizes = node.fetch_blocks(sid, req)
    got = np.frombuffer(buf.to_bytes(), np.uint8)
    buf.release(len(req))

    pos, hot = 0, 0
    outs = {}
    for m in range(M):
        d, lengths, ix, _ = O.write_map(opart, ogen(seed, m * rpm, rpm), 100)
        outs[m] = (d, ix)
        want = d[ix[lo]:ix[hi]]
        assert sizes[m] == len(want), (rank, m, sizes[m], len(want))
        assert got[pos:pos + len(want)].tobytes() == want.tobytes(), (rank, m)
        pos += len(want)
        hot = max(hot, int(lengths.max()))
    for i, (m, p) in enumerate(own_single):
        d, ix = outs[m]
        want = d[ix[p]:ix[p + 1]]
        assert sizes[M + i] == len(want), (rank, m, p)
        assert got[pos:pos + len(want)].tobytes() == want.tobytes(), (rank, m, p)
        pos += len(want)
    for i, (m, a_, b_) in enumerate(remote):
        d, ix = outs[m]
        want = d[ix[a_]:ix[b_]]
        k = M + len(own_single) + i
        assert sizes[k] == len(want), ("remote", rank, m, a_, b_)
        assert got[pos:pos + len(want)].tobytes() == want.tobytes(), ("remote", rank, m)
        pos += len(want)
    assert pos == got.size
    node.check()
    dist.barrier()
    node.unregister_shuffle(sid)
    node.close()
    if rank == 0:
        print(f"shuffle exchange ok: workload={a.workload} world={W} maps={M} R={R} windows={K} "
              f"batch_maps={a.batch_maps} loopback={a.loopback} "
              f"hot partition {hot} B of a {rpm * 100} B map", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
