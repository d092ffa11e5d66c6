"""Multi-process GPU check of the shuffle-level exchange (run by tests/test_gpu_shuffle_exchange.py):

    python -m torch.distributed.run --nproc-per-node W --master-addr 127.0.0.1 \
        --master-port P tests/gpu_shuffle_exchange_check.py --workload terasort|zipf

W executors share cuda:0 (RCCL refuses two ranks on one device), so the node gets no RCCL
communicator and the exchange runs over the bootstrap transport: the directory of committed maps
travels through a host all-gather (gloo here; Spark RPC in a JVM) and every rank PULLS its
partitions from the owners' IPC-mapped map outputs.  The flow is the plugin's:
registerShuffle -> getWriter(...).write for this executor's map tasks (one batched
sux_write_map_outputs) -> sux_exchange -> UcxShuffleClient.fetchBlocks of one ShuffleBlockBatchId
per map for this rank's partitions.  Every fetched block is compared with the CPU oracle's map
output, regenerated on every rank from the counter-based generator.
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
    a = ap.parse_args()
    dist.init_process_group("gloo")
    rank, W = dist.get_rank(), dist.get_world_size()
    R, M, rpm, seed = a.R, a.maps, a.rpm, 0x5EED0007

    node = Node(device=0, rank=rank, world_size=W)

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
    # this executor runs map tasks [m0, m1) (uneven split when W does not divide M)
    m0, m1 = (rank * M) // W, ((rank + 1) * M) // W
    if m1 > m0:
        recs = node.generate(gen_kind, seed, m0 * rpm, (m1 - m0) * rpm, 100)
        node.write_map_outputs(sid, m0, part, recs, rpm, (m1 - m0) * rpm)
    node.exchange(sid)

    lo, hi = node.owned_partitions(sid)
    blocks = [(m, lo, hi) for m in range(M)]  # ShuffleBlockBatchId per map
    buf, sizes = node.fetch_blocks(sid, blocks)
    got = np.frombuffer(buf.to_bytes(), np.uint8)
    buf.release(len(blocks))

    pos, hot = 0, 0
    for m in range(M):
        d, lengths, ix, _ = O.write_map(opart, ogen(seed, m * rpm, rpm), 100)
        want = d[ix[lo]:ix[hi]]
        assert sizes[m] == len(want), (rank, m, sizes[m], len(want))
        assert got[pos:pos + len(want)].tobytes() == want.tobytes(), (rank, m)
        pos += len(want)
        hot = max(hot, int(lengths.max()))
    assert pos == got.size
    dist.barrier()
    node.unregister_shuffle(sid)
    node.close()
    if rank == 0:
        print(f"shuffle exchange ok: workload={a.workload} world={W} maps={M} R={R} "
              f"hot partition {hot} B of a {rpm * 100} B map", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
