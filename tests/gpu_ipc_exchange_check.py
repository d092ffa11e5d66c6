"""Multi-process GPU exchange over HIP IPC (run by tests/test_gpu_ipc_exchange.py):

    python -m torch.distributed.run --nproc-per-node W --master-addr 127.0.0.1 \
        --master-port P tests/gpu_ipc_exchange_check.py

W processes share cuda:0 (the box has one GPU; RCCL refuses two ranks on one device, HIP IPC does
not).  Each rank partitions its own map batches peer-major on the GPU, exports its send buffer's
IPC handle (the rkey analog), all-gathers the index tables (gloo), then PULLS its partitions from
every rank's send buffer with sux_pull_group — the device-side planner + one-sided GET copy —
and checks every received (source, map, partition) block against the CPU oracle.
"""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import oracle as O  # noqa: E402
from sparkucx_amd import native as N  # noqa: E402
from sparkucx_amd.shuffle import Node  # noqa: E402


def main():
    dist.init_process_group("gloo")
    rank, W = dist.get_rank(), dist.get_world_size()
    R, M, rpm = 200, 3, 20000
    node = Node(device=0)
    opart = O.terasort_partitioner(R)
    part = node.partitioner(N.PART_RANGE_BYTES, R, key_offset=0, key_len=10, bounds=opart.bounds)
    seed = 20 + rank
    recs = node.generate(N.GEN_TERASORT, seed, 0, M * rpm, 100)
    send, index, peer = node.partition_maps_peer_major(part, recs, 100, rpm, W)
    torch.cuda.synchronize()

    # rkey analog: every rank maps every other rank's send buffer
    handles = [None] * W
    dist.all_gather_object(handles, node.ipc_handle(send))
    ptrs = [send.data_ptr() if g == rank else node.ipc_open(handles[g]) for g in range(W)]
    # driver-table analog: all-gather the index tables
    idx = index.cpu()
    gathered = [torch.empty_like(idx) for _ in range(W)]
    dist.all_gather(gathered, idx)
    gi = torch.stack(gathered).reshape(-1).cuda()
    dist.barrier()  # every rank's partition step has completed (synchronized above)

    cap = int(M * rpm * 100 * 1.5)
    recv = torch.empty(cap, dtype=torch.uint8, device="cuda")
    rb = torch.zeros(1, dtype=torch.int64, device="cuda")
    src = torch.tensor(ptrs, dtype=torch.int64, device="cuda")
    node.pull_group(W, rank, src, gi, M, R, recv, rb)
    torch.cuda.synchronize()
    got = recv.cpu().numpy()
    total = int(rb.item())

    gnp = np.ascontiguousarray(torch.stack(gathered).numpy())
    lib = N.load()
    lo, hi = (rank * R) // W, ((rank + 1) * R) // W
    want_total = 0
    for g in range(W):
        grecs = O.gen_terasort(20 + g, 0, M * rpm)
        for m in range(M):
            d, _, ix, _ = O.write_map(opart, grecs[m * rpm * 100:(m + 1) * rpm * 100], 100)
            for p in range(lo, hi):
                off = lib.sux_plan_block_offset(W, rank, M, R, gnp.ctypes.data, g, m, p)
                want = d[ix[p]:ix[p + 1]]
                assert got[off:off + len(want)].tobytes() == want.tobytes(), (rank, g, m, p)
                want_total += len(want)
    assert total == want_total, (total, want_total)
    dist.barrier()  # peers are done reading my send buffer
    for g in range(W):
        if g != rank:
            node.ipc_close(ptrs[g])
    node.close()
    if rank == 0:
        print(f"ipc exchange ok: world={W} bytes/rank~{want_total}", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
