"""Diagnose the N > 1 plugin path on one GPU (gloo + IPC bootstrap, every rank on cuda:0).

Each rank writes its map tasks group by group (sux_write_map_outputs, peer-major slabs),
exchanges window by window (sux_exchange_maps) and waits; then it fetches its owned range of
every map and compares each block with the same map partitioned locally (map-major
sux_partition_maps of the regenerated input of the map's owner), printing the first few
mismatching blocks: source rank, map, expected vs fetched size, first differing byte.
usage: python -m torch.distributed.run --nproc-per-node 8 tools/plugin_diag.py RPM GM GROUPS
       [serial]   (serial: exchange only after every write completed)
"""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from sparkucx_amd import native as N  # noqa: E402
from sparkucx_amd.shuffle import Node  # noqa: E402


def main():
    rpm, gm, groups = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
    serial = len(sys.argv) > 4 and sys.argv[4] == "serial"
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    R, rs, seed = 200, 100, 0x5EED0002
    n = groups * gm * rpm
    node = Node(device=0, rank=rank, world_size=world)
    node.set_bootstrap(lambda b: (lambda out: (dist.all_gather_object(out, b), out)[1])([None] * world))
    part = node.partitioner(N.PART_RANGE_BYTES, R, key_offset=0, key_len=10,
                            bounds=bench.uniform_bounds(R))
    data = node.generate(N.GEN_TERASORT, seed, rank * n, n, rs)
    torch.cuda.synchronize()
    sid, M = 9, groups * world * gm
    node.register_shuffle(sid, M, R, rs)
    xs = torch.cuda.Stream(dev)
    for g in range(groups):
        r0 = g * gm * rpm
        node.write_map_outputs(sid, (g * world + rank) * gm, part, data[r0 * rs:(r0 + gm * rpm) * rs],
                               rpm, gm * rpm)
        if g and not serial:
            node.exchange_maps(sid, (g - 1) * world * gm, world * gm, stream=xs)
    if serial:
        node.wait_map_outputs(sid)
        for g in range(groups - 1):
            node.exchange_maps(sid, g * world * gm, world * gm, stream=xs)
    node.exchange_maps(sid, (groups - 1) * world * gm, world * gm, stream=xs)
    node.exchange_wait(sid)
    torch.cuda.synchronize()
    lo, hi = node.owned_partitions(sid)
    bad = []
    for m in range(M):
        g, rem = divmod(m, world * gm)
        src, j = divmod(rem, gm)  # map m = (g * world + src) * gm + j
        first = src * n + (g * gm + j) * rpm
        recs = node.generate(N.GEN_TERASORT, seed, first, rpm, rs)
        out, index, _ = node.partition_maps(part, recs, rs, rpm)
        ix = index.cpu().numpy()
        want = out[ix[lo]:ix[hi]].cpu().numpy()
        buf, sizes = node.fetch_blocks(sid, [(m, lo, hi)])
        got = np.frombuffer(buf.to_bytes(), np.uint8)
        buf.release(1)
        if sizes[0] != len(want) or not np.array_equal(got, want):
            k = len(got) if len(got) != len(want) else int(np.argmax(got != want))
            nz = int((got != want).sum()) if len(got) == len(want) else -1
            bad.append((m, src, g, j, len(want), sizes[0], k, nz))
    # the bench's check: 64 maps per fetch, the pooled buffer copied device to device
    bad64 = []
    wants = {}
    for m in range(M):
        g, rem = divmod(m, world * gm)
        src, j = divmod(rem, gm)
        recs = node.generate(N.GEN_TERASORT, seed, src * n + (g * gm + j) * rpm, rpm, rs)
        out, index, _ = node.partition_maps(part, recs, rs, rpm)
        ix = index.cpu().numpy()
        wants[m] = out[ix[lo]:ix[hi]].cpu().numpy()
    for b0 in range(0, M, 64):
        ms = list(range(b0, min(M, b0 + 64)))
        buf, sizes = node.fetch_blocks(sid, [(m, lo, hi) for m in ms])
        ptr, size, _ = buf.info()
        t = torch.empty(max(4, size), dtype=torch.uint8, device=dev)
        if size:
            N.hip_memcpy(t.data_ptr(), ptr, size, N.HIP_D2D)
        buf.release(len(ms))
        got = t[:size].cpu().numpy()
        want = np.concatenate([wants[m] for m in ms])
        pos = 0
        for m, sz in zip(ms, sizes):
            if sz != len(wants[m]) or not np.array_equal(got[pos:pos + sz], wants[m]):
                bad64.append((m, sz, len(wants[m])))
            pos += sz
        if len(got) != len(want):
            bad64.append(("total", len(got), len(want)))
    print(f"rank {rank}: batched fetch: {len(bad64)} bad: {bad64[:4]}", flush=True)
    # the index file bytes each map's slot now serves (sux_map_output_index) vs the local ones
    badix = []
    for m in range(M):
        g, rem = divmod(m, world * gm)
        src, j = divmod(rem, gm)
        recs = node.generate(N.GEN_TERASORT, seed, src * n + (g * gm + j) * rpm, rpm, rs)
        out, index, index_be = node.partition_maps(part, recs, rs, rpm)
        got = node.map_output_index(sid, m, R)
        if got != index_be.cpu().numpy().tobytes():
            gi = np.frombuffer(got, ">i8")
            wi = index.cpu().numpy()
            k = int(np.argmax(gi != wi))
            badix.append((m, src, k, int(gi[k]), int(wi[k])))
    print(f"rank {rank}: map_output_index: {len(badix)} bad: {badix[:4]}", flush=True)
    # the bench's pid check (k_pids over the batched fetch)
    badpid = []
    for b0 in range(0, M, 64):
        ms = list(range(b0, min(M, b0 + 64)))
        buf, sizes = node.fetch_blocks(sid, [(m, lo, hi) for m in ms])
        ptr, size, _ = buf.info()
        t = torch.empty(max(4, size), dtype=torch.uint8, device=dev)
        if size:
            N.hip_memcpy(t.data_ptr(), ptr, size, N.HIP_D2D)
        buf.release(len(ms))
        t = t[:size]
        pid = node.partition_ids(part, t, rs).to(torch.int64)
        cnt = torch.tensor([sz // rs for sz in sizes], dtype=torch.int64, device=dev)
        seg = torch.repeat_interleave(torch.arange(len(ms), device=dev), cnt)
        inr = bool(((pid >= lo) & (pid < hi)).all())
        rise = bool(((pid[1:] >= pid[:-1]) | (seg[1:] != seg[:-1])).all())
        runs = torch.bincount(seg * (hi - lo) + (pid - lo), minlength=len(ms) * (hi - lo))
        want = []
        for m in ms:
            ix = np.frombuffer(node.map_output_index(sid, m, R), dtype=">i8").astype(np.int64)
            want.append((ix[lo + 1:hi + 1] - ix[lo:hi]) // rs)
        want = torch.from_numpy(np.concatenate(want)).to(dev)
        eq = torch.equal(runs, want)
        if not (inr and rise and eq):
            pid_ref = []
            badpid.append((b0, inr, rise, eq, int(pid.min()), int(pid.max()), runs.numel(), want.numel()))
    print(f"rank {rank}: pid check: {len(badpid)} bad: {badpid[:4]}", flush=True)
    print(f"rank {rank}: {len(bad)} of {M} maps differ; serial={serial}; first: "
          + "; ".join(f"map {m} (src {s}, group {g}, job {j}) want {w} B got {z} B first diff "
                      f"at {k}, {nz} bytes differ" for m, s, g, j, w, z, k, nz in bad[:4]),
          flush=True)
    node.unregister_shuffle(sid)
    dist.barrier()
    node.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
