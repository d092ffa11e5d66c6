"""bench.py — shuffle GB/s/node (partition + exchange), TeraSort 100-byte records.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload terasort|zipf|small]
    torchrun --nproc-per-node N bench.py --gpus N ...      (one rank per GPU, RCCL over xGMI)

A step = one full shuffle of the rank's resident input: every map batch is partitioned by the
gfx950 kernels (P1-P3) and, for N > 1, its partition-aligned share is exchanged with every other
GPU (RCCL grouped send/recv, overlapped with the next launch group on a second stream).  At N = 1
the reduce side resolves its blocks zero-copy from the index tables (no bytes move), and the line
also carries BASELINE configs C4 (Zipf keys) and C5 (16-byte records, R = 10 000) as `c4` / `c5`.
Inputs are generated on the device before timing (counter-based) and stay in HBM.

value = input bytes of all ranks / max-over-ranks wall time of K steps, in GB/s (1e9 B/s).
Rank 0 prints ONE JSON line; everything else goes to stderr.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import threading
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from sparkucx_amd import native as N  # noqa: E402
from sparkucx_amd.shuffle import Node  # noqa: E402

HBM_PEAK_GBS = 8000.0     # MI355X HBM3E spec (MI355X_MICROARCH.md, chip table)
XGMI_LINK_GBS = 153.0     # per xGMI link, per direction (task statement; 7 links per GPU)
METRIC = "shuffle GB/s/node (partition+exchange), TeraSort 100B recs at 1/2/4/8 GPUs"


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def uniform_bounds(R: int, key_len: int = 10) -> bytes:
    """bound i = floor((i+1) * 2^64 / R) as the big-endian key prefix (oracle: o_range_bounds_uniform)."""
    out = bytearray()
    for i in range(R - 1):
        v = ((i + 1) << 64) // R
        out += v.to_bytes(8, "big") + bytes(key_len - 8)
    return bytes(out)


WORKLOADS = {
    # name: (record size, R, generator, partitioner kind, key_len, per-GPU records at N=1 / N>1)
    "terasort": (100, 200, N.GEN_TERASORT, N.PART_RANGE_BYTES, 10, 1_000_000_000, 1_250_000_000),
    "zipf": (100, 200, N.GEN_ZIPF, N.PART_MURMUR3_LONG, 8, 1_000_000_000, 1_000_000_000),
    "small": (16, 10000, N.GEN_SMALL, N.PART_MURMUR3_LONG, 8, 1 << 30, 1 << 30),
}


def host_cores() -> dict:
    """Host CPUs this process may use: os.cpu_count() (nproc of the whole machine), the affinity
    mask, and the cgroup CPU quota (cgroup v2 cpu.max) — on the GPU box the job's share is set by
    the quota, while nproc reports every CPU of the machine."""
    nproc = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = nproc
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, period = f.read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) // int(period)))
    except (OSError, ValueError):
        pass
    use = min(aff, quota) if quota else aff
    return {"nproc": nproc, "affinity": aff, "cgroup_quota": quota, "use": use}


def cpu_baseline(args, seed: int, node=None, part=None, data=None, wl: str = "terasort",
                 sample_bytes: int | None = None) -> dict | None:
    """Oracle CPU shuffle (Spark sort-shuffle write to /dev/shm files + UCX-style two-phase fetch)
    on a bounded sample of the same workload: the first records of the GPU run (same seed, same
    counter-based generator, the workload's record size, partitioner and R; args.cpu_records
    TeraSort records = 1 GB, or sample_bytes of the workload's records), 8 map tasks, on every
    host core this job may use (host_cores()['use']; --cpu-threads overrides), median of
    args.cpu_reps runs after a warm-up.  With node/part/data, the GPU partitions
    the same records as the same 8 map tasks and its index tables and per-reducer fetch checksums
    are compared with the CPU's (the two paths are parity-checked on every config)."""
    try:
        from oracle import oracle as O  # test infrastructure: timed as the baseline only
    except Exception as e:  # pragma: no cover
        log("cpu baseline unavailable:", e)
        return None
    hc = host_cores()
    rs, R, _, kind, key_len, _, _ = WORKLOADS[wl]
    n = args.cpu_records if sample_bytes is None else sample_bytes // rs
    maps = 8
    threads = args.cpu_threads if args.cpu_threads > 0 else hc["use"]
    log(f"cpu baseline ({wl}): nproc={hc['nproc']} affinity={hc['affinity']} "
        f"cgroup_quota={hc['cgroup_quota']} -> {threads} threads")
    if wl == "terasort":
        recs, opart = O.gen_terasort(seed, 0, n), O.terasort_partitioner(R)
    elif wl == "zipf":
        recs = O.gen_zipf(seed, 0, n, 1.1, 1 << 24)
        opart = O.Partitioner(kind, R, 0, key_len, 42)
    else:
        recs = O.gen_small(seed, 0, n)
        opart = O.Partitioner(kind, R, 0, key_len, 42)
    d = "/dev/shm" if os.path.isdir("/dev/shm") and os.access("/dev/shm", os.W_OK) else None
    tmp = tempfile.mkdtemp(prefix="sux_cpu_", dir=d)
    times = []
    cpu_index = np.zeros(maps * (R + 1), np.int64)
    checksum = None
    try:
        for i in range(args.cpu_reps + 1):
            r = O.cpu_shuffle(opart, recs, rs, maps, threads, tmp, index_out=cpu_index)
            if r.bytes_fetched != recs.size:
                raise RuntimeError("cpu baseline fetched the wrong byte count")
            checksum = r.checksum
            if i:
                times.append((r.total_s, r.map_s, r.fetch_s))
    finally:
        try:
            os.rmdir(tmp)
        except OSError:
            pass
    times.sort()
    t, tm, tf = times[len(times) // 2]
    names = {"terasort": "TeraSort", "zipf": "Zipf(1.1) TeraSort-shape", "small": "16-byte"}
    out = {"value": round(recs.size / t / 1e9, 3), "unit": "GB/s", "cores": threads,
           "kind": "port", "host": hc, "seed": hex(seed),
           "sample": f"{names[wl]} records [0, {n}) of the GPU run's input (seed {hex(seed)}; "
                     f"{recs.size / 1e9:.2f} GB), R={R}, {maps} map tasks, "
                     f"{threads} threads (nproc {hc['nproc']}, affinity {hc['affinity']}, "
                     f"cgroup quota {hc['cgroup_quota']}); Spark-style write to "
                     f"{'/dev/shm' if d else '/tmp'} files + two-phase offset/block fetch; "
                     f"median of {len(times)} after a warm-up (map {tm:.3f}s, fetch {tf:.3f}s)"}
    if node is not None and data is not None:
        # the same records, the same 8 map tasks, on the GPU: index tables must be equal and
        # every reducer's fetched bytes (blocks of all maps in map order) must checksum equal
        per = -(-n // maps)
        g_out, g_ix, _ = node.partition_maps(part, data[:n * rs], rs, per, num_records=n)
        torch.cuda.synchronize()
        gi = g_ix.cpu().numpy()
        gb = g_out.cpu().numpy()
        ix = gi.reshape(maps, R + 1)
        lib = O.lib()
        gsum = 0
        for r_ in range(R):
            buf = np.concatenate([gb[m * per * rs + ix[m, r_]:m * per * rs + ix[m, r_ + 1]]
                                  for m in range(maps)])
            gsum = (gsum + int(lib.o_checksum(buf.ctypes.data, buf.size))) % (1 << 64)
        out["parity"] = {"index_tables_equal": bool(np.array_equal(gi, cpu_index)),
                         "fetch_checksum_equal": gsum == int(checksum) % (1 << 64),
                         "maps": maps, "records_per_map": per}
        if not (out["parity"]["index_tables_equal"] and out["parity"]["fetch_checksum_equal"]):
            raise RuntimeError(f"cpu baseline and GPU disagree ({wl}): {out['parity']}")
    return out


def reduce_sort(node, recs, ns: int, rs: int, dev) -> dict:
    """Reduce-side consumer: stable GPU sort of one reduce partition's
    worth of TeraSort records by their 10-byte key (the reader's ExternalSorter step).  Reported
    as record bytes sorted per second; the algorithmic bytes are 2 x records x S (read and write
    each record once), the radix passes over 16-byte (key, index) pairs come on top."""
    out = torch.empty(ns * rs, dtype=torch.uint8, device=dev)
    ws = torch.empty(node.sort_workspace_size(ns, rs), dtype=torch.uint8, device=dev)
    for _ in range(2):  # warm-up
        node.sort_records(recs, rs, N.SORT_BYTES, 0, 10, num_records=ns, out=out, workspace=ws)
    torch.cuda.synchronize(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 5
    e0.record()
    for _ in range(reps):
        node.sort_records(recs, rs, N.SORT_BYTES, 0, 10, num_records=ns, out=out, workspace=ws)
    e1.record()
    torch.cuda.synchronize(dev)
    ms = e0.elapsed_time(e1) / reps
    # the sort is planned on the device (no host wait), so it can be captured into a HIP graph
    # and replayed: the same sort without per-call launch overhead
    st = torch.cuda.Stream(device=dev)
    st.wait_stream(torch.cuda.current_stream(dev))
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=st):
        node.sort_records(recs, rs, N.SORT_BYTES, 0, 10, num_records=ns, out=out, workspace=ws,
                          stream=st)
    graph.replay()
    torch.cuda.synchronize(dev)
    e0.record()
    for _ in range(reps):
        graph.replay()
    e1.record()
    torch.cuda.synchronize(dev)
    gms = e0.elapsed_time(e1) / reps
    return {"records": ns, "record_bytes": ns * rs, "ms": round(ms, 3),
            "GB/s": round(ns * rs / (ms / 1e3) / 1e9, 1), "key": "10-byte unsigned, stable",
            "alg_bytes": 2 * ns * rs, "host_waits": 0, "graph_ms": round(gms, 3),
            "graph_GB/s": round(ns * rs / (gms / 1e3) / 1e9, 1)}


def reduce_sort_long(node, ns: int, dev) -> dict:
    """Reduce-side sort of Spark SQL-style 16-byte rows (int64 key in [0, 2^31) + int64 value):
    the key span leaves the top digits constant, so 3 of 6 radix passes are skipped."""
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    rows = torch.empty((ns, 2), dtype=torch.int64, device=dev)
    rows[:, 0] = torch.randint(0, 1 << 31, (ns,), generator=g, device=dev)
    rows[:, 1] = torch.arange(ns, device=dev)
    recs = rows.view(torch.uint8).view(-1)
    out = torch.empty(ns * 16, dtype=torch.uint8, device=dev)
    ws = torch.empty(node.sort_workspace_size(ns, 16), dtype=torch.uint8, device=dev)
    for _ in range(2):
        node.sort_records(recs, 16, N.SORT_LONG, 0, 8, num_records=ns, out=out, workspace=ws)
    torch.cuda.synchronize(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 5
    e0.record()
    for _ in range(reps):
        node.sort_records(recs, 16, N.SORT_LONG, 0, 8, num_records=ns, out=out, workspace=ws)
    e1.record()
    torch.cuda.synchronize(dev)
    ms = e0.elapsed_time(e1) / reps
    k = out.view(torch.int64).view(ns, 2)[:, 0]
    assert bool((k[1:] >= k[:-1]).all()), "long-key sort not ascending"
    return {"records": ns, "record_bytes": ns * 16, "ms": round(ms, 3),
            "Mrec/s": round(ns / (ms / 1e3) / 1e6, 1), "key": "int64 in [0, 2^31), stable"}


def gen_unsafe_rows_dev(n: int, seed: int, dev, max_words: int = 12):
    """Synthetic Spark SQL UnsafeRowSerializer stream on the device (same framing as
    oracle.gen_unsafe_rows, other random draws): 4-byte BE length L | 8-byte null bitset |
    int64 key | k payload words, k uniform in [0, max_words]."""
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    k = torch.randint(0, max_words + 1, (n,), device=dev, generator=g)
    L = 8 * (2 + k)
    offs = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    torch.cumsum(4 + L, 0, out=offs[1:])
    total = int(offs[-1].item())
    data = torch.randint(0, 256, (total,), dtype=torch.uint8, device=dev, generator=g)
    st = offs[:-1]
    for b in range(4):
        data[st + b] = ((L >> (8 * (3 - b))) & 255).to(torch.uint8)
    for b in range(4, 12):
        data[st + b] = 0
    return data, offs


def varlen_leg(node, rows: int, rpm: int, R: int, dev, compress: bool = False) -> dict:
    """§8f item 3: the map side over variable-length UnsafeRow-framed rows (sux_partition_varlen,
    Spark SQL hash of the int64 key at byte 12, R partitions).  GB/s of row bytes; the algorithmic
    HBM bytes are 2 x row bytes (read + write each row) + 44 B per row (offsets read twice, the
    key, the pid written and read back)."""
    data, offs = gen_unsafe_rows_dev(rows, 77, dev)
    part = node.partitioner(N.PART_MURMUR3_LONG, R, key_offset=12, key_len=8)
    out = torch.empty_like(data)
    maps = -(-rows // rpm)
    index = torch.empty(maps * (R + 1), dtype=torch.int64, device=dev)
    be = torch.empty(maps * (R + 1) * 8, dtype=torch.uint8, device=dev)
    ws = torch.empty(node.varlen_workspace_size(part, rpm, rows), dtype=torch.uint8, device=dev)
    run = lambda: node.partition_varlen(part, data, offs, rpm, out=out, index=index, index_be=be,
                                        workspace=ws)
    for _ in range(2):
        run()
    torch.cuda.synchronize(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 5
    e0.record()
    for _ in range(reps):
        run()
    e1.record()
    torch.cuda.synchronize(dev)
    ms = e0.elapsed_time(e1) / reps
    nb = data.numel()
    alg = 2 * nb + 44 * rows
    res = {"rows": rows, "row_bytes": nb, "avg_row": round(nb / rows, 1), "R": R,
           "rows_per_map": rpm, "ms": round(ms, 3), "GB/s": round(nb / (ms / 1e3) / 1e9, 1),
           "alg_bytes": alg, "alg_GB/s": round(alg / (ms / 1e3) / 1e9, 1)}
    if compress:
        res["compress"] = compress_leg(node, out, index, maps, R, dev)
    return res


def compress_leg(node, data, index, maps: int, R: int, dev, bs: int = 32768) -> dict:
    """§8f item 3: spark.shuffle.compress=true (lz4) over map outputs already in HBM
    (sux_compress_map_outputs: one LZ4Block stream per (map, partition) run).  GB/s of
    uncompressed map-output bytes; ratio = framed output / input."""
    nb = data.numel()
    out = torch.empty(node.compress_bound(nb, maps, R, bs), dtype=torch.uint8, device=dev)
    oix = torch.empty(maps * (R + 1), dtype=torch.int64, device=dev)
    obe = torch.empty(maps * (R + 1) * 8, dtype=torch.uint8, device=dev)
    ob = torch.zeros(1, dtype=torch.int64, device=dev)
    ws = torch.empty(node.compress_workspace_size(nb, maps, R, bs), dtype=torch.uint8, device=dev)
    run = lambda: node.compress_map_outputs(data, index, maps, R, bs, out=out, out_index=oix,
                                            out_index_be=obe, out_bytes=ob, workspace=ws)
    run()
    torch.cuda.synchronize(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 3
    e0.record()
    for _ in range(reps):
        run()
    e1.record()
    torch.cuda.synchronize(dev)
    ms = e0.elapsed_time(e1) / reps
    res = {"input_bytes": nb, "maps": maps, "R": R, "block_size": bs, "ms": round(ms, 3),
           "GB/s": round(nb / (ms / 1e3) / 1e9, 1), "ratio": round(int(ob.item()) / nb, 4)}
    # the reader's side: every (map, partition) stream decoded back (sux_decompress_blocks, lz4-
    # java's LZ4BlockInputStream checks included); GB/s of decoded bytes; checked = the input
    ox = oix.view(maps, R + 1)
    base = torch.cumsum(ox[:, R], 0) - ox[:, R]
    boffs = torch.cat([(base[:, None] + ox[:, :R]).reshape(-1), (base[-1] + ox[-1, R]).view(1)])
    cb = int(ob.item())
    dec = torch.empty(nb + 16, dtype=torch.uint8, device=dev)
    doff = torch.empty(maps * R + 1, dtype=torch.int64, device=dev)
    dws = torch.empty(node.decompress_workspace_size(cb, maps * R, bs), dtype=torch.uint8,
                      device=dev)
    drun = lambda: node.decompress_blocks(out, boffs, bs, out=dec, out_offsets=doff,  # noqa: E731
                                          workspace=dws, in_bytes=cb)
    drun()
    torch.cuda.synchronize(dev)
    node.check()
    tot = int(index.view(maps, R + 1)[:, R].sum().item())  # the runs' bytes (maps consecutive)
    ok = int(doff[-1].item()) == tot and torch.equal(dec[:tot], data[:tot])
    if not ok:
        raise RuntimeError("compress leg: the decoded streams differ from the map outputs")
    e0.record()
    for _ in range(reps):
        drun()
    e1.record()
    torch.cuda.synchronize(dev)
    dms = e0.elapsed_time(e1) / reps
    res["decompress"] = {"ms": round(dms, 3), "GB/s": round(tot / (dms / 1e3) / 1e9, 1),
                         "blocks": maps * R, "checked": "decoded bytes = the map outputs"}
    return res


def files_leg(node, out, index, maps: int, R: int, dev) -> dict:
    """§8f item 3: Spark's on-disk files from device map outputs (sux_write_map_files: pinned
    double-buffered D2H + temp file + commit; sux_read_file_blocks back for every map).  PCIe-
    and page-cache-bound; written to /dev/shm (tmpfs) so the disk is not what is measured."""
    import shutil
    import tempfile
    root = "/dev/shm" if os.path.isdir("/dev/shm") else None
    d = tempfile.mkdtemp(prefix="sux_files_", dir=root)
    try:
        dps = [os.path.join(d, f"shuffle_0_{m}_0.data") for m in range(maps)]
        ips = [os.path.join(d, f"shuffle_0_{m}_0.index") for m in range(maps)]
        nb = sum(int(index[m * (R + 1) + R].item()) for m in range(maps))
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        node.write_map_files(out[:nb], index[:maps * (R + 1)], maps, R, dps, ips)
        tw = time.perf_counter() - t0
        buf = torch.empty(int(index[R].item()) + 16, dtype=torch.uint8, device=dev)
        t0 = time.perf_counter()
        for m in range(maps):
            node.read_file_blocks(dps[m], ips[m], R, 0, R, out=buf)
        torch.cuda.synchronize(dev)
        tr = time.perf_counter() - t0
    finally:
        shutil.rmtree(d, ignore_errors=True)
    return {"maps": maps, "bytes": nb, "dir": root or "tmp", "write_s": round(tw, 3),
            "write_GB/s": round(nb / tw / 1e9, 2), "read_s": round(tr, 3),
            "read_GB/s": round(nb / tr / 1e9, 2)}


def maps_2e27_leg(node, part, data, out, n: int, rs: int, R: int, dev, steps: int = 3) -> dict:
    """SURVEY.md §8(d) C2 as written: map batches of 2^27 records (13.4 GB per map task), one
    map per launch group, the same sux_partition_maps_pipelined step as `value` (no resolve)."""
    rpm = 1 << 27
    maps = -(-n // rpm)
    index = torch.empty(maps * (R + 1), dtype=torch.int64, device=dev)
    be = torch.empty(maps * (R + 1) * 8, dtype=torch.uint8, device=dev)
    run = lambda: node.partition_maps_pipelined(part, data, rs, rpm, num_records=n,
                                                group_records=rpm, out=out, index=index,
                                                index_be=be)
    run()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        run()
    torch.cuda.synchronize(dev)
    dt = (time.perf_counter() - t0) / steps
    ix = index.view(maps, R + 1)
    ok = bool((ix[:, 0] == 0).all()) and int(ix[:, R].sum()) == n * rs
    return {"records_per_map": rpm, "maps": maps, "steps": steps, "ms_per_step": round(dt * 1e3, 3),
            "GB/s": round(n * rs / dt / 1e9, 1), "index_consistent": ok}


# newest first: a (workload, kernel) pair not profiled in a later round falls back to an earlier
# round's counters (round 5 re-profiled C5's small-record kernels, whose shape changed)
PMC_FILES = [os.path.join(ROOT, "profiles", f) for f in ("pmc_r06.json", "pmc_r05.json",
                                                          "pmc_r04.json", "pmc_r03.json")]


def plugin_leg(node, part, data, rs: int, R: int, rpm: int, gm: int, groups: int, dev,
               reps: int = 3) -> dict:
    """The drop-in path as Spark drives it, timed end to end through the
    C-ABI: registerShuffle -> getWriter(...).write for every map task (sux_write_map_outputs, one
    launch group of `gm` map tasks per call, published on completion) -> the reduce side resolving
    every (map, reduce partition) block (sux_resolve_blocks, the zero-copy local read at N = 1)
    -> unregisterShuffle.  GB/s of input bytes, to set beside the stateless `value`; plus one
    reducer's fetch (sux_fetch_blocks: its partition from every map into one pooled buffer,
    OnOffsetsFetchCallback's copy)."""
    maps = groups * gm
    n = maps * rpm
    stream = torch.cuda.current_stream(dev)
    # every (map, reduce partition) block, reducer by reducer
    # (sux_block_id rows (map, p, p + 1, 0), built once)
    blocks = node._blocks(np.stack([np.tile(np.arange(maps), R), np.repeat(np.arange(R), maps)],
                                   1).astype(np.int32))

    phase = {"register": 0.0, "write": 0.0, "wait": 0.0, "resolve": 0.0, "unregister": 0.0}

    def one(sid, acc=None):
        t = [time.perf_counter()]
        node.register_shuffle(sid, maps, R, rs)
        t.append(time.perf_counter())
        for g in range(groups):
            r0 = g * gm * rpm
            node.write_map_outputs(sid, g * gm, part, data[r0 * rs:(r0 + gm * rpm) * rs], rpm,
                                   gm * rpm, stream=stream)
        t.append(time.perf_counter())
        node.wait_map_outputs(sid)  # every map published (Spark: the map stage's end)
        t.append(time.perf_counter())
        addrs, sizes = node.resolve_blocks(sid, blocks)
        t.append(time.perf_counter())
        assert int(sizes.sum()) == n * rs
        if acc is not None:
            for k, a, b in zip(("register", "write", "wait", "resolve"), t, t[1:]):
                acc[k] += b - a
        return sid

    one(1000)
    node.unregister_shuffle(1000)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for k in range(reps):
        one(1001 + k, phase)
        tu = time.perf_counter()
        node.unregister_shuffle(1001 + k)
        phase["unregister"] += time.perf_counter() - tu
    torch.cuda.synchronize(dev)
    dt = (time.perf_counter() - t0) / reps
    # one reducer's fetch of partition R//2 from every map: the first call also takes the
    # pooled destination from the allocator; the second (timed) reuses it, as the reducers of
    # a running stage do (MemoryPool.get, MemoryPool.java:137-168)
    sid = one(2000)
    torch.cuda.synchronize(dev)
    req = np.stack([np.arange(maps), np.full(maps, R // 2)], 1).astype(np.int32)
    t0 = time.perf_counter()
    buf, sizes = node.fetch_blocks(sid, req, stream=stream)
    ft_first = time.perf_counter() - t0
    buf.release(maps)
    t0 = time.perf_counter()
    buf, sizes = node.fetch_blocks(sid, req, stream=stream)
    ft = time.perf_counter() - t0
    fb = sum(sizes)
    buf.release(maps)
    node.unregister_shuffle(sid)
    st = node.pool_stats()
    return {"maps": maps, "records": n, "bytes": n * rs, "ms": round(dt * 1e3, 3),
            "GB/s": round(n * rs / dt / 1e9, 1),
            "phase_ms": {k: round(v / reps * 1e3, 3) for k, v in phase.items()},
            "path": "register -> write_map_outputs x%d (%d maps each) -> resolve %d blocks -> "
                    "unregister" % (groups, gm, len(blocks)),
            "fetch_one_reducer": {"blocks": maps, "bytes": fb, "ms": round(ft * 1e3, 3),
                                  "GB/s": round(fb / ft / 1e9, 1),
                                  "first_call_ms": round(ft_first * 1e3, 3)},
            "pool": st}


def plugin_host_leg(node, part, data, rs: int, R: int, rpm: int, maps: int, dev,
                    threads: int = 8, reps: int = 2) -> dict:
    """The drop-in path from the JVM writer's real entry: Spark's map tasks
    serialize rows into HOST memory and GpuShuffleWriter hands them over by address
    (SuxNative.writeMapOutputHostAddr -> sux_write_map_output_host: H2D staging, partition,
    publish, one call per map task), `threads` task threads at once, each on its own stream
    (the executor's cores; getThreadLocalWorker), then every block resolved.  The rows sit in
    pinned memory (a writer's staging area), so the bound is the host->device copy over PCIe:
    `h2d_GB/s` is a plain pinned copy of the same bytes on one stream, measured beside it."""
    import threading
    n = maps * rpm
    host = torch.empty(n * rs, dtype=torch.uint8, pin_memory=True)
    host.copy_(data[:n * rs])  # the rows the tasks serialized (untimed)
    stage = torch.empty(n * rs, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    stage.copy_(host, non_blocking=True)
    torch.cuda.synchronize(dev)
    h2d = n * rs / (time.perf_counter() - t0) / 1e9
    del stage
    streams = [torch.cuda.Stream(dev) for _ in range(threads)]
    blocks = node._blocks(np.stack([np.tile(np.arange(maps), R), np.repeat(np.arange(R), maps)],
                                   1).astype(np.int32))

    def one(sid):
        node.register_shuffle(sid, maps, R, rs)
        errs = []

        def task(k):
            try:
                for m in range(k, maps, threads):
                    node.write_map_output_host(sid, m, part, host[m * rpm * rs:(m + 1) * rpm * rs],
                                               rpm, stream=streams[k])
            except Exception as e:  # pragma: no cover
                errs.append(e)
        ts = [threading.Thread(target=task, args=(k,)) for k in range(threads)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        if errs:
            raise errs[0]
        _, sizes = node.resolve_blocks(sid, blocks)
        assert int(sizes.sum()) == n * rs
        node.unregister_shuffle(sid)

    one(3000)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for k in range(reps):
        one(3001 + k)
    torch.cuda.synchronize(dev)
    dt = (time.perf_counter() - t0) / reps
    gbs = n * rs / dt / 1e9
    return {"maps": maps, "records": n, "bytes": n * rs, "threads": threads,
            "ms": round(dt * 1e3, 3), "GB/s": round(gbs, 1), "h2d_GB/s": round(h2d, 1),
            "of_pcie_bound": round(gbs / h2d, 3),
            "path": f"register -> {threads} task threads x sux_write_map_output_host (pinned host "
                    f"rows, one map task per call) -> resolve {len(blocks)} blocks -> unregister",
            "bound": "PCIe host->device copy (h2d_GB/s: pinned copy of the same bytes, one stream)"}


def plugin_leg_multi(node, part, data, rs: int, R: int, rpm: int, gm: int, groups: int,
                     world: int, rank: int, dev, ctl, xstream) -> dict:
    """The drop-in path at N > 1, as Spark drives it, through the C-ABI:
    registerShuffle -> every rank writes its map tasks launch group by launch group
    (sux_write_map_outputs: peer-major batch slabs) -> the exchange of window g-1 (all ranks' maps
    of group g-1: sux_exchange_maps, one partition-aligned ncclAllToAllv per round of batches on
    its own stream) is enqueued after group g's writes, so it overlaps group g's map kernels ->
    sux_exchange_wait.  Timed (max over ranks) from the first write to the wait; then, untimed,
    every rank fetches its partitions of every map (UcxShuffleClient.fetchBlocks of one
    ShuffleBlockBatchId per map) and checks them on the device: partition ids (k_pids) inside
    its range, non-decreasing per map, run lengths = the map's index file, and the word multiset
    of all ranks' fetched bytes = the inputs'."""
    M = groups * world * gm
    stream = torch.cuda.current_stream(dev)

    def max_over_ranks(v):
        tt = torch.tensor([v], dtype=torch.float64, device=ctl)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        return float(tt.item())

    def run(sid, overlap):
        """(seconds to the exchange's completion, seconds to the last write's completion) of
        one shuffle; overlap=False exchanges only after every write completed (the reference's
        order: the reduce stage starts after the map stage)"""
        node.register_shuffle(sid, M, R, rs)
        torch.cuda.synchronize(dev)
        dist.barrier()
        t0 = time.perf_counter()
        for g in range(groups):
            r0 = g * gm * rpm
            node.write_map_outputs(sid, (g * world + rank) * gm, part,
                                   data[r0 * rs:(r0 + gm * rpm) * rs], rpm, gm * rpm, stream=stream)
            if overlap and g:
                node.exchange_maps(sid, (g - 1) * world * gm, world * gm, stream=xstream)
        tw = None
        if not overlap:
            node.wait_map_outputs(sid)
            torch.cuda.synchronize(dev)
            tw = time.perf_counter() - t0
            for g in range(groups - 1):
                node.exchange_maps(sid, g * world * gm, world * gm, stream=xstream)
        node.exchange_maps(sid, (groups - 1) * world * gm, world * gm, stream=xstream)
        node.exchange_wait(sid)
        torch.cuda.synchronize(dev)
        return time.perf_counter() - t0, tw

    # an untimed first pass fills the device pool (the slabs' first allocations), then the
    # timed shuffle; after its check, the map stage and the exchange once more, serially: how
    # long each takes alone
    run(7001, False)
    node.unregister_shuffle(7001)
    sid = 7000
    dt = max_over_ranks(run(sid, True)[0])
    # ---- untimed device check of everything this rank now serves
    lo, hi = node.owned_partitions(sid)
    sums = torch.zeros(4, dtype=torch.int64, device=dev)

    def wsum(buf):
        acc = torch.zeros(2, dtype=torch.int64, device=dev)
        w32 = buf.view(torch.int32)
        for w0 in range(0, w32.numel(), 1 << 28):
            w = w32[w0:w0 + (1 << 28)].to(torch.int64)
            acc[0] += w.sum()
            acc[1] += (w * w).sum()
        return acc

    sums[:2] += wsum(data[:groups * gm * rpm * rs])
    fetched = 0
    for b0 in range(0, M, 64):
        ms = list(range(b0, min(M, b0 + 64)))
        buf, sizes = node.fetch_blocks(sid, [(m, lo, hi) for m in ms])
        ptr, size, _ = buf.info()
        t = torch.empty(max(4, size), dtype=torch.uint8, device=dev)
        if size:
            N.hip_memcpy(t.data_ptr(), ptr, size, N.HIP_D2D)
        buf.release(len(ms))
        t = t[:size]
        fetched += size
        if size:
            pid = node.partition_ids(part, t, rs).to(torch.int64)
            cnt = torch.tensor([sz // rs for sz in sizes], dtype=torch.int64, device=dev)
            seg = torch.repeat_interleave(torch.arange(len(ms), device=dev), cnt)
            runs = torch.bincount(seg * (hi - lo) + (pid - lo), minlength=len(ms) * (hi - lo))
            want = []
            for m in ms:
                ix = np.frombuffer(node.map_output_index(sid, m, R), dtype=">i8").astype(np.int64)
                want.append((ix[lo + 1:hi + 1] - ix[lo:hi]) // rs)
            want = torch.from_numpy(np.concatenate(want)).to(dev)
            inr = bool(((pid >= lo) & (pid < hi)).all())
            rise = bool(((pid[1:] >= pid[:-1]) | (seg[1:] != seg[:-1])).all())
            eq = torch.equal(runs, want)
            if not (inr and rise and eq):
                raise RuntimeError(f"plugin leg: rank {rank} maps {ms[0]}..{ms[-1]} fetched "
                                   "blocks are not this rank's partitions as indexed (in range "
                                   f"{inr}, grouped {rise}, runs = index {eq}; pids "
                                   f"{int(pid.min())}..{int(pid.max())} for [{lo}, {hi}); "
                                   f"{size} B fetched)")
            sums[2:] += wsum(t)
    tot = sums.to(ctl)
    dist.all_reduce(tot)
    tot = tot.cpu().tolist()
    if tot[0] != tot[2] or tot[1] != tot[3]:
        raise RuntimeError("plugin leg: fetched words differ from the inputs' over all ranks")
    node.unregister_shuffle(sid)
    ts, tw = run(7002, False)
    ts, tw = max_over_ranks(ts), max_over_ranks(tw)
    node.unregister_shuffle(7002)
    n_all = world * groups * gm * rpm
    tx = max(ts - tw, 1e-9)  # the exchange alone, after the map stage
    return {"maps": M, "records": n_all, "bytes": n_all * rs, "ms": round(dt * 1e3, 3),
            "GB/s": round(n_all * rs / dt / 1e9, 1), "fetched_bytes_rank": fetched,
            "serial_ms": {"writes": round(tw * 1e3, 3), "then_exchange": round(tx * 1e3, 3)},
            "exchange_hidden": round(min(1.0, max(0.0, (ts - dt) / tx)), 3),
            "self_check": "ok",
            "path": f"register -> write_map_outputs x{groups} per rank ({gm} maps each) with "
                    f"sux_exchange_maps of the previous window on a second stream -> "
                    f"sux_exchange_wait; then fetch + device check of every owned block"}


GROUP_BYTES = 32 * (1 << 20) * 100  # the default launch group: 3.36 GB of input


def self_check(node, part, data, out, index, n: int, rs: int, rpm: int, R: int,
               group_recs: int, dev) -> dict:
    """Untimed check of the map outputs of one step written into a zeroed buffer, with no CPU
    oracle (the data are 100 GB): every map's index table starts at 0, rises, and ends at the
    map's bytes; its output holds the same multiset of 4-byte words as its input (sum and sum
    of squares); and the partition ids of its output records (the independent k_pids kernel)
    never decrease and count exactly the index table's run lengths.  A sweep's number is only
    reported when its bytes pass this."""
    maps = -(-n // rpm)
    ix = index[:maps * (R + 1)].view(maps, R + 1)
    lens = torch.full((maps,), rpm * rs, dtype=torch.int64, device=dev)
    lens[-1] = (n - (maps - 1) * rpm) * rs
    if not (bool((ix[:, 0] == 0).all()) and bool((ix[:, 1:] >= ix[:, :-1]).all())
            and torch.equal(ix[:, R], lens)):
        raise RuntimeError("self-check: index tables are not each map's run offsets")
    for r0 in range(0, n, group_recs):
        r1 = min(n, r0 + group_recs)
        # the multiset of a launch group's 4-byte words, summed in bounded slices (int64 copies
        # of a whole 13 GB group would not fit beside the data)
        sa = [0, 0]
        sb = [0, 0]
        step = 1 << 28
        for w0 in range(r0 * rs // 4, r1 * rs // 4, step):
            w1 = min(r1 * rs // 4, w0 + step)
            for src, acc in ((data, sa), (out, sb)):
                w = src.view(torch.int32)[w0:w1].to(torch.int64)
                acc[0] += int(w.sum())
                acc[1] += int((w * w).sum())
                del w
        if sa[0] != sb[0] or sa[1] % (1 << 64) != sb[1] % (1 << 64):
            raise RuntimeError(f"self-check: records [{r0}, {r1}) are not a permutation")
        pid = node.partition_ids(part, out[r0 * rs:r1 * rs], rs).to(torch.int64)
        m0 = r0 // rpm
        for m in range(m0, -(-r1 // rpm)):
            p = pid[(m * rpm - r0):(min(r1, (m + 1) * rpm) - r0)]
            cnt = torch.bincount(p, minlength=R) * rs
            if not (bool((p[1:] >= p[:-1]).all()) and torch.equal(cnt, ix[m, 1:] - ix[m, :-1])):
                raise RuntimeError(f"self-check: map {m} is not grouped by partition as indexed")
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    return {"maps": maps, "records": n, "ok": True,
            "checks": "index offsets; word multiset per launch group; output pids (k_pids) "
                      "non-decreasing per map with counts = index runs"}


def make_n1_step(node, part, data, out, index, index_be, n: int, rs: int, R: int, rpm: int,
                 gm: int, comp, resolve: int, map_pipeline: int, nstreams: int, ws_bytes: int,
                 dev):
    """The N = 1 step: every map batch of `data` partitioned (P1-P3) into `out` / `index`,
    either as one sux_partition_maps_pipelined call (two launch groups in flight) or one
    sux_partition_maps call per launch group dealt over `nstreams` streams; with `resolve`, the
    reduce side's local block resolve of config C2 inside the step.  Returns (step, resolved
    counters)."""
    maps = -(-n // rpm)
    group_recs = gm * rpm
    groups = -(-maps // gm)
    ns = max(1, nstreams)
    streams = [comp] + [torch.cuda.Stream(dev) for _ in range(ns - 1)]
    wss = [torch.empty(ws_bytes, dtype=torch.uint8, device=dev) for _ in range(ns)] \
        if not map_pipeline else []

    def step_groups():
        for s in streams[1:]:
            s.wait_stream(comp)
        for g in range(groups):
            r0 = g * group_recs
            r1 = min(n, r0 + group_recs)
            m0 = g * gm
            mg = -(-(r1 - r0) // rpm)
            node.partition_maps(part, data[r0 * rs:r1 * rs], rs, rpm, num_records=r1 - r0,
                                out=out[r0 * rs:r1 * rs],
                                index=index[m0 * (R + 1):(m0 + mg) * (R + 1)],
                                index_be=index_be[m0 * (R + 1) * 8:(m0 + mg) * (R + 1) * 8],
                                workspace=wss[g % ns], stream=streams[g % ns])
        for s in streams[1:]:
            comp.wait_stream(s)

    def step_pipelined():
        node.partition_maps_pipelined(part, data, rs, rpm, num_records=n,
                                      group_records=group_recs, out=out, index=index,
                                      index_be=index_be, stream=comp)

    # the reduce side's local block resolve (config C2): every (map, reduce partition) block
    # of the step's shuffle is resolved through the plugin's C-ABI — the map outputs are
    # committed in place (sux_adopt_map_outputs: index tables read back on the stream,
    # published on completion) and sux_resolve_blocks returns each block's device address
    # and size (OnOffsetsFetchCallback.java:53-72's offsets -> sizes, zero-copy at N = 1)
    # Reduce tasks: at most 200 (TeraSort's R = 200: one ShuffleBlockId per (map, task)); at
    # larger R each task reads a contiguous range of partitions as one ShuffleBlockBatchId per
    # map, as Spark's reducers do with batch fetch (UcxShuffleClient.java:67-73; C5's R = 10 000
    # in 200 tasks of 50 partitions: per-partition resolves would be 10^7 host calls a step)
    tasks = min(R, 200)
    lo_t = (np.arange(tasks) * R) // tasks
    hi_t = (np.arange(1, tasks + 1) * R) // tasks
    # sux_block_id rows (map, start, end, 0), built once: a reducer keeps its block list
    all_blocks = np.ascontiguousarray(np.stack(
        [np.repeat(np.arange(maps), tasks), np.tile(lo_t, maps), np.tile(hi_t, maps),
         np.zeros(maps * tasks, np.int64)], 1).astype(np.int32))
    resolved = {"blocks": 0, "bytes": 0}
    sid_next = [5000]

    def step_resolved(inner):
        def run():
            sid = sid_next[0]
            sid_next[0] += 1
            node.register_shuffle(sid, maps, R, rs)
            inner()
            node.adopt_map_outputs(sid, 0, out, rpm, n, index, stream=comp)
            _, sizes = node.resolve_blocks(sid, all_blocks)
            node.unregister_shuffle(sid)
            resolved["blocks"] += len(sizes)
            resolved["bytes"] += int(sizes.sum())
        return run

    step = step_pipelined if map_pipeline else step_groups
    if resolve:
        step = step_resolved(step)
    return step, resolved


# Measured ceilings on the box (tools/copy_probe.hip sweep, profiles/r02_sweeps/copy_probe.txt:
# streaming read 6.1-6.4 TB/s, copy 5.65-5.76 TB/s of read + write bytes; they move +-5 % from
# box to box).  They set the floor of a two-pass map side: a design cannot run
# faster than reading every record once at the read ceiling and then moving it at the copy one.
READ_CEIL_GBS = 6300.0
COPY_CEIL_GBS = 5760.0


def map_side_floor(kernels: dict, rs: int) -> dict:
    """The map side's design floor: the fastest the launched kernel set can run
    at the measured read and copy ceilings, as GB/s of algorithmic bytes (2 x S per record) and
    as a fraction of the 8 TB/s spec.  Three designs:
    - K1 histogram + K3 scatter (k_hist*, k_scatter*): S read, then 2 S copied per record;
    - two-level MSD (k_msd16a + k_msd16b): two passes that each copy 2 S per record;
    - one pass (no K1): 2 S copied per record."""
    h = kernels.get("hist") or ""
    if h.startswith("k_msd16"):
        t, design = 2 * (2 * rs) / COPY_CEIL_GBS, "two copy passes (MSD pass A + pass B)"
    elif not h:
        t, design = 2 * rs / COPY_CEIL_GBS, "one copy pass"
    else:
        t, design = rs / READ_CEIL_GBS + 2 * rs / COPY_CEIL_GBS, "K1 read + K3 copy"
    ach = 2 * rs / t
    return {"floor_achieved": round(ach, 1), "floor_frac": round(ach / HBM_PEAK_GBS, 4),
            "floor_design": design,
            "ceilings": {"read": READ_CEIL_GBS, "copy": COPY_CEIL_GBS,
                         "source": "tools/copy_probe.hip, profiles/r02_sweeps/copy_probe.txt"}}


def rooflines(node, kt, elapsed: float, steps: int, n: int, rs: int, R: int, maps: int,
              workload: str, pipelined: bool, overlapped: bool):
    """(roofline of the dominant kernel K3, roofline of the whole map side) for one timed run.
    K3: algorithmic bytes (2 x S per record) per launch / its mean launch duration (HIP events on
    the launch stream, node.kernel_times); traffic = PMC bytes per record of the kernel the library
    reports it launched (profiles/pmc_r0x.json).  Map side: (2 N S + 8 (R + 1) per map) per step /
    the wall clock of the timed steps when launch groups overlap (N = 1), else / the sum of the map
    kernels' durations (N > 1: one map stream); floor_frac = the design's two-pass floor."""
    launches, sc_ms = kt["scatter"]
    recs_per_launch = n * steps / max(1, launches)
    alg = 2 * recs_per_launch * rs                       # read + write every record once
    sc_avg = sc_ms / max(1, launches) / 1e3
    achieved = alg / sc_avg / 1e9 if sc_avg else None
    map_ms = kt["hist"][1] + kt["scan"][1] + kt["scatter"][1]
    map_alg = (2 * n * rs + 8 * (R + 1) * maps) * steps
    map_time_ms = elapsed * 1e3 if not pipelined else map_ms
    map_side = map_alg / (map_time_ms / 1e3) / 1e9 if map_time_ms else None
    names = {k: node.kernel_variant(i) for i, k in enumerate(N.KERNELS)}
    tr = {k: load_traffic(workload, names[k]) for k in ("hist", "scatter") if names[k]}
    sc_tr = tr.get("scatter")
    traffic = round(sc_tr["bytes_per_record"] * recs_per_launch) if sc_tr else None
    map_traffic = None
    if sc_tr and (tr.get("hist") or names["hist"] == ""):  # one-pass kernels have no K1
        per_rec = sc_tr["bytes_per_record"] + (tr["hist"]["bytes_per_record"] if tr.get("hist") else 0)
        map_traffic = round(per_rec * n)  # per step; the scans' few KB per map are left out
    roof = {"bound": "hbm", "achieved": None if achieved is None else round(achieved, 1),
            "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": None if achieved is None else round(achieved / HBM_PEAK_GBS, 4),
            "traffic": traffic, "kernel": names["scatter"],
            "traffic_source": sc_tr["source"] if sc_tr else None,
            "alg_bytes_per_launch": int(alg),
            "avg_launch_ms": round(sc_avg * 1e3, 4)}
    floor = map_side_floor(names, rs)
    roof_map = {"bound": "hbm",
                "achieved": None if map_side is None else round(map_side, 1),
                "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": None if map_side is None else round(map_side / HBM_PEAK_GBS, 4),
                "floor_frac": floor["floor_frac"],
                "of_floor": None if map_side is None else round(map_side / floor["floor_achieved"], 4),
                "floor": floor,
                "traffic_per_step": map_traffic,
                "alg_bytes_per_step": int(map_alg / steps),
                "time": ("wall clock of the timed steps (launch groups overlap)"
                         if overlapped else "wall clock of the timed steps"
                         if not pipelined else "sum of the map kernels' durations"),
                "kernels": names,
                "kernels_ms": {k: round(v[1], 3) for k, v in kt.items()},
                "launches": {k: v[0] for k, v in kt.items()}}
    return roof, roof_map


def xgmi_probe(node, world: int, rank: int, dev, nbytes: int, transport: str,
               reps: int = 5, timeout_s: float = 120.0) -> dict:
    """Measured exchange peak (SURVEY §5 calls 153 GB/s per xGMI link "an
    assumption to re-measure on the box"): every rank sends nbytes to every peer at once, through
    the transport the run's exchange uses, with no map side beside it —
    - rccl: the library's own all-to-all (sux_exchange_group over a one-map, R = world group:
      rank h owns partition h, nbytes from each source; grouped ncclSend/ncclRecv pieces);
    - ipc: every rank pulls its share from every peer's IPC-mapped buffer (sux_pull_group).
    Returns the remote bytes per rank per second (the own share is a local copy and is left out
    of the bytes, as in roofline_exchange), and each phase's duration (`phases_ms`: buffers,
    handle all-gather, every peer's ipc_open, the barrier, the first exchange).  Every phase is
    bounded (a W = 8 one-GPU run once stalled after the handle all-gather with no
    word of where): device work is polled against a deadline instead of waited on, and a blocking
    call (an IPC import, a barrier) runs under a watchdog that names the phase and the peer and
    ends the process if it does not return in timeout_s."""
    R = world
    phases = {}
    clock = [time.perf_counter()]

    def mark(name):
        now = time.perf_counter()
        phases[name] = round((now - clock[0]) * 1e3, 3)
        clock[0] = now

    def bounded(what, fn):
        """fn() under a watchdog: a call that does not return in timeout_s is reported (phase,
        peer) and the rank exits — a blocking HIP or gloo call cannot be interrupted."""
        def fire():
            sys.stderr.write(f"[rank {rank}] xgmi probe: {what} did not return in {timeout_s} s\n")
            sys.stderr.flush()
            os._exit(3)
        t = threading.Timer(timeout_s, fire)
        t.daemon = True
        t.start()
        try:
            return fn()
        finally:
            t.cancel()

    def wait_stream(st, what):
        """Device work polled against the deadline (no blocking synchronize)."""
        deadline = time.perf_counter() + timeout_s
        while not st.query():
            if time.perf_counter() > deadline:
                raise RuntimeError(f"[rank {rank}] xgmi probe: {what} still running after "
                                   f"{timeout_s} s")
            time.sleep(0.0005)

    def sync_ranks(what):
        if dist.is_initialized():
            bounded(f"barrier ({what})", dist.barrier)
    send = torch.empty(world * nbytes, dtype=torch.uint8, device=dev)
    send.fill_(rank & 255)
    recv = torch.empty(world * nbytes, dtype=torch.uint8, device=dev)
    rb = torch.zeros(1, dtype=torch.int64, device=dev)
    index = torch.arange(R + 1, dtype=torch.int64, device=dev) * nbytes
    gathered = index.repeat(world)
    st = torch.cuda.Stream(dev)
    st.wait_stream(torch.cuda.current_stream(dev))
    torch.cuda.synchronize(dev)
    mark("buffers")
    ptrs = []
    opens = {}
    if transport == "rccl":
        def once():
            node.exchange_group(send, index, 1, R, gathered, recv, stream=st)
    else:
        hs = [None] * world
        bounded("handle all-gather", lambda: dist.all_gather_object(hs, node.ipc_handle(send)))
        mark("handles")
        for g in range(world):
            if g == rank:
                ptrs.append(send.data_ptr())
                continue
            t0 = time.perf_counter()
            ptrs.append(bounded(f"ipc_open of peer {g}'s {world * nbytes >> 20} MiB buffer",
                                lambda: node.ipc_open(hs[g])))
            opens[g] = round((time.perf_counter() - t0) * 1e3, 3)
        clock[0] = time.perf_counter()
        phases["ipc_open_ms"] = opens
        srcs = torch.tensor(ptrs, dtype=torch.int64, device=dev)

        def once():
            node.pull_group(world, rank, srcs, gathered, 1, R, recv, rb, stream=st)
    sync_ranks("every buffer filled and mapped")  # before anyone reads it
    mark("barrier")
    try:
        once()
        wait_stream(st, "the first exchange" + (" (pulls from every peer)" if ptrs else ""))
        mark("first_exchange")
        once()
        wait_stream(st, "the warm-up exchange")
        sync_ranks("after the warm-up")
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(reps):
            once()
        e1.record(st)
        wait_stream(st, f"{reps} timed exchanges")
        ms = e0.elapsed_time(e1) / reps
        ok = all(int(recv[g * nbytes]) == (g & 255) and int(recv[(g + 1) * nbytes - 1]) == (g & 255)
                 for g in range(world))
        sync_ranks("every rank done reading")  # before any mapping goes away
        mark("timed")
    finally:
        for g, p in enumerate(ptrs):
            if g != rank:
                node.ipc_close(p)
    remote = max(world - 1, 1) * nbytes  # world 1 (--rccl-at-one): the self copy, flagged
    return {"GB/s": round(remote / (ms / 1e3) / 1e9, 1), "bytes_per_peer": nbytes,
            "ms": round(ms, 3), "reps": reps, "ok": ok, "transport": transport,
            "phases_ms": phases,
            "what": ("every rank sends bytes_per_peer to every peer at once, nothing else "
                     "running: " + ("sux_exchange_group (RCCL grouped send/recv)"
                                    if transport == "rccl" else
                                    "sux_pull_group from IPC-mapped peer buffers")
                     + "; GB/s = remote bytes per rank / time")}


def first_mismatch(a: torch.Tensor, b: torch.Tensor, chunk: int = 1 << 28) -> tuple[int, int]:
    """(index of the first differing byte, differing bytes counted up to and including the chunk
    that holds it) of two equal-length byte tensors, in bounded chunks: a whole-buffer
    `(a != b).nonzero()` over a >= 2^31-byte group asks torch for an index tensor of the whole
    buffer's size, so it would report a bogus OOM instead of the mismatch."""
    n = min(a.numel(), b.numel())
    seen = 0
    for c0 in range(0, n, chunk):
        d = (a[c0:c0 + chunk] != b[c0:c0 + chunk])
        k = int(d.sum())
        if k:
            return c0 + int(d.nonzero()[0, 0]), seen + k
    return -1, 0


SEEDS = {"terasort": 0x5EED0002, "zipf": 0x5EED0004, "small": 0x5EED0005}


def make_partitioner(node, kind: int, R: int, key_len: int):
    if kind == N.PART_RANGE_BYTES:
        return node.partitioner(kind, R, key_offset=0, key_len=key_len, bounds=uniform_bounds(R))
    return node.partitioner(kind, R, key_offset=0, key_len=key_len, seed=42)


def generate_input(node, gen: int, seed: int, first: int, n: int, rs: int, out) -> None:
    """Counter-based records [first, first + n) of the workload, written on the device."""
    chunk = 1 << 27
    for c0 in range(0, n, chunk):
        c1 = min(n, c0 + chunk)
        node.generate(gen, seed, first + c0, c1 - c0, rs, zipf_s=1.1, zipf_n=1 << 24,
                      out=out[c0 * rs:c1 * rs])


def config_leg(wl: str, data_buf, dev, steps: int, warmup: int = 1, cpu_args=None) -> dict:
    """BASELINE configs C4 (Zipf-skewed keys) and C5 (small records) on the driver-timed line
    (VERDICT r04 #2): the same N = 1 step as `value` — every map batch partitioned with two launch
    groups in flight, then the local block resolve — on the workload's own full-size input
    (regenerated into the headline's input buffer), on a fresh node; `warmup` untimed steps, then
    `steps` timed ones (wall clock, synchronised), its own roofline / roofline_map_side (PMC
    traffic keyed by workload and kernel), and one more step into zeroed outputs self-checked."""
    rs, R, gen, kind, key_len, n, _ = WORKLOADS[wl]
    rpm = 1 << 20
    gm = max(1, round(GROUP_BYTES / (rpm * rs)))
    maps = -(-n // rpm)
    node = Node(device=dev.index)
    part = None
    try:
        part = make_partitioner(node, kind, R, key_len)
        data = data_buf[:n * rs] if data_buf.numel() >= n * rs else \
            torch.empty(n * rs, dtype=torch.uint8, device=dev)
        generate_input(node, gen, SEEDS[wl], 0, n, rs, data)
        out = torch.empty(n * rs, dtype=torch.uint8, device=dev)
        index = torch.empty(maps * (R + 1), dtype=torch.int64, device=dev)
        index_be = torch.empty(maps * (R + 1) * 8, dtype=torch.uint8, device=dev)
        comp = torch.cuda.current_stream(dev)
        step, resolved = make_n1_step(node, part, data, out, index, index_be, n, rs, R, rpm, gm,
                                      comp, 1, 1, 1, 0, dev)
        for _ in range(warmup):
            step()
        torch.cuda.synchronize(dev)
        node.kernel_times()
        node.set_kernel_timing(True)
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        torch.cuda.synchronize(dev)
        el = time.perf_counter() - t0
        node.set_kernel_timing(False)
        kt = node.kernel_times()
        node.check()
        roof, roof_map = rooflines(node, kt, el, steps, n, rs, R, maps, wl, False, True)
        out.zero_()
        index.zero_()
        step()
        torch.cuda.synchronize(dev)
        sc = self_check(node, part, data, out, index, n, rs, rpm, R, gm * rpm, dev)
        node.check()
        if resolved["bytes"] != n * rs * (warmup + steps + 1):
            raise RuntimeError(f"{wl}: resolved blocks do not cover the input")
        res = {"workload": f"{wl}: {n} x {rs}-byte records ({n * rs / 1e9:.0f} GB), R={R}, map "
                           f"batches of {rpm} records, {gm} maps per launch group, two launch "
                           "groups in flight, zero-copy local block resolve",
               "value": round(n * rs * steps / el / 1e9, 2), "unit": "GB/s", "steps": steps,
               "warmup": warmup, "ms_per_step": round(el / steps * 1e3, 3),
               "roofline": roof, "roofline_map_side": roof_map, "self_check": sc,
               "resolve_blocks_per_step": resolved["blocks"] // (warmup + steps + 1)}
        if cpu_args is not None:
            # the reference CPU shuffle on a 1 GB sample of this config's own input (VERDICT r05
            # #5, BASELINE.md: CPU/GPU parity on every config), outside the timed steps; the
            # output buffer goes first (the parity check partitions the sample on this node)
            out = index = index_be = step = None
            torch.cuda.empty_cache()
            res["cpu_baseline"] = cpu_baseline(cpu_args, SEEDS[wl], node, part, data, wl=wl,
                                               sample_bytes=1 << 30)
        return res
    finally:
        if part is not None:
            part.close()
        node.close()
        # the leg's 100 GB output goes back to the device, not to torch's cache: the next leg's
        # node allocates its workspaces with hipMalloc
        out = index = index_be = step = None
        torch.cuda.empty_cache()


def load_traffic(workload: str, kernel: str) -> dict | None:
    """HBM bytes per record of `kernel` under `workload`, from the committed PMC summary
    (profiles/pmc_r04.json, else pmc_r03.json; written by profiles/collect_pmc.py: one rocprofv3 pass per counter
    group; 2 x FETCH_SIZE + WRITE_SIZE per the microarch guide).  The entry is keyed by workload
    and by the kernel the library reports it launched (sux_kernel_variant), so a line never
    borrows another kernel's counters; None when that pair was not profiled."""
    for path in PMC_FILES:
        try:
            with open(path) as f:
                ks = json.load(f)["workloads"][workload]["kernels"]
            # a slot that runs several kernels ("k_bucket16a+k_bucket16b") sums their bytes
            per = sum(ks[k]["hbm_bytes_per_launch"] / ks[k]["records_per_launch"]
                      for k in kernel.split("+"))
            return {"bytes_per_record": per,
                    "source": f"profiles/{os.path.basename(path)}:{workload}/{kernel}"}
        except (OSError, KeyError, ValueError, ZeroDivisionError):
            continue
    return None


def launched_rank() -> bool:
    """True when a launcher (torch.distributed.run / torchrun / the driver) started this process
    as one rank of a job: it exports WORLD_SIZE and RANK."""
    return "WORLD_SIZE" in os.environ and "RANK" in os.environ


def launch_ranks(args) -> int:
    """`python bench.py --gpus N` (N > 1) with no launcher: start the N ranks as CHILD processes
    (python -m torch.distributed.run, one rank per GPU, rendezvous on 127.0.0.1), relay rank 0's
    JSON line, and return the children's exit status.  Runs before this process touches the GPU
    (no HIP call has been made: torch's CUDA state is initialised lazily, the library is loaded
    but not called), and it never replaces itself (no exec): the parent only waits and relays."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr=127.0.0.1", f"--master-port={port}",
           os.path.abspath(__file__), *sys.argv[1:]]
    log(f"bench: --gpus {args.gpus} without a launcher: starting {args.gpus} ranks: "
        + " ".join(cmd))
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    # the ranks' stderr is inherited (progress stays visible); their stdout carries rank 0's line
    p = subprocess.run(cmd, stdout=subprocess.PIPE, env=env)
    lines = [l for l in p.stdout.decode(errors="replace").splitlines() if l.startswith("{")]
    if p.returncode != 0:
        log(f"bench: the {args.gpus} ranks exited with status {p.returncode}")
        return p.returncode
    if len(lines) != 1:
        log(f"bench: expected one JSON line from rank 0, got {len(lines)}")
        return 1
    res = json.loads(lines[0])
    if res.get("n_gpus") != args.gpus:
        log(f"bench: rank 0 reported n_gpus={res.get('n_gpus')} for --gpus {args.gpus}")
        return 1
    res["launch"] = f"bench.py started {args.gpus} ranks (torch.distributed.run, child processes)"
    sys.stdout.write(json.dumps(res) + "\n")
    sys.stdout.flush()
    return 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default="terasort", choices=sorted(WORKLOADS))
    ap.add_argument("--records", type=int, default=0, help="records per GPU (0 = workload default)")
    ap.add_argument("--partitions", type=int, default=0,
                    help="reduce partitions R (0 = the workload's; sweeps only)")
    ap.add_argument("--map-records", type=int, default=1 << 20, help="records per map batch")
    ap.add_argument("--group-maps", type=int, default=0,
                    help="map batches per kernel launch group (0: ~3.4 GB of input per group — "
                         "32 x 100 MB TeraSort maps, 200 x 16 MB small-record maps: the 256 MiB "
                         "Infinity Cache's write-back and the launch tails are amortised)")
    ap.add_argument("--transport", default="rccl", choices=["rccl", "ipc"],
                    help="N>1 exchange: ncclAllToAllv, or one-sided pull over HIP IPC")
    ap.add_argument("--rehearse-one-gpu", action="store_true",
                    help="test mode: every rank on cuda:0, gloo process group, ipc transport "
                         "(exercises the N>1 pipeline on a 1-GPU box; not a benchmark)")
    ap.add_argument("--loopback-rccl", action="store_true",
                    help="test mode: like --rehearse-one-gpu (every rank on cuda:0, gloo process "
                         "group) but the exchange keeps the rccl transport, through the library "
                         "build whose RCCL calls go to tests/loopback_rccl (files under /dev/shm): "
                         "the RCCL code path's pairing and bytes at W > 1 on a 1-GPU box, where "
                         "RCCL itself refuses two ranks on one GPU; not a benchmark")
    ap.add_argument("--rccl-at-one", action="store_true",
                    help="test mode at N=1: run the N>1 pipeline (peer-major partition, "
                         "overlapped ncclAllGather + ncclAllToAllv) on a one-rank RCCL "
                         "communicator, so the RCCL calls run on a 1-GPU box")
    ap.add_argument("--exchange", default="one-call", choices=["one-call", "post-issue"],
                    help="rccl: 'one-call' = each group's all-gather + plan + all-to-all in one "
                         "sux_exchange_group call on one communicator (the default until a "
                         "multi-rank run has verified the other); 'post-issue' = the all-gather "
                         "of group k (sux_exchange_group_post) beside the all-to-all of k - 1 "
                         "(sux_exchange_group_issue) on a split communicator")
    ap.add_argument("--ownership", default="auto", choices=["auto", "balanced", "equal"],
                    help="N>1: reduce-partition ownership — contiguous ranges balanced by the "
                         "sampled partition bytes (sux_plan_ownership), the equal split, or "
                         "'auto' (balanced when the equal split's busiest owner is > 5 %% over "
                         "the mean)")
    ap.add_argument("--xgmi-probe-mib", type=int, default=256,
                    help="N>1: before the run, time every rank sending this many MiB to every "
                         "peer at once through the run's transport (the measured exchange peak; "
                         "0: skip)")
    ap.add_argument("--c4-steps", type=int, default=3,
                    help="N=1: after the headline, also time BASELINE config C4 (Zipf-skewed "
                         "keys, 100 GB, R=200) for this many steps, self-checked (0: skip)")
    ap.add_argument("--c5-steps", type=int, default=3,
                    help="N=1: after the headline, also time BASELINE config C5 (2^30 16-byte "
                         "records, R=10000) for this many steps, self-checked (0: skip)")
    ap.add_argument("--force-mismatch", action="store_true",
                    help="test mode (pipelined self-check): flip a key byte in the middle of the "
                         "first checked group's received bytes, so the check must fail and "
                         "report the first differing byte")
    ap.add_argument("--map-pipeline", type=int, default=1,
                    help="N=1: 1 = one sux_partition_maps_pipelined call per step (launch "
                         "groups on the node's two map streams, co-resident K1/K3 shapes); "
                         "0 = one sux_partition_maps call per launch group on --streams streams")
    ap.add_argument("--streams", type=int, default=1,
                    help="N=1 with --map-pipeline 0: launch groups dealt round-robin to this "
                         "many HIP streams")
    ap.add_argument("--tuning", default="",
                    help="node tuning table overrides, 'field=value,...' (sux_tuning fields; "
                         "sweeps only — the defaults are the measured best)")
    ap.add_argument("--reserve-cus", type=int, default=-1,
                    help="CUs kept free of map-side kernels for the exchange (-1: 32 if N>1, "
                         "else 0)")
    ap.add_argument("--reduce-sort-records", type=int, default=-1,
                    help="N=1: also time the reduce-side sort (sux_sort_records) of one reduce "
                         "partition (-1: partition R/2's blocks of every map; > 0: that many "
                         "records from the start of the map outputs; 0: skip)")
    ap.add_argument("--varlen-rows", type=int, default=-1,
                    help="N=1: also time the map side over variable-length UnsafeRow-framed rows "
                         "(sux_partition_varlen; -1: 32 Mi rows in 1 Mi-row maps; 0: skip)")
    ap.add_argument("--compress-maps", type=int, default=-1,
                    help="N=1: also time sux_compress_map_outputs (lz4, 32 KiB chunks) over the "
                         "first map outputs (-1: one launch group; 0: skip); the varlen leg's "
                         "rows are compressed too")
    ap.add_argument("--file-maps", type=int, default=-1,
                    help="N=1: also time writing/reading Spark's data + index files for this "
                         "many map outputs (sux_write_map_files; -1: 8; 0: skip)")
    ap.add_argument("--plugin-groups", type=int, default=-1,
                    help="N=1: also time the plugin path (register -> write -> resolve -> "
                         "unregister) over this many launch groups of map tasks (-1: 16; 0: skip)")
    ap.add_argument("--plugin-host-maps", type=int, default=-1,
                    help="N=1: also time the plugin path from pinned host rows through "
                         "sux_write_map_output_host (the JVM writer's entry) over this many map "
                         "tasks (-1: 64; 0: skip)")
    ap.add_argument("--resolve", type=int, default=1,
                    help="N=1: the timed step also commits the map outputs in place and resolves "
                         "every (map, reduce partition) block through sux_resolve_blocks (C2's "
                         "local block resolve)")
    ap.add_argument("--maps-2e27", type=int, default=1,
                    help="N=1 terasort: also time SURVEY C2's 2^27-record map batches (3 steps)")
    ap.add_argument("--self-check", type=int, default=1,
                    help="N=1: after the timed steps, run one more step into a zeroed output "
                         "and check it (index offsets, record multiset, partition grouping)")
    ap.add_argument("--cpu-records", type=int, default=10_000_000)
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="CPU baseline threads (0: every core this job may use, host_cores())")
    ap.add_argument("--cpu-reps", type=int, default=5)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--verify", action="store_true",
                    help="test mode (N>1): check every received block of every group against "
                         "the CPU oracle; timing is then not a benchmark")
    args = ap.parse_args()
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    if args.gpus > 1 and not launched_rank():
        # no launcher: this process becomes the parent of the N ranks (before any GPU call)
        sys.exit(launch_ranks(args))
    # stdout carries exactly one JSON line: RCCL and the HIP runtime print banners from C code,
    # so file descriptor 1 goes to stderr for the whole run and the result is written to a
    # duplicate of the original stdout
    result_fd = os.dup(1)
    sys.stdout.flush()
    os.dup2(2, 1)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        # a line whose n_gpus differs from --gpus would misreport the scaling curve
        raise SystemExit(f"bench: --gpus {args.gpus} but the launcher started WORLD_SIZE={world} "
                         "ranks; pass --gpus equal to --nproc-per-node")
    if args.loopback_rccl:  # before the library is first loaded (Node below)
        N.LIB_PATH = os.path.join(os.path.dirname(N.LIB_PATH), "libsparkucx_amd_loop.so")
    rehearse = (args.rehearse_one_gpu or args.loopback_rccl) and world > 1
    if rehearse:
        local = 0
        if not args.loopback_rccl:
            args.transport = "ipc"
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)
    ctl = torch.device("cpu") if rehearse else dev  # device of the small control collectives
    # the N>1 pipeline (peer-major map outputs + overlapped exchange); at N=1 only on request
    pipelined = world > 1 or args.rccl_at_one
    if args.rccl_at_one:
        args.transport = "rccl"

    rs, R, gen, kind, key_len, n1, nN = WORKLOADS[args.workload]
    R = args.partitions or R
    n = args.records or (n1 if world == 1 else nN)
    rpm, gm = args.map_records, args.group_maps
    if gm <= 0:
        gm = max(1, round(GROUP_BYTES / (rpm * rs)))
    maps = -(-n // rpm)
    groups = -(-maps // gm)
    group_recs = gm * rpm

    # ---- node + communicator bootstrap (unique id carried by torch.distributed) ----------
    comm_id = None
    if world == 1 and args.rccl_at_one:
        comm_id = N.unique_id()
    elif world > 1 and args.transport == "rccl":
        t = torch.zeros(128, dtype=torch.uint8, device=ctl)
        if rank == 0:
            t.copy_(torch.frombuffer(bytearray(N.unique_id()), dtype=torch.uint8))
        dist.broadcast(t, 0)
        comm_id = bytes(t.cpu().numpy())
    # the ipc transport needs no RCCL communicator inside the library
    node = Node(device=local, rank=rank if comm_id else 0, world_size=world if comm_id else 1,
                comm_id=comm_id)
    if args.tuning:
        node.set_tuning(**{k.strip(): int(v) for k, v in
                           (kv.split("=") for kv in args.tuning.split(",") if kv.strip())})
    part = make_partitioner(node, kind, R, key_len)

    # ---- resident input (generated on device, untimed) ---------------------------------------
    seed = SEEDS[args.workload]
    data = torch.empty(n * rs, dtype=torch.uint8, device=dev)
    generate_input(node, gen, seed, rank * n, n, rs, data)
    index = torch.empty(maps * (R + 1), dtype=torch.int64, device=dev)
    ws_bytes = node.workspace_size(part, rs, rpm, min(n, group_recs))
    comp = torch.cuda.current_stream(dev)
    reserve = args.reserve_cus if args.reserve_cus >= 0 else (32 if pipelined else 0)
    if reserve > 0:
        # map-side kernels on a CU-masked stream that leaves `reserve` CUs (spread over the 8
        # XCDs) to the exchange: the partition kernels fill every CU they get (LDS-bound), so
        # an unmasked partition would starve the overlapped all-to-all of CUs
        comp = torch.cuda.ExternalStream(node.cu_stream(reserve, complement=True), device=dev)
        comp.wait_stream(torch.cuda.current_stream(dev))  # the generated input

    if not pipelined:
        out = torch.empty(n * rs, dtype=torch.uint8, device=dev)
        index_be = torch.empty(maps * (R + 1) * 8, dtype=torch.uint8, device=dev)
        step, resolved = make_n1_step(node, part, data, out, index, index_be, n, rs, R, rpm, gm,
                                      comp, args.resolve, args.map_pipeline, args.streams,
                                      ws_bytes, dev)
    else:
        comm = torch.cuda.Stream(dev)
        # send-buffer ring: rccl frees slot s when ITS all-to-all is done (2 slots); ipc frees
        # slot s only when every peer has pulled from it, which rank-locally is known once the
        # NEXT group's all-gather completed (3 slots keep partition(k) off that dependency)
        NB = 3 if args.transport == "ipc" else 2
        send = [torch.empty(group_recs * rs, dtype=torch.uint8, device=dev) for _ in range(NB)]
        # receive ring (Spark's reducer consumes fetched blocks as a stream, maxBytesInFlight).
        # A rank receives at most every rank's whole group (all keys in its partitions), so
        # world x group bytes can never overflow, whatever the skew: Zipf's hot owner at 8 GPUs
        # needs 1.79x (C4).  At C3 that is 2 x 26.8 GB beside 125 GB of input, within 288 GB.
        recv = [torch.empty(world * group_recs * rs, dtype=torch.uint8, device=dev)
                for _ in range(2)]
        ws = [torch.empty(ws_bytes, dtype=torch.uint8, device=dev) for _ in range(NB)]
        # one all-gathered index table per group (kept for the exact byte accounting)
        gidx = torch.empty(groups, world * gm * (R + 1), dtype=torch.int64, device=dev)
        rbytes = torch.zeros(groups, dtype=torch.int64, device=dev)
        peer = [torch.empty(world, dtype=torch.int64, device=dev) for _ in range(NB)]
        part_done = [torch.cuda.Event() for _ in range(NB)]
        send_free = [torch.cuda.Event() for _ in range(NB)]
        xfer_ev = []
        if args.transport == "ipc":
            # rkey analog: map every peer's two send buffers once
            srcs = []
            for sb in send:
                hs = [None] * world
                dist.all_gather_object(hs, node.ipc_handle(sb))
                srcs.append(torch.tensor([sb.data_ptr() if g == rank else node.ipc_open(hs[g])
                                          for g in range(world)], dtype=torch.int64, device=dev))

        # rccl: the index all-gather of group k is POSTED on its own stream right after group k's
        # partition is enqueued, and the all-to-all of group k - 1 is ISSUED on `comm` after that
        # (sux_exchange_group_post / _issue): the host's wait for the gathered counts happens one
        # group late, so `comm` is fed before its previous all-to-all drains and never waits on
        # the host; the all-gather and the all-to-all use two communicators
        gstream = torch.cuda.Stream(dev)
        tickets = {}

        def post(j):
            s = j % NB
            r0 = j * group_recs
            r1 = min(n, r0 + group_recs)
            m0 = j * gm
            mg = -(-(r1 - r0) // rpm)
            gstream.wait_event(part_done[s])
            tickets[j] = node.exchange_group_post(index[m0 * (R + 1):(m0 + mg) * (R + 1)], mg, R,
                                                  gidx[j, :world * mg * (R + 1)], stream=gstream)

        def exchange(j):
            s = j % NB
            r0 = j * group_recs
            r1 = min(n, r0 + group_recs)
            m0 = j * gm
            mg = -(-(r1 - r0) // rpm)
            gi = gidx[j, :world * mg * (R + 1)]
            ix = index[m0 * (R + 1):(m0 + mg) * (R + 1)]
            comm.wait_event(part_done[s])
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(comm)
            if args.transport == "ipc":
                with torch.cuda.stream(comm):
                    # completes only after every rank finished partition(j) and pull(j-1)
                    if rehearse:  # gloo: through the host (synchronous; a test of the logic)
                        comm.synchronize()
                        parts = [torch.empty(ix.numel(), dtype=torch.int64) for _ in range(world)]
                        dist.all_gather(parts, ix.cpu())
                        gi.copy_(torch.cat(parts).to(dev))
                    else:
                        dist.all_gather_into_tensor(gi, ix)
                    send_free[(j - 1) % NB].record(comm)
                    node.pull_group(world, rank, srcs[s], gi, mg, R, recv[j % 2],
                                    rbytes[j:j + 1], stream=comm)
            elif args.exchange == "one-call":
                rb = node.exchange_group(send[s], ix, mg, R, gi, recv[j % 2], stream=comm)
                rbytes[j] = int(rb.sum())
                send_free[s].record(comm)
            else:
                rb = node.exchange_group_issue(tickets.pop(j), send[s], recv[j % 2], stream=comm)
                rbytes[j] = int(rb.sum())
                send_free[s].record(comm)
            e1.record(comm)
            xfer_ev.append((e0, e1))
            if args.verify:
                verify_group(j, recv[j % 2], gi, mg, r0, r1)
            if checking[0]:
                device_check_group(j, recv[j % 2], gi, mg, r0, r1)

        opart = None
        if args.verify:  # test mode: every received block vs the CPU oracle (checker only)
            from oracle import oracle as O
            opart = (O.terasort_partitioner(R) if kind == N.PART_RANGE_BYTES
                     else O.Partitioner(O.MURMUR3_LONG, R, 0, 8, 42))
            ogen = {"terasort": O.gen_terasort, "zipf": O.gen_zipf, "small": O.gen_small}[args.workload]
            lib = N.load()

        def verify_group(j, rbuf, gi, mg, r0, r1):
            torch.cuda.synchronize(dev)
            got = rbuf.cpu().numpy()
            gnp = np.ascontiguousarray(gi.cpu().numpy())
            lo, hi = int(owner[rank]), int(owner[rank + 1])
            for g in range(world):
                grecs = ogen(seed, g * n + r0, r1 - r0)
                for m in range(mg):
                    a, b = m * rpm, min(r1 - r0, (m + 1) * rpm)
                    d, _, ix, _ = O.write_map(opart, grecs[a * rs:b * rs], rs)
                    for p in range(lo, hi):
                        off = lib.sux_plan_block_offset_owned(world, rank, mg, R,
                                                              gnp.ctypes.data,
                                                              owner.ctypes.data, g, m, p)
                        want = d[ix[p]:ix[p + 1]]
                        if off < 0 or got[off:off + len(want)].tobytes() != want.tobytes():
                            raise RuntimeError(f"verify: rank {rank} group {j} source {g} "
                                               f"map {m} partition {p} differs")
            verified[0] += 1

        verified = [0]
        checking = [False]
        # word sums (sum, sum of squares; int64, wrapping) of the inputs / received bytes of the
        # check step, all-reduced over ranks at its end: every record reaches exactly one owner
        msums = torch.zeros(4, dtype=torch.int64, device=dev)
        check_stats = {"groups": 0, "received_bytes": 0, "records": 0}

        def word_sums(buf):
            acc = torch.zeros(2, dtype=torch.int64, device=dev)
            w32 = buf.view(torch.int32)
            step_w = 1 << 28
            for w0 in range(0, w32.numel(), step_w):
                w = w32[w0:w0 + step_w].to(torch.int64)
                acc[0] += w.sum()
                acc[1] += (w * w).sum()
                del w
            return acc

        def locate(t, own, lo, hi, mg, rec):
            """(source rank, map of the group, partition) whose block holds received record
            `rec` by the gathered index: the first mismatch named the way the oracle checks it."""
            ends = torch.cumsum((own // rs).reshape(-1), 0).cpu().tolist()
            segi = next((i for i, e in enumerate(ends) if rec < e), len(ends) - 1)
            g, m = divmod(segi, mg)
            off = (rec - (ends[segi - 1] if segi else 0)) * rs
            row = (t[g, m, lo:hi + 1] - t[g, m, lo]).cpu().tolist()
            p = lo + max(0, next((k for k in range(hi - lo) if off < row[k + 1]), hi - lo - 1))
            return f"source {g} map {j_map0[0] + m} (group map {m}) partition {p} (record {rec})"

        j_map0 = [0]

        def device_check_group(j, rbuf, gi, mg, r0, r1):
            """N > 1 self-check of one launch group's exchange, on the device (no oracle): the
            received bytes equal the exact sum from the gathered index; every received record's
            partition id (recomputed by the independent k_pids kernel) lies in this rank's owned
            range, is non-decreasing within each (source, map) block run and counts exactly the
            index runs; the word multiset is checked across ranks at the end of the step.  A
            failure raises (the run exits non-zero) naming the first mismatching (source, map,
            partition)."""
            torch.cuda.synchronize(dev)
            lo, hi = int(owner[rank]), int(owner[rank + 1])
            j_map0[0] = j * gm
            t = gi.view(world, mg, R + 1)
            own = t[:, :, hi] - t[:, :, lo]
            exp = int(own.sum())
            got = int(rbytes[j].item())
            if got != exp:
                raise RuntimeError(f"self-check: rank {rank} group {j} received {got} bytes, "
                                   f"the gathered index says {exp}")
            if exp and args.force_mismatch and check_stats["groups"] == 0:
                # test mode: corrupt the first key byte of the middle received record
                k = (exp // rs // 2) * rs
                rbuf[k:k + 1].bitwise_xor_(0x80)
            if exp:
                pid = node.partition_ids(part, rbuf[:exp], rs).to(torch.int64)
                inr = (pid >= lo) & (pid < hi)
                if not bool(inr.all()):
                    k0 = int((~inr).nonzero().flatten()[0])
                    raise RuntimeError(f"self-check: rank {rank} group {j} received a record "
                                       f"outside its partitions [{lo}, {hi}): first mismatch at "
                                       f"{locate(t, own, lo, hi, mg, k0)}, pid {int(pid[k0])}")
                cnt = (own // rs).reshape(-1)
                seg = torch.repeat_interleave(torch.arange(world * mg, device=dev), cnt)
                rise = (pid[1:] >= pid[:-1]) | (seg[1:] != seg[:-1])
                runs = torch.bincount(seg * (hi - lo) + (pid - lo), minlength=world * mg * (hi - lo))
                want = ((t[:, :, lo + 1:hi + 1] - t[:, :, lo:hi]) // rs).reshape(-1)
                if not (bool(rise.all()) and torch.equal(runs, want)):
                    bad = (~rise).nonzero().flatten()
                    sb = send[j % NB]
                    same = world == 1 and torch.equal(rbuf[:exp], sb[:exp])
                    spid = node.partition_ids(part, sb[:exp], rs).to(torch.int64) if world == 1 else None
                    sdesc = "" if spid is None else (
                        f"; send slab falls {int((spid[1:] < spid[:-1]).sum())} times, "
                        f"first at {(spid[1:] < spid[:-1]).nonzero().flatten()[:4].tolist()}")
                    if world == 1:
                        d0, nd = first_mismatch(rbuf[:exp], sb[:exp])
                        sdesc += (f"; first differing byte at {d0} ({nd} differ up to the end of "
                                  f"its 256 MiB chunk); received bytes there "
                                  f"{rbuf[max(d0, 0):max(d0, 0) + 8].tolist()} send "
                                  f"{sb[max(d0, 0):max(d0, 0) + 8].tolist()}")
                        if args.transport == "rccl":  # again, synchronously, on one stream
                            torch.cuda.synchronize(dev)
                            node.exchange_group(sb, index[j * gm * (R + 1):(j * gm + mg) * (R + 1)],
                                                mg, R, gi, rbuf)
                            torch.cuda.synchronize(dev)
                            sdesc += f"; equal after a synchronous re-exchange: {torch.equal(rbuf[:exp], sb[:exp])}"
                    k0 = int(bad[0]) + 1 if bad.numel() else None
                    if k0 is None:  # the run counts differ: the first differing (block, partition)
                        d = int((runs != want).nonzero().flatten()[0])
                        blk, pp = divmod(d, hi - lo)
                        g_, m_ = divmod(blk, mg)
                        where = f"source {g_} map {j * gm + m_} (group map {m_}) partition {lo + pp}"
                    else:
                        where = locate(t, own, lo, hi, mg, k0)
                    raise RuntimeError(
                        f"self-check: rank {rank} group {j}: first mismatch at {where}; "
                        f"received blocks are not grouped by "
                        f"partition as the index says ({bad.numel()} falls, first at records "
                        f"{bad[:4].tolist()}, pids there {pid[bad[:4]].tolist()} -> "
                        f"{pid[bad[:4] + 1].tolist()}; runs differ at "
                        f"{(runs != want).nonzero().flatten()[:4].tolist()} of {runs.numel()}, "
                        f"{cnt.tolist()[:4]} records in the first blocks; received == send slab: "
                        f"{same}{sdesc})")
                msums[2:] += word_sums(rbuf[:exp])
            msums[:2] += word_sums(data[r0 * rs:r1 * rs])
            check_stats["groups"] += 1
            check_stats["received_bytes"] += exp
            check_stats["records"] += exp // rs

        def step():
            for k in range(groups):
                s = k % NB
                r0 = k * group_recs
                r1 = min(n, r0 + group_recs)
                m0 = k * gm
                mg = -(-(r1 - r0) // rpm)
                if k >= NB:
                    # rccl: the all-to-all of k-2 has read send[s]; ipc: the all-gather of k-2
                    # completed, so every peer finished pulling group k-3 out of send[s]
                    comp.wait_event(send_free[s])
                node.partition_maps_peer_major(part, data[r0 * rs:r1 * rs], rs, rpm, world,
                                               num_records=r1 - r0, out=send[s],
                                               index=index[m0 * (R + 1):(m0 + mg) * (R + 1)],
                                               peer_bytes=peer[s], workspace=ws[s], stream=comp)
                part_done[s].record(comp)
                if args.transport == "rccl" and args.exchange == "post-issue":
                    post(k)
                if k >= 1:
                    exchange(k - 1)
            exchange(groups - 1)
            comp.wait_stream(comm)
            comp.wait_stream(gstream)

    def barrier():
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)

    # ---- reduce-partition ownership (N > 1): contiguous ranges, balanced by bytes ----------
    # Planned once, before the shuffle, from a sample: the partition sizes of every rank's first
    # launch group, summed over ranks (as Spark's RangePartitioner samples keys in a job of its
    # own before a sort's shuffle).  'auto' takes the balanced split when the equal one leaves
    # its busiest owner > 5 % above the mean (Zipf keys, C4), else keeps the equal split.
    owner = np.array([(h * R) // world for h in range(world + 1)], np.int32)
    own_info = None
    if pipelined and world > 1 and args.ownership != "equal":
        torch.cuda.synchronize(dev)
        t_own = time.perf_counter()
        sn = min(n, group_recs)
        pid = node.partition_ids(part, data[:sn * rs], rs).to(torch.int64)
        cnt = (torch.bincount(pid, minlength=R) * rs).to(ctl)
        del pid
        dist.all_reduce(cnt)
        cnt = cnt.cpu().numpy()
        bal = N.plan_ownership(world, cnt)
        mean = cnt.sum() / world
        r_eq = max(int(cnt[owner[h]:owner[h + 1]].sum()) for h in range(world)) / mean
        r_bal = max(int(cnt[bal[h]:bal[h + 1]].sum()) for h in range(world)) / mean
        use = args.ownership == "balanced" or r_eq > 1.05
        if use:
            owner = bal
            node.set_ownership(world, R, owner)
        own_info = {"plan": "balanced" if use else "equal", "sample_records_per_rank": sn,
                    "sampled_max_over_mean": {"equal": round(r_eq, 4), "balanced": round(r_bal, 4)},
                    "plan_ms": round((time.perf_counter() - t_own) * 1e3, 3),
                    "bounds": owner.tolist() if world <= 16 else None}
        log(f"[rank {rank}] ownership: {own_info}")

    xprobe = None
    if pipelined and (world > 1 or args.rccl_at_one) and args.xgmi_probe_mib > 0:
        # the one-GPU rehearsal (W ranks sharing one GPU's memory) probes with 16 MiB per peer:
        # its 256 MiB probe stalls inside hipIpcOpenMemHandle (profiles/r06_ipc/: the runtime's
        # import, reproduced with no call of this library; every phase is now bounded and named)
        mib = min(args.xgmi_probe_mib, 16) if rehearse else args.xgmi_probe_mib
        xprobe = xgmi_probe(node, world, rank, dev, mib << 20, args.transport)
        if rehearse:
            xprobe["one_gpu"] = "every rank on cuda:0: an on-chip copy, not xGMI"
        elif world == 1:
            xprobe["one_gpu"] = "--rccl-at-one: the self copy through a one-rank communicator"
        log(f"[rank {rank}] xgmi probe: {xprobe}")
    log(f"[rank {rank}] {args.workload}: {n} records x {rs} B = {n * rs / 1e9:.1f} GB/GPU, "
        f"R={R}, {maps} maps of {rpm}, {groups} launch groups of {gm} maps, world={world}")
    for _ in range(args.warmup):
        step()
    barrier()
    node.kernel_times()  # drop warm-up timings
    node.set_kernel_timing(True)
    if pipelined:
        xfer_ev.clear()
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    barrier()
    t1 = time.perf_counter()
    node.set_kernel_timing(False)
    kt = node.kernel_times()
    node.check()  # no kernel recorded a failure in the device error word

    elapsed = t1 - t0
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=ctl)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    ms_per_step = elapsed / args.steps * 1e3
    total_bytes = n * rs * world * args.steps
    value = total_bytes / elapsed / 1e9

    # ---- roofline of the dominant kernel (scatter) + the whole map-side pass --------------
    overlapped = not pipelined and (args.map_pipeline or args.streams > 1)
    roof, roof_map = rooflines(node, kt, elapsed, args.steps, n, rs, R, maps, args.workload,
                               pipelined, overlapped)
    result = {
        "metric": METRIC, "value": round(value, 2), "unit": "GB/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic (counter-based generator, resident in HBM before timing)",
        "config": {"workload": f"{args.workload}: {n} x {rs}-byte records per GPU "
                               f"({n * rs / 1e9:.0f} GB/GPU, {n * rs * world / 1e9:.0f} GB total), "
                               f"R={R}, map batches of {rpm} records, {gm} maps per launch group"
                               + (", two launch groups in flight (sux_partition_maps_pipelined)"
                                  if not pipelined and args.map_pipeline else
                                  f" on {args.streams} streams" if not pipelined and args.streams > 1
                                  else "")
                               + (f", map side on {256 - reserve} CUs" if reserve > 0 else "")
                               + (", zero-copy local block resolve (one block per map and "
                                  "reduce task, <= 200 tasks)" if not pipelined and args.resolve else
                                  "" if not pipelined else
                                  ", partition-aligned all-to-all exchange (RCCL grouped "
                                  "send/recv)" if args.transport == "rccl" else
                                  ", partition-aligned one-sided IPC pull exchange"),
                   "global_batch": n * world, "seq_len": rs, "parallelism": f"shuffle{world}"},
        "roofline": roof,
        "roofline_map_side": roof_map,
        "cpu_baseline": None,
    }
    if pipelined:
        torch.cuda.synchronize(dev)
        xms = sum(a.elapsed_time(b) for a, b in xfer_ev)
        xfer_n = len(xfer_ev)
        # exact off-GPU bytes per step from the all-gathered index tables
        gh = gidx.cpu().numpy()
        lo, hi = int(owner[rank]), int(owner[rank + 1])
        remote = ingress = 0
        for j in range(groups):
            mg = -(-(min(n, (j + 1) * group_recs) - j * group_recs) // rpm)
            t = gh[j, :world * mg * (R + 1)].reshape(world, mg, R + 1)
            own = t[:, :, hi] - t[:, :, lo]
            remote += int(own.sum() - own[rank].sum())
            ingress += int(own.sum())
        # the exchange runs at its busiest owner's ingress: max / mean of the ranks' received bytes
        ing = torch.tensor([ingress, ingress], dtype=torch.float64, device=ctl)
        if world > 1:
            dist.all_reduce(ing[0:1], op=dist.ReduceOp.MAX)
            dist.all_reduce(ing[1:2])
        ing = ing.cpu().tolist()
        ingress_ratio = ing[0] / (ing[1] / world) if ing[1] else None
        if int(rbytes.min().item()) < 0:
            raise RuntimeError("exchange overflowed a receive buffer")
        remote *= args.steps
        peak = (world - 1) * XGMI_LINK_GBS
        ach = remote / (xms / 1e3) / 1e9 if xms and remote else None
        if args.verify:
            result["verified_groups"] = verified[0]
        if args.self_check:
            # one more (untimed) step with every launch group's exchange checked on the device
            checking[0] = True
            step()
            torch.cuda.synchronize(dev)
            checking[0] = False
            tot = msums.to(ctl)
            if world > 1:
                dist.all_reduce(tot)
            tot = tot.cpu().tolist()
            if tot[0] != tot[2] or tot[1] != tot[3]:
                raise RuntimeError("self-check: the multiset of exchanged words differs from the "
                                   "inputs' over all ranks")
            result["self_check"] = {"ok": True, "groups": check_stats["groups"],
                                    "received_bytes": check_stats["received_bytes"],
                                    "checks": "received bytes = gathered-index sums per group; "
                                              "k_pids of every received record in the owned "
                                              "range, non-decreasing per (source, map) run, "
                                              "run counts = index; word multiset over all "
                                              "ranks = the inputs'"}
        # how much of the exchange the map side hides: the partition kernels run
        # on `comp`, the all-to-alls on `comm`; serial would take map + exchange, the step took
        # ms_per_step, so the overlap saved (map + exchange - step) of the exchange's time
        map_ms_step = (kt["hist"][1] + kt["scan"][1] + kt["scatter"][1]) / args.steps
        x_ms_step = xms / args.steps
        hidden = None
        if x_ms_step > 0:
            hx = torch.tensor([(map_ms_step + x_ms_step - ms_per_step) / x_ms_step],
                              dtype=torch.float64, device=ctl)
            if world > 1:  # the rank that hides the least bounds the node
                dist.all_reduce(hx, op=dist.ReduceOp.MIN)
            hidden = round(min(1.0, max(0.0, float(hx.item()))), 3)
        result["roofline_exchange"] = {
            "bound": "xgmi", "achieved": None if ach is None else round(ach, 1), "peak": peak,
            "peak_source": f"(world - 1) x {XGMI_LINK_GBS} GB/s per xGMI link (spec assumption)",
            "unit": "GB/s", "frac": None if ach is None else round(ach / peak, 4),
            "remote_bytes_per_rank": remote // args.steps, "exchange_ms": round(xms, 2),
            "exchange": args.exchange if args.transport == "rccl" else "ipc pull",
            "ingress_max_over_mean": None if ingress_ratio is None else round(ingress_ratio, 4),
            "exchange_hidden": hidden,
            "exchange_hidden_from": {"map_kernels_ms_per_step": round(map_ms_step, 3),
                                     "exchange_ms_per_step": round(x_ms_step, 3),
                                     "ms_per_step": round(ms_per_step, 3),
                                     "formula": "(map + exchange - step) / exchange, min over "
                                                "ranks, clamped to [0, 1]"},
            "ownership": own_info}
        if args.self_check:
            result["roofline_exchange"]["device_self_check"] = "ok"
        if xprobe is not None:
            mp = xprobe["GB/s"]
            if world > 1:  # the slowest rank's peer-read rate bounds the node
                tt = torch.tensor([mp], dtype=torch.float64, device=ctl)
                dist.all_reduce(tt, op=dist.ReduceOp.MIN)
                mp = float(tt.item())
            result["roofline_exchange"]["measured_peak"] = round(mp, 1)
            result["roofline_exchange"]["frac_of_measured"] = (
                None if ach is None or not mp else round(ach / mp, 4))
            result["roofline_exchange"]["probe"] = xprobe
    if pipelined and world > 1 and args.plugin_groups != 0:
        # the stateless pipeline's rings go back first: the plugin leg's slabs and receive
        # buffers take their HBM.  Every rank first unmaps its peers' send buffers and all
        # ranks agree on it before any buffer is freed: a freed allocation's address comes back
        # for the next one, and an importer still holding the old mapping of that address would
        # be handed the stale memory when it opens the new allocation's handle
        if args.transport == "ipc":
            torch.cuda.synchronize(dev)
            for tab in srcs:
                for g, ptr in enumerate(tab.tolist()):
                    if g != rank:
                        node.ipc_close(ptr)
            srcs.clear()
            torch.cuda.synchronize(dev)
            dist.barrier()
        send.clear()
        recv.clear()
        ws.clear()
        torch.cuda.empty_cache()
        if node.world_size == 1:  # ipc transport: the plugin's exchange needs the host bootstrap
            node = Node(device=local, rank=rank, world_size=world)
            node.set_bootstrap(lambda b: (lambda out: (dist.all_gather_object(out, b), out)[1])(
                [None] * world))
            part = make_partitioner(node, kind, R, key_len)
        pg = min(n // group_recs, args.plugin_groups if args.plugin_groups > 0 else 8)
        if pg:
            xs = torch.cuda.Stream(dev)
            result["plugin"] = plugin_leg_multi(node, part, data, rs, R, rpm, gm, pg, world, rank,
                                                dev, ctl, xs)
    if not pipelined and args.self_check:
        out.zero_()
        index.zero_()
        step()
        torch.cuda.synchronize(dev)
        result["self_check"] = self_check(node, part, data, out, index, n, rs, rpm, R,
                                          group_recs, dev)
    if not pipelined and args.resolve:
        steps_run = args.warmup + args.steps + (1 if args.self_check else 0)
        result["resolve"] = {"blocks_per_step": resolved["blocks"] // max(1, steps_run),
                             "bytes_per_step": resolved["bytes"] // max(1, steps_run),
                             "path": "sux_register_shuffle -> partition -> sux_adopt_map_outputs "
                                     "-> sux_resolve_blocks(one block per (map, reduce task): "
                                     "min(R, 200) tasks, ShuffleBlockBatchId ranges when R > 200) -> "
                                     "sux_unregister_shuffle, inside every timed step"}
        if resolved["bytes"] != n * rs * steps_run:
            raise RuntimeError("resolved blocks do not cover the input")
    if not pipelined and args.workload == "terasort" and args.reduce_sort_records != 0:
        if args.reduce_sort_records > 0:  # the first records of the map outputs
            ns = min(args.reduce_sort_records, n)
            recs, what = out[:ns * rs], f"the first {ns} records of the map outputs"
        else:
            # one real reduce partition: partition R/2's block of every map, in map order (what
            # a reducer fetches: random order inside one 1/R slice of the key range)
            p = R // 2
            idx = index.view(maps, R + 1)[:, p:p + 2].cpu().tolist()
            recs = torch.cat([out[m * rpm * rs + a:m * rpm * rs + b]
                              for m, (a, b) in enumerate(idx) if b > a])
            ns = recs.numel() // rs
            what = f"reduce partition {p}: its block of each of the {maps} map outputs"
        if ns > 0:
            result["reduce_sort"] = reduce_sort(node, recs, ns, rs, dev)
            result["reduce_sort"]["input"] = what
            del recs
            result["reduce_sort_long"] = reduce_sort_long(node, 32 << 20, dev)
    if not pipelined and args.maps_2e27 and args.workload == "terasort" and n >= (1 << 27) \
            and rpm != (1 << 27):
        result["maps_2e27"] = maps_2e27_leg(node, part, data, out, n, rs, R, dev)
    if not pipelined and args.compress_maps != 0:
        cm = min(maps, args.compress_maps if args.compress_maps > 0 else gm)
        if cm:
            # maps are consecutive in `out`: the first cm map outputs
            nb = sum(int(index[m * (R + 1) + R].item()) for m in range(cm))
            result["compress"] = compress_leg(node, out[:nb], index[:cm * (R + 1)], cm, R, dev)
    if not pipelined and args.file_maps != 0:
        fm = min(maps, args.file_maps if args.file_maps > 0 else 8)
        result["files"] = files_leg(node, out, index, fm, R, dev)
    if not pipelined and args.plugin_groups != 0:
        # the stateless output is no longer needed: its HBM goes to the plugin path's slabs
        out = None
        torch.cuda.empty_cache()
        pg = min(groups, args.plugin_groups if args.plugin_groups > 0 else 16)
        if pg and n >= pg * group_recs:
            result["plugin"] = plugin_leg(node, part, data, rs, R, rpm, gm, pg, dev)
        if args.plugin_host_maps != 0:
            hm = min(maps, args.plugin_host_maps if args.plugin_host_maps > 0 else 64)
            result["plugin_host"] = plugin_host_leg(node, part, data, rs, R, rpm, hm, dev)
    if not pipelined and args.varlen_rows != 0:
        vr = args.varlen_rows if args.varlen_rows > 0 else 32 << 20
        result["varlen"] = varlen_leg(node, vr, min(vr, 1 << 20), 200, dev,
                                      compress=args.compress_maps != 0)
    if rank == 0 and not args.no_cpu_baseline:
        # the reference CPU shuffle beside every line, N > 1 included (north_star: "at 1, 2, 4
        # and 8 GPUs beside the reference CPU shuffle"): the same bounded sample on rank 0's host
        # cores.  Rank 0's shard starts at global record 0, so its first records ARE the
        # sample, and the GPU parity check partitions them on this rank's device.
        cpu_n = min(args.cpu_records, n)
        args.cpu_records = cpu_n
        result["cpu_baseline"] = cpu_baseline(
            args, seed, node, part, data if args.workload == "terasort" and R == 200 else None)
        if world > 1 and result["cpu_baseline"]:
            result["cpu_baseline"]["beside"] = f"N={world}: rank 0 only, after the timed steps"
    if not pipelined and args.workload == "terasort" and (args.c4_steps > 0 or args.c5_steps > 0):
        # the other BASELINE configs on the same driver-timed line: the headline's node and
        # output go first (the config legs take a fresh node and the input buffer)
        part.close()
        node.close()
        out = None
        torch.cuda.empty_cache()
        cfg = {}
        if args.c4_steps > 0:
            cfg["c4"] = config_leg("zipf", data, dev, args.c4_steps,
                                   cpu_args=None if args.no_cpu_baseline else args)
            log(f"c4: {cfg['c4']['value']} GB/s")
        if args.c5_steps > 0:
            cfg["c5"] = config_leg("small", data, dev, args.c5_steps,
                                   cpu_args=None if args.no_cpu_baseline else args)
            log(f"c5: {cfg['c5']['value']} GB/s")
        result.update(cfg)
    if world > 1:
        dist.barrier()  # the other ranks wait for rank 0's baseline before tearing down
    if rank == 0:
        os.write(result_fd, (json.dumps(result) + "\n").encode())
    part.close()
    node.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
