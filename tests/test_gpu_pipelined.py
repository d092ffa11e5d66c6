"""GPU parity: the pipelined map side (sux_partition_maps_pipelined, two launch groups in flight
on the node's map streams with the co-resident K1/K3 shapes) and every kernel shape the node's
tuning table (sux_tuning) can select, against the CPU oracle — bit-exact on data bytes, native
index tables and Spark's big-endian index bytes.  No tuning value may change a byte.
"""
import numpy as np
import pytest
import torch

from oracle import oracle as O
from sparkucx_amd import native as N

pytestmark = pytest.mark.gpu


def host(t):
    return t.cpu().numpy()


def gpu_part(node, p):
    return node.partitioner(p.kind, p.R, key_offset=p.key_offset, key_len=p.key_len, seed=p.seed,
                            ascending=p.ascending, bounds=p.bounds)


def expect(opart, recs, rs, rpm, out, index, index_be):
    n = recs.size // rs
    maps = -(-n // rpm)
    want_data, want_index, want_be = O.write_maps(opart, recs, rs, rpm)
    assert host(out)[: n * rs].tobytes() == bytes(want_data), "data bytes differ"
    assert host(index)[: maps * (opart.R + 1)].tolist() == want_index.tolist()
    if index_be is not None:
        assert host(index_be)[: maps * (opart.R + 1) * 8].tobytes() == want_be


@pytest.mark.parametrize("R,n,rpm,gmaps", [
    (200, 7 * 20000 + 1234, 20000, 2),     # 4 groups, ragged last map and group
    (200, 9 * 8192, 8192, 1),              # one map per group: 9 groups over 2 streams
    (64, 50000, 50000, 3),                 # one group only (the second stream idles)
    (512, 6 * 30000, 30000, 2),            # v7's largest R
    (1000, 5 * 12000 + 17, 12000, 2),      # v6 territory
    (7, 3 * 4096, 4096, 1),
])
def test_pipelined_matches_oracle(gpu_node, R, n, rpm, gmaps):
    recs = O.gen_terasort(31, 0, n)
    opart = O.terasort_partitioner(R)
    gp = gpu_part(gpu_node, opart)
    d = torch.from_numpy(recs).cuda()
    out, index, index_be = gpu_node.partition_maps_pipelined(gp, d, 100, rpm,
                                                             group_records=gmaps * rpm)
    torch.cuda.synchronize()
    expect(opart, recs, 100, rpm, out, index, index_be)
    gp.close()


@pytest.mark.parametrize("co", [1, -1])
def test_pipelined_coresident_shapes(gpu_node, tuned, co):
    tuned(coresident=co, hist_wgs_per_cu=1 if co == 1 else 0)
    n, rpm = 5 * 30000 + 77, 30000
    recs = O.gen_terasort(38, 0, n)
    opart = O.terasort_partitioner(200)
    gp = gpu_part(gpu_node, opart)
    out, index, index_be = gpu_node.partition_maps_pipelined(gp, torch.from_numpy(recs).cuda(),
                                                             100, rpm, group_records=2 * rpm)
    torch.cuda.synchronize()
    expect(opart, recs, 100, rpm, out, index, index_be)
    gp.close()


@pytest.mark.parametrize("split", [32, 64, 96, 224])
@pytest.mark.parametrize("R,n,rpm,gmaps", [
    (200, 7 * 20000 + 1234, 20000, 2),     # 4 groups: both workspace slots reused
    (200, 9 * 8192, 8192, 1),              # 9 one-map groups
    (64, 50000, 50000, 3),                 # one group
    (1000, 5 * 12000 + 17, 12000, 2),
])
def test_pipelined_split_mode_matches_oracle(gpu_node, tuned, split, R, n, rpm, gmaps):
    """split_cus: K1 of group g on `split` CUs beside K2 + K3 of group g - 1 on the others
    (workspace slots reused by group g + 2 behind an event); twice in a row on one node, the
    second call reusing the split streams.  Bytes and both index forms vs the oracle."""
    tuned(split_cus=split)
    recs = O.gen_terasort(33 + split, 0, n)
    opart = O.terasort_partitioner(R)
    gp = gpu_part(gpu_node, opart)
    d = torch.from_numpy(recs).cuda()
    for _ in range(2):
        out, index, index_be = gpu_node.partition_maps_pipelined(gp, d, 100, rpm,
                                                                 group_records=gmaps * rpm)
        torch.cuda.synchronize()
        expect(opart, recs, 100, rpm, out, index, index_be)
    gp.close()


@pytest.mark.parametrize("kind,key_len,off", [(O.MURMUR3_LONG, 8, 0), (O.HASH_INT, 4, 4),
                                              (O.MURMUR3_BYTES, 12, 8)])
def test_pipelined_hash_kinds_and_skew(gpu_node, kind, key_len, off):
    recs = O.gen_zipf(32, 0, 60000, 1.1, 1 << 12)
    opart = O.Partitioner(kind, 200, off, key_len, seed=42)
    gp = gpu_part(gpu_node, opart)
    out, index, index_be = gpu_node.partition_maps_pipelined(gp, torch.from_numpy(recs).cuda(),
                                                             100, 10000, group_records=20000)
    torch.cuda.synchronize()
    expect(opart, recs, 100, 10000, out, index, index_be)
    gp.close()


def test_pipelined_small_records_and_default_group(gpu_node):
    """16-byte records with many partitions (the k_hist16/k_scatter16b path), default group."""
    recs = O.gen_small(33, 0, 300000)
    opart = O.Partitioner(O.MURMUR3_LONG, 5000, 0, 8, seed=42)
    gp = gpu_part(gpu_node, opart)
    out, index, index_be = gpu_node.partition_maps_pipelined(gp, torch.from_numpy(recs).cuda(),
                                                             16, 100000)
    torch.cuda.synchronize()
    expect(opart, recs, 16, 100000, out, index, index_be)
    gp.close()


def test_pipelined_on_a_side_stream_and_repeated(gpu_node):
    """Ordered after the caller's stream (input generated there) and joined back into it; the
    node's group workspaces are reused by the next call (and grow when a group is larger)."""
    opart = O.terasort_partitioner(200)
    gp = gpu_part(gpu_node, opart)
    s = torch.cuda.Stream()
    for n, rpm, g in [(40000, 10000, 1), (160000, 20000, 3), (40000, 10000, 2)]:
        with torch.cuda.stream(s):
            d = gpu_node.generate(N.GEN_TERASORT, 34, 0, n, 100, stream=s)
            out, index, index_be = gpu_node.partition_maps_pipelined(
                gp, d, 100, rpm, group_records=g * rpm, stream=s)
            ix = index.clone()  # on s: must see the joined result
        s.synchronize()
        expect(opart, O.gen_terasort(34, 0, n), 100, rpm, out, ix, index_be)
    gp.close()


def test_pipelined_full_size_equals_single_launch_path(gpu_node):
    """0.84 GB (64 maps of 131072 TeraSort records, the bench map shape) in 8-map groups:
    identical bytes to one sux_partition_maps launch over the same input."""
    n, rpm, R = 64 * 131072, 131072, 200
    opart = O.terasort_partitioner(R)
    gp = gpu_part(gpu_node, opart)
    d = gpu_node.generate(N.GEN_TERASORT, 0x5EED0002, 0, n, 100)
    a = gpu_node.partition_maps_pipelined(gp, d, 100, rpm, group_records=8 * rpm)
    b = gpu_node.partition_maps(gp, d, 100, rpm)
    torch.cuda.synchronize()
    for x, y in zip(a, b):
        assert torch.equal(x, y)
    idx = a[1].view(-1, R + 1)
    assert bool((idx[:, R] == rpm * 100).all()) and bool((idx[:, 1:] >= idx[:, :-1]).all())
    gp.close()


def test_pipelined_rejects_partial_map_groups(gpu_node):
    gp = gpu_part(gpu_node, O.terasort_partitioner(8))
    d = torch.zeros(1000 * 100, dtype=torch.uint8, device="cuda")
    with pytest.raises(N.SuxError) as e:
        gpu_node.partition_maps_pipelined(gp, d, 100, 300, group_records=500)
    assert e.value.code == N.SUX_EINVAL
    gp.close()


# ---- every shape the tuning table selects, bit-exact ----------------------------------------
TUNINGS = [
    {"scatter_chunk": 768},                              # the co-resident K3 shape
    {"scatter_chunk": 768, "hist_wgs_per_cu": 1},
    {"coresident": -1},
    {"scatter_chunk": 768, "scatter_depth": 2},
    {"scatter_chunk": 512},
    {"scatter_chunk": 1024, "hist_stage": 128},
    {"hist_stage": 64, "hist_wgs_per_cu": 2},
    {"tiles_per_item": 1},
    {"tiles_per_item": 64},
    {"scatter_kernel": 7},
    {"scatter_kernel": 7, "tiles_per_item": 1},
    {"scatter_order": 2},
    {"scatter_order": 2, "tile_records": 1024},
    {"scatter_kernel": 6},
    {"scatter_kernel": 6, "s6_chunk": 384},
    {"scatter_kernel": 1, "hist_kernel": 1},
    {"hist_kernel": 3},
    {"tile_records": 1024},
    {"hist_nt": -1},                                     # plain K1 loads (non-temporal: default)
    {"counts_layout": 1},                                # partition-major tile counts
    {"scatter_counters": 1},                             # partition-major k_scatter8 counters
]


@pytest.mark.parametrize("tn", TUNINGS, ids=lambda t: ",".join(f"{k}={v}" for k, v in t.items()))
@pytest.mark.parametrize("R", [200, 512])
def test_tuning_shapes_are_bit_exact(gpu_node, tuned, tn, R):
    tuned(**tn)
    n, rpm = 3 * 40000 + 999, 40000
    recs = O.gen_terasort(35, 0, n)
    opart = O.terasort_partitioner(R)
    gp = gpu_part(gpu_node, opart)
    ws = torch.empty(gpu_node.workspace_size(gp, 100, rpm, n), dtype=torch.uint8, device="cuda")
    out, index, index_be = gpu_node.partition_maps(gp, torch.from_numpy(recs).cuda(), 100, rpm,
                                                   num_records=n, workspace=ws)
    torch.cuda.synchronize()
    expect(opart, recs, 100, rpm, out, index, index_be)
    gp.close()


@pytest.mark.parametrize("kernel,groups", [(1, 1), (1, 2), (1, 4), (2, 0), (4, 0)])
def test_small_record_kernels_bit_exact(gpu_node, tuned, kernel, groups):
    """Every small-record scatter: turn-taking k_scatter16b (1, 2, 4 groups per turn), the
    turn-free sorted-chunk k_scatter16s and the two-level k_msd16a + k_msd16b (no K1)."""
    tuned(small_kernel=kernel, small_groups=groups)
    recs = O.gen_small(36, 0, 200000)
    opart = O.Partitioner(O.MURMUR3_LONG, 3000, 0, 8, seed=42)
    gp = gpu_part(gpu_node, opart)
    out, index, index_be = gpu_node.partition_maps(gp, torch.from_numpy(recs).cuda(), 16, 50000)
    torch.cuda.synchronize()
    expect(opart, recs, 16, 50000, out, index, index_be)
    gp.close()
    gpu_node.check()


@pytest.mark.parametrize("R,n,rpm,skew", [
    (1025, 70000, 70000, None),         # just above the per-wave-counter limit
    (10000, 300000, 100000, None),      # C5's R; 4096-record chunks + a ragged tail per tile
    (10000, 123457, 123457, "one"),     # every record in one partition: 4096-long runs
    (10000, 200000, 50000, "zipf"),     # Zipf-skewed keys
    (16384, 150000, 75000, None),       # largest R of the sorted-chunk kernel (14 pid bits)
    (16385, 100000, 100000, None),      # one above: the turn-taking kernel
    (4096, 5000, 1000, None),           # maps shorter than one chunk
    (2000, 300000, 300000, "one"),      # one bucket holds the whole map (many LDS chunks)
    (1100, 90000, 30000, "zipf"),       # a short last bucket (1100 = 17 x 64 + 12)
])
@pytest.mark.parametrize("kernel", [2, 4])
def test_sorted_chunk_scatter_shapes(gpu_node, tuned, kernel, R, n, rpm, skew):
    """kernel 2: the sorted-chunk scatter; kernel 4: the two-level MSD path (segments larger
    than its LDS piece in the 'one' and 'zipf' rows)"""
    tuned(small_kernel=kernel)
    if skew == "zipf":
        recs = O.gen_zipf(39, 0, n, 1.1, 1 << 12)
        recs = recs.reshape(-1, 100)[:, :16].copy().ravel()
    else:
        recs = O.gen_small(39, 0, n)
    if skew == "one":
        recs.reshape(-1, 16)[:, :8] = 7
    opart = O.Partitioner(O.MURMUR3_LONG, R, 0, 8, seed=42)
    gp = gpu_part(gpu_node, opart)
    out, index, index_be = gpu_node.partition_maps(gp, torch.from_numpy(recs).cuda(), 16, rpm)
    torch.cuda.synchronize()
    expect(opart, recs, 16, rpm, out, index, index_be)
    want = "k_scatter16b" if R > 16384 else "k_scatter16s" if kernel == 2 else "k_msd16b"
    assert gpu_node.kernel_variant(2) == want
    gp.close()
    gpu_node.check()


def test_kernel_variant_reports_the_coresident_shape(gpu_node, tuned):
    """The timing slots name the variant that ran (bench.py's roofline cites it)."""
    gp = gpu_part(gpu_node, O.terasort_partitioner(200))
    d = gpu_node.generate(N.GEN_TERASORT, 37, 0, 100000, 100)
    gpu_node.partition_maps_pipelined(gp, d, 100, 25000, group_records=50000)
    torch.cuda.synchronize()
    assert gpu_node.kernel_variant(0) == "k_hist4" and gpu_node.kernel_variant(2) == "k_scatter8"
    gp.close()


@pytest.mark.parametrize("kernel,order", [(8, 0), (8, 1), (7, 0)])
def test_launch_group_over_8_gib_keeps_the_image_scatter(gpu_node, tuned, kernel, order):
    """One 2^27-record TeraSort map (13.4 GB; r01 fell back to k_scatter2 above 8 GiB of group
    output, 29-bit image units).  Checked on the device without the oracle: the index is the
    map's run offsets, and every run p equals the input records whose k_pids id is p, in input
    order (stable) — for the first, a middle and the last partitions in full, and the runs that
    straddle the 8 GiB output offset."""
    tuned(scatter_kernel=kernel, scatter_order=order)
    n, R = 1 << 27, 200
    gp = gpu_part(gpu_node, O.terasort_partitioner(R))
    d = gpu_node.generate(N.GEN_TERASORT, 41, 0, n, 100)
    out, index, _ = gpu_node.partition_maps(gp, d, 100, n, want_be=False)
    torch.cuda.synchronize()
    assert gpu_node.kernel_variant(2) == f"k_scatter{kernel}"
    ix = index[:R + 1]
    assert int(ix[0]) == 0 and int(ix[R]) == n * 100 and bool((ix[1:] >= ix[:-1]).all())
    pids = gpu_node.partition_ids(gp, d, 100).to(torch.int64)
    cnt = torch.bincount(pids, minlength=R) * 100
    assert torch.equal(cnt, ix[1:] - ix[:-1])
    rows = d.view(n, 100)
    ixh = ix.cpu().tolist()
    over = [p for p in range(R) if ixh[p] < (8 << 30) <= ixh[p + 1]]
    for p in sorted({0, R // 2, R - 1, *over, *(q + 1 for q in over if q + 1 < R)}):
        want = rows[pids == p].reshape(-1)
        assert torch.equal(out[ixh[p]:ixh[p + 1]], want), p
    del pids, rows
    gp.close()


@pytest.mark.parametrize("R,n,rpm,tile,tpi", [
    (200, 300000, 300000, 4096, 1),     # an item per tile: a seam every 4 chunks
    (200, 250001, 70001, 4096, 0),      # ragged maps: items end mid-line everywhere
    (208, 200000, 100000, 4096, 3),     # largest R of k_scatter8 (its LDS tables' RMAX)
    (7, 100000, 50000, 4096, 2),        # few partitions: long runs, many full lines per chunk
    (150, 90000, 90000, 1024, 1),       # short tiles: one chunk per item
    (209, 60000, 60000, 4096, 0),       # above k_scatter8's RMAX: k_scatter7
])
def test_line_carry_scatter_shapes(gpu_node, tuned, R, n, rpm, tile, tpi):
    """k_scatter8 (whole-line writes, carried partial lines): item seams at every tile, runs
    ending mid-line, a partition absent from most chunks, records skewed into few partitions."""
    tuned(tile_records=tile, tiles_per_item=tpi)
    recs = O.gen_zipf(42, 0, n, 1.3, 1 << 10) if R == 7 else O.gen_terasort(42, 0, n)
    if R == 7:
        opart = O.Partitioner(O.MURMUR3_LONG, R, 0, 8, seed=42)
    else:
        opart = O.terasort_partitioner(R)
    gp = gpu_part(gpu_node, opart)
    out, index, index_be = gpu_node.partition_maps(gp, torch.from_numpy(recs).cuda(), 100, rpm)
    torch.cuda.synchronize()
    expect(opart, recs, 100, rpm, out, index, index_be)
    assert gpu_node.kernel_variant(2) == ("k_scatter8" if R <= 208 else "k_scatter7")
    gp.close()


@pytest.mark.parametrize("R,n,rpm,skew", [
    (10000, 3 * 131072 + 5000, 131072, None),   # 32 chunks per map, ragged last map
    (10000, 100000, 100000, "hot"),             # 30 % of the records in one partition
    (4096, 70000, 20000, None),                 # 256 buckets: 8-bit pass A digits
    (4097, 70000, 20000, None),                 # 257 buckets: 9-bit pass A digits
    (8193, 70000, 20000, None),                 # 513 buckets: 10-bit pass A digits
    (16384, 3 * 65536, 65536, None),            # 1024 buckets, the largest R
    (1025, 4096 * 3, 4096, "one"),              # whole chunks of one partition
    (3000, 1, 1, None),                         # a single record
])
@pytest.mark.parametrize("wpc,direct", [(2, 0), (1, 0), (2, -1), (1, -1), (2, 3), (1, 3), (2, 1),
                                        (2, 2), (2, 4), (2, 6), (2, 8), (2, 16), (1, 16),
                                        (2, 56), (1, 56), (2, 88), (1, 88), (2, 72),
                                        (2, 152), (1, 152), (2, 136)])
def test_msd16_pids_and_shapes(gpu_node, tuned, R, n, rpm, skew, wpc, direct):
    """The two-level small-record path (small_kernel 4, 2 or 1 workgroups per CU; msd_direct:
    each pass stores records from registers instead of through its LDS stage (bits 0, 1), pass A
    by LDS-DMA (bit 2), 32-partition buckets (bit 3), pass B's element -> run map (bit 4), pass B
    gathering the next segment while it writes the current one (bit 5), pass A ranking with
    one LDS atomic per digit group (bit 6), pass A matching digits on a 6-bit lane tag (bit 7)):
    bytes, both
    index tables and the caller-requested pid array (written by pass A in input order) equal
    the oracle's."""
    tuned(small_kernel=4, small_wgs_per_cu=wpc, msd_direct=direct)
    recs = O.gen_small(41, 0, n)
    if skew == "one":
        recs.reshape(-1, 16)[:, :8] = 3
    elif skew == "hot":
        recs.reshape(-1, 16)[: n * 3 // 10: 3, :8] = 11
    opart = O.Partitioner(O.MURMUR3_LONG, R, 0, 8, seed=42)
    gp = gpu_part(gpu_node, opart)
    pids = torch.empty(n, dtype=torch.int16, device="cuda")
    out, index, index_be = gpu_node.partition_maps(gp, torch.from_numpy(recs).cuda(), 16, rpm,
                                                   pids=pids)
    torch.cuda.synchronize()
    expect(opart, recs, 16, rpm, out, index, index_be)
    assert (host(pids).view(np.uint16) == opart.ids(recs, 16)).all()
    assert gpu_node.kernel_variant(0) == "k_msd16a" and gpu_node.kernel_variant(2) == "k_msd16b"
    gp.close()
    gpu_node.check()


def test_msd16_falls_back_for_the_exchange_layout(gpu_node, tuned):
    """Peer-major outputs (N > 1) are not map-major: small_kernel 4 keeps the sorted-chunk
    scatter there, bit-exact."""
    tuned(small_kernel=4)
    recs = O.gen_small(42, 0, 60000)
    opart = O.Partitioner(O.MURMUR3_LONG, 5000, 0, 8, seed=42)
    gp = gpu_part(gpu_node, opart)
    d = torch.from_numpy(recs).cuda()
    out = torch.empty_like(d)
    index = torch.empty(3 * 5001, dtype=torch.int64, device="cuda")
    peer = torch.empty(4, dtype=torch.int64, device="cuda")
    gpu_node.partition_maps_peer_major(gp, d, 16, 20000, 4, out=out, index=index, peer_bytes=peer)
    torch.cuda.synchronize()
    assert gpu_node.kernel_variant(2) == "k_scatter16s"
    want_data, want_index, want_peer = O.peer_major(opart, recs, 16, 20000, 4)
    assert host(out).tobytes() == want_data.tobytes()
    assert host(index).tolist() == want_index.tolist()
    assert host(peer).tolist() == want_peer.tolist()
    gp.close()


@pytest.mark.parametrize("R,n,rpm,skew", [
    (10000, 3 * 65536 + 777, 65536, None),   # C5's R, 64 Ki-record maps, a ragged last map
    (10000, 2 * 65536, 65536, "one"),        # one segment far above the LDS piece
    (16384, 2 * 65536, 65536, "zipf"),       # 64 buckets of 256 partitions, skewed
    (1025, 3 * 8192, 8192, None),            # 5 buckets (the last of 1 partition), 2-chunk maps
    (10000, 2 * 262144, 262144, None),       # 64 chunks per map: the short run table's limit
])
@pytest.mark.parametrize("direct", [0, -1, 3, 4, 16])
def test_msd16_short_maps_256_partition_buckets(gpu_node, tuned, R, n, rpm, skew, direct):
    """Default tuning, maps too short for 16-partition segments: the two-level path with
    256-partition buckets (pass A digits pid >> 8, pass B sorts by pid & 255).  Bytes, both index
    tables and the pids equal the oracle's."""
    tuned(msd_direct=direct)
    if skew == "zipf":
        recs = O.gen_zipf(45, 0, n, 1.1, 1 << 12)
        recs = recs.reshape(-1, 100)[:, :16].copy().ravel()
    else:
        recs = O.gen_small(44, 0, n)
    if skew == "one":
        recs.reshape(-1, 16)[: n // 2, :8] = 5
    opart = O.Partitioner(O.MURMUR3_LONG, R, 0, 8, seed=42)
    gp = gpu_part(gpu_node, opart)
    pids = torch.empty(n, dtype=torch.int16, device="cuda")
    out, index, index_be = gpu_node.partition_maps(gp, torch.from_numpy(recs).cuda(), 16, rpm,
                                                   pids=pids)
    torch.cuda.synchronize()
    expect(opart, recs, 16, rpm, out, index, index_be)
    assert (host(pids).view(np.uint16) == opart.ids(recs, 16)).all()
    assert gpu_node.kernel_variant(2) == "k_msd16b"
    gp.close()
    gpu_node.check()


@pytest.mark.parametrize("rpm,want", [(16384, "k_scatter16s"), (65536, "k_msd16b"),
                                      (100000, "k_msd16b"), (655360, "k_msd16b")])
def test_default_small_kernel_picks_by_segment_length(gpu_node, rpm, want):
    """Default tuning: the two-level path only when a (map, bucket) segment holds >= 1024
    records on average — 16-partition buckets for maps of >= 640 000 records at R = 10 000,
    256-partition buckets for maps of >= 40 960 (64 Ki-record maps: 1677-record segments);
    shorter maps take the sorted-chunk scatter.  All bit-exact."""
    n = 2 * rpm + 12345
    recs = O.gen_small(43, 0, n)
    opart = O.Partitioner(O.MURMUR3_LONG, 10000, 0, 8, seed=42)
    gp = gpu_part(gpu_node, opart)
    out, index, index_be = gpu_node.partition_maps(gp, torch.from_numpy(recs).cuda(), 16, rpm)
    torch.cuda.synchronize()
    expect(opart, recs, 16, rpm, out, index, index_be)
    assert gpu_node.kernel_variant(2) == want
    gp.close()
