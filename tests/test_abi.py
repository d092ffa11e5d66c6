"""CPU: the C-ABI library loads, exports every header symbol, and its host-only logic is right.

No compute call is made here (there is no GPU in the CPU job); the exchange planner is pure host
arithmetic and is checked against a direct restatement.
"""
import ctypes as C

import numpy as np
import pytest

from sparkucx_amd import native as N


def test_library_loads_and_exports_every_header_symbol():
    lib = N.load()
    declared = N.header_symbols()
    assert len(declared) >= 30
    missing = [s for s in declared if not hasattr(lib, s)]
    assert not missing, missing
    assert set(declared) == set(N._SIGS), set(declared) ^ set(N._SIGS)
    assert lib.sux_abi_version() == 6
    assert C.sizeof(N.Conf) == 432  # sux_conf of ABI v2 (prealloc pairs appended)
    assert C.sizeof(N.Tuning) == 128  # sux_tuning: 31 knobs + 1 reserved


def test_conf_defaults_mirror_ucx_shuffle_conf():
    c = N.default_conf()
    assert c.world_size == 1 and c.rank == 0
    assert c.min_buffer_size == 1024          # spark.shuffle.ucx.memory.minBufferSize
    assert c.min_allocation_size == 4 << 20   # spark.shuffle.ucx.memory.minAllocationSize
    assert c.metadata_block_size == 300       # 2 * spark.shuffle.ucx.rkeySize


@pytest.mark.parametrize("spec,want", [
    ("", []),
    ("4k:1000,16k:500", [(4096, 1000), (16384, 500)]),    # UcxShuffleConf.scala:53 doc example
    (" 1m : 3 ,, 2048:1", [(1 << 20, 3), (2048, 1)]),      # trimmed, empty entries skipped
    ("1g:2,8kb:4,100b:7", [(1 << 30, 2), (8192, 4), (100, 7)]),
])
def test_prealloc_spec_parses_like_spark(spec, want):
    c = N.default_conf(prealloc=spec)
    got = [(c.prealloc_size[k], c.prealloc_count[k]) for k in range(c.num_prealloc)]
    assert got == want


@pytest.mark.parametrize("spec", ["4k", "4k:1:2", "x:1", "4q:1", "4k:-1", "4k:1e3"])
def test_prealloc_spec_rejects_malformed_entries(spec):
    with pytest.raises(N.SuxError) as e:
        N.default_conf(prealloc=spec)
    assert e.value.code == N.SUX_EINVAL


def test_bootstrap_and_pool_entry_points_validate_arguments():
    lib = N.load()
    assert lib.sux_node_set_bootstrap(None, N.ALLGATHER_FN(0), None) == N.SUX_EINVAL
    assert lib.sux_pool_stats(None, None, None, None, None) == N.SUX_EINVAL
    assert lib.sux_wait_map_outputs(None, 0) == N.SUX_EINVAL
    assert lib.sux_write_map_outputs(None, 0, 0, None, None, 1, 0, None) == N.SUX_EINVAL


@pytest.mark.parametrize("field,value", [
    ("hist_kernel", 5), ("scatter_kernel", 3), ("coresident", 2), ("scatter_chunk", 256),
    ("scatter_depth", 3), ("hist_stage", 32), ("hist_wgs_per_cu", 9), ("small_kernel", 5), ("small_waves", 12), ("scatter_order", 3), ("small_wgs_per_cu", 3), ("sort_msd", 4), ("s6_chunk", 100), ("tiles_per_item", -1),
    ("small_groups", 3), ("tile_records", 96), ("tile_records", 32), ("onepass", 2),
    ("varlen_kernel", 4), ("varlen_tile", 100), ("sort_max_digit_bits", 17), ("sort_gather", 2),
    ("sort_all_passes", -1), ("hist_kernel", 2), ("scatter_kernel", 2), ("small_kernel", 3),
    ("hist_nt", 2), ("counts_layout", 3), ("scatter_counters", 3), ("lz4_queue", 3), ("scatter_nt", 4), ("gather_kernel", 4), ("split_cus", 48), ("split_cus", 256), ("msd_direct", 256), ("msd_direct", -2),
    ("exchange_self", 2), ("reserved", 1)])
def test_tuning_table_rejects_values_outside_each_fields_set(field, value):
    """sux_node_set_tuning validates the whole table before it looks at the node, so every
    field's range is checkable without a GPU: an out-of-set value is EINVAL naming the field."""
    lib = N.load()
    t = N.Tuning()
    if field == "reserved":
        t.reserved[len(t.reserved) - 1] = value
    else:
        setattr(t, field, value)
    assert lib.sux_node_set_tuning(None, C.byref(t)) == N.SUX_EINVAL
    buf = C.create_string_buffer(256)
    lib.sux_last_error(buf, 256)
    assert field.split("_")[0] in buf.value.decode()


@pytest.mark.parametrize("fields", [{}, {"coresident": -1}, {"coresident": 1, "hist_stage": 128},
                                    {"scatter_chunk": 768, "scatter_depth": 2},
                                    {"tile_records": 1 << 22, "varlen_tile": 65536},
                                    {"sort_max_digit_bits": 8, "onepass": 1}])
def test_tuning_table_accepts_listed_values(fields):
    lib = N.load()
    t = N.Tuning()
    for f, v in fields.items():
        setattr(t, f, v)
    assert lib.sux_node_set_tuning(None, C.byref(t)) == N.SUX_EINVAL  # valid table, no node
    buf = C.create_string_buffer(256)
    lib.sux_last_error(buf, 256)
    assert buf.value.decode() == "NULL node"
    assert lib.sux_node_get_tuning(None, C.byref(t)) == N.SUX_EINVAL
    assert lib.sux_node_check(None) == N.SUX_EINVAL


def test_null_arguments_fail_with_einval_and_message():
    lib = N.load()
    assert lib.sux_node_create(None, 0, None) == N.SUX_EINVAL
    assert "NULL" in N.last_error()
    assert lib.sux_partitioner_create(None, None, None) == N.SUX_EINVAL
    assert lib.sux_buffer_release(None) == N.SUX_EINVAL
    assert lib.sux_plan_group(2, 0, 1, 1, None, None, None, None, None) == N.SUX_EINVAL


def _plan_ref(W, rank, M, R, gi):
    lo = lambda h: (h * R) // W  # noqa: E731
    sc = [sum(int(gi[rank, m, lo(h + 1)] - gi[rank, m, lo(h)]) for m in range(M)) for h in range(W)]
    rc = [sum(int(gi[g, m, lo(rank + 1)] - gi[g, m, lo(rank)]) for m in range(M)) for g in range(W)]
    sd = np.concatenate([[0], np.cumsum(sc)[:-1]]).tolist()
    rd = np.concatenate([[0], np.cumsum(rc)[:-1]]).tolist()
    return sc, sd, rc, rd


@pytest.mark.parametrize("W,M,R", [(1, 1, 1), (2, 3, 8), (4, 2, 200), (8, 5, 200), (3, 4, 10)])
def test_plan_group_matches_restatement(W, M, R):
    rng = np.random.default_rng(W * 100 + M)
    lengths = rng.integers(0, 5, size=(W, M, R)) * 100
    gi = np.zeros((W, M, R + 1), np.int64)
    gi[:, :, 1:] = np.cumsum(lengths, axis=2)
    lib = N.load()
    for rank in range(W):
        out = [(C.c_uint64 * W)() for _ in range(4)]
        rc = lib.sux_plan_group(W, rank, M, R, gi.ctypes.data, *out)
        assert rc == 0, N.last_error()
        got = [list(o) for o in out]
        assert got == [list(x) for x in _plan_ref(W, rank, M, R, gi)]
        # block offsets tile rank's receive buffer exactly, in [source][map][partition] order
        lo, hi = (rank * R) // W, ((rank + 1) * R) // W
        pos = 0
        for g in range(W):
            for m in range(M):
                for p in range(lo, hi):
                    off = lib.sux_plan_block_offset(W, rank, M, R, gi.ctypes.data, g, m, p)
                    assert off == pos
                    pos += int(gi[g, m, p + 1] - gi[g, m, p])
        assert pos == sum(got[2])
        if hi < R:
            assert lib.sux_plan_block_offset(W, rank, M, R, gi.ctypes.data, 0, 0, hi) == -1


def test_bench_bounds_match_oracle():
    import bench
    from oracle import oracle as O

    for R in (2, 7, 200, 10000):
        assert bench.uniform_bounds(R) == O.uniform_range_bounds(R, 10)


@pytest.mark.parametrize("blocks", [
    [(0, 1), (3, 4), (2, 0)],                       # (map, partition): end = start + 1
    [(0, 1, 5), (3, 4, 4), (2, 0, 9)],              # (map, start, end)
    [(0, 1), (3, 4, 7)],                            # ragged: the per-block path
    np.array([[0, 1], [3, 4], [2, 0]], np.int32),
    np.array([[0, 1, 5], [3, 4, 4]], np.int64),
    [],
])
def test_block_lists_convert_the_same_by_every_path(blocks):
    """Node._blocks (the sux_block_id array of sux_fetch_blocks / sux_resolve_blocks) gives the same
    ids for tuples, uniform tuples (one numpy conversion) and arrays."""
    from sparkucx_amd.shuffle import Node

    arr = Node._blocks(blocks)
    want = [(int(b[0]), int(b[1]), int(b[2]) if len(b) > 2 else int(b[1]) + 1, 0) for b in blocks]
    got = [tuple(int(x) for x in row) for row in arr][:len(want)] if want else []
    assert got == want
    assert len(arr) == max(1, len(want))


def test_group_ranks_executors_by_first_arrival():
    """sux_group (the driver's Hello handling, GpuNode.scala): eight executors with identical
    confs get ranks 0..7 in arrival order, a repeated hello its own rank back, local indices per
    host, and a ninth executor SUX_ERANGE.  Host-only: no HIP call."""
    lib = N.load()
    g = C.c_void_p()
    assert lib.sux_group_create(8, C.byref(g)) == 0
    try:
        order = [5, 2, 7, 0, 3, 1, 6, 4]
        got = {}
        for k, e in enumerate(order):
            r, l = C.c_int32(), C.c_int32()
            host = b"hostA" if e % 2 == 0 else b"hostB"
            assert lib.sux_group_join(g, f"exec-{e}".encode(), host, C.byref(r), C.byref(l)) == 0
            got[e] = (r.value, l.value)
            assert r.value == k
        assert sorted(v[0] for v in got.values()) == list(range(8))
        for host_parity in (0, 1):
            locals_ = [got[e][1] for e in order if e % 2 == host_parity]
            assert locals_ == [0, 1, 2, 3]
        r, l = C.c_int32(), C.c_int32()
        assert lib.sux_group_join(g, b"exec-7", b"hostB", C.byref(r), C.byref(l)) == 0
        assert (r.value, l.value) == got[7]
        assert lib.sux_group_join(g, b"exec-8", b"hostA", C.byref(r), C.byref(l)) == N.SUX_ERANGE
        assert lib.sux_group_join(g, b"", b"hostA", C.byref(r), C.byref(l)) == N.SUX_EINVAL
        n = C.c_int32()
        assert lib.sux_group_size(g, C.byref(n)) == 0 and n.value == 8
    finally:
        assert lib.sux_group_destroy(g) == 0


def test_decompress_entry_points_validate_arguments():
    """sux_decompress_blocks / _workspace_size (the reader's side of spark.shuffle.compress):
    block-size range, block count, NULL arguments — all checked before any HIP call."""
    lib = N.load()
    b = C.c_uint64()
    assert lib.sux_decompress_workspace_size(1 << 20, 10, 32768, C.byref(b)) == 0 and b.value > 0
    small = b.value
    assert lib.sux_decompress_workspace_size(1 << 30, 10, 32768, C.byref(b)) == 0 and b.value > small
    for bs in (0, 63, 65537):
        assert lib.sux_decompress_workspace_size(1 << 20, 10, bs, C.byref(b)) == N.SUX_EINVAL
        assert "max_block_size" in N.last_error()
    assert lib.sux_decompress_workspace_size(1 << 20, -1, 32768, C.byref(b)) == N.SUX_EINVAL
    assert lib.sux_decompress_workspace_size(1 << 20, 10, 32768, None) == N.SUX_EINVAL
    assert lib.sux_decompress_blocks(None, None, 0, None, 0, 32768, None, 0, None, None, 0,
                                     None) == N.SUX_EINVAL
