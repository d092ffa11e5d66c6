"""GPU parity: variable-length rows in Spark SQL's UnsafeRowSerializer framing (SURVEY.md §8f
item 3) — the map-side P1-P3 of sux_partition_varlen against oracle.varlen_write_maps.

Bit-exact: data bytes, native and big-endian index (byte offsets), partition ids.
"""
import numpy as np
import pytest
import torch

from oracle import oracle as O
from sparkucx_amd import native as N
from sparkucx_amd.native import SuxError

pytestmark = pytest.mark.gpu


def to_dev(a: np.ndarray) -> torch.Tensor:
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def run(node, part, data, offs, rpm, pids_in=None):
    n = offs.size - 1
    d = to_dev(data) if data.size else torch.zeros(4, dtype=torch.uint8, device="cuda")
    o = to_dev(offs.astype(np.int64))
    pids = torch.empty(max(1, n), dtype=torch.int16, device="cuda")
    pin = None if pids_in is None else to_dev(pids_in.astype(np.int16))
    out, ix, be = node.partition_varlen(part, d, o, rpm, pids_in=pin,
                                        pids=None if pin is not None else pids)
    torch.cuda.synchronize()
    return (out.cpu().numpy()[: data.size], ix.cpu().numpy(), be.cpu().numpy().tobytes(),
            pids.cpu().numpy().view(np.uint16)[:n])


def check(node, R, data, offs, rpm, kind=O.MURMUR3_LONG, key_offset=12, key_len=8, bounds=None,
          pids_in=None):
    gp = node.partitioner(kind, R, key_offset=key_offset, key_len=key_len, bounds=bounds)
    op = O.Partitioner(kind, R, key_offset, key_len, bounds=bounds)
    out, ix, be, pids = run(node, gp, data, offs, rpm, pids_in)
    eo, eix, ebe, epids = O.varlen_write_maps(op, data, offs, rpm, R=R, pids=pids_in)
    n = offs.size - 1
    if pids_in is None and n:
        assert np.array_equal(pids, epids)
    maps = -(-n // rpm) if n else 0
    assert np.array_equal(ix[: maps * (R + 1)], eix)
    assert be[: maps * (R + 1) * 8] == ebe
    assert out.tobytes() == eo.tobytes()


@pytest.mark.parametrize("n,rpm", [(0, 10), (1, 1), (63, 64), (1000, 300), (50_000, 7_001),
                                   (300_000, 100_000)])
@pytest.mark.parametrize("R", [1, 7, 200])
def test_spark_sql_hash(gpu_node, n, rpm, R):
    data, offs = O.gen_unsafe_rows(100 + n, n)
    check(gpu_node, R, data, offs, rpm)


@pytest.mark.parametrize("R", [2048, 2049, 10_000, 16_384])
def test_many_partitions(gpu_node, R):
    """R past the 4-waves-per-workgroup LDS budget: one wave per workgroup."""
    data, offs = O.gen_unsafe_rows(R, 120_000)
    check(gpu_node, R, data, offs, 50_000)


def test_caller_pids(gpu_node):
    """Spark SQL projects the partition id itself: ids passed in replace the partitioner."""
    rng = np.random.default_rng(5)
    data, offs = O.gen_unsafe_rows(6, 80_000)
    pids = rng.integers(0, 333, offs.size - 1).astype(np.uint16)
    check(gpu_node, 333, data, offs, 30_000, pids_in=pids)


def test_range_key_inside_rows(gpu_node):
    """RangePartitioner on a 10-byte binary key inside the row (bytes 12..21)."""
    data, offs = O.gen_unsafe_rows(7, 40_000)
    check(gpu_node, 200, data, offs, 15_000, kind=O.RANGE_BYTES, key_len=10,
          bounds=O.uniform_range_bounds(200, 10))


def test_int_key_and_skewed(gpu_node):
    """Murmur3 int key at 12 (low half of the long field); few distinct keys -> hot partitions."""
    data, offs = O.gen_unsafe_rows(8, 100_000, key_mod=5)
    check(gpu_node, 64, data, offs, 100_000, kind=O.MURMUR3_INT, key_len=4)


def test_long_rows_and_offset_base(gpu_node):
    """Rows up to ~16 KiB, and offsets that start past 0 (a slice of a larger buffer)."""
    d0, o0 = O.gen_unsafe_rows(9, 2_000, max_payload_words=2_000)
    shift = 4096
    check(gpu_node, 31, d0, o0 + shift, 700)


def test_empty_partitions_and_single_map(gpu_node):
    data, offs = O.gen_unsafe_rows(10, 5, max_payload_words=0)
    check(gpu_node, 1000, data, offs, 5)


def test_rejects_bad_arguments(gpu_node):
    data, offs = O.gen_unsafe_rows(11, 100)
    big = gpu_node.partitioner(O.MURMUR3_LONG, 20_000, key_offset=12, key_len=8)
    with pytest.raises(SuxError):
        gpu_node.partition_varlen(big, to_dev(data), to_dev(offs), 100)
    p = gpu_node.partitioner(O.MURMUR3_LONG, 16, key_offset=12, key_len=8)
    with pytest.raises(SuxError):
        gpu_node.partition_varlen(p, to_dev(data)[1:], to_dev(offs), 100)  # misaligned data


def test_full_size_properties(gpu_node):
    """8 maps x 1 Mi rows (~0.7 GB): per map, the output is a permutation of its rows grouped by
    partition — each partition's byte run parses as whole frames whose keys hash to it, and the
    index matches the per-partition byte sums computed from the GPU's own pids."""
    n, rpm, R = 8 << 20, 1 << 20, 200
    data, offs = O.gen_unsafe_rows(12, n, max_payload_words=8)
    gp = gpu_node.partitioner(O.MURMUR3_LONG, R, key_offset=12, key_len=8)
    out, ix, be, pids = run(gpu_node, gp, data, offs, rpm)
    lens = np.diff(offs)
    ix = ix.reshape(-1, R + 1)
    for m in range(n // rpm):
        sl = slice(m * rpm, (m + 1) * rpm)
        sizes = np.bincount(pids[sl].astype(np.int64), weights=lens[sl], minlength=R)
        assert np.array_equal(np.diff(ix[m]), sizes.astype(np.int64))
    # the 4-byte frame lengths chain through every map's output and the keys hash to their run
    pos, frames = 0, 0
    b = out
    starts = []
    while pos < b.size and frames < 200_000:
        starts.append(pos)
        pos += 4 + int.from_bytes(b[pos:pos + 4].tobytes(), "big")
        frames += 1
    starts = np.array(starts)
    keys = b[starts[:, None] + 12 + np.arange(8)].copy().view("<i8").ravel()
    op = O.Partitioner(O.MURMUR3_LONG, R, 0, 8)
    kp = op.ids(keys.view(np.uint8), 8).astype(np.int64)
    run_of = np.searchsorted(ix[0][1:], starts, side="right")
    assert np.array_equal(kp, run_of)
    assert np.array_equal(np.sort(out[: offs[rpm]]), np.sort(data[: offs[rpm]]))


# ---- k_vscatter3 (128-byte line image, varlen_kernel 3) ----------------------------------------
V3_SHAPES = [  # (seed, n, rpm, R, max_payload_words, key_mod, varlen_tile)
    (20, 1, 1, 7, 12, None, 0),
    (21, 63, 64, 200, 12, None, 0),
    (22, 1000, 300, 1, 12, None, 0),
    (23, 50_000, 7_001, 200, 12, None, 0),
    (24, 300_000, 100_000, 215, 12, None, 0),
    (25, 120_000, 40_000, 246, 12, None, 0),   # the LDS limit
    (26, 120_000, 40_000, 247, 12, None, 0),   # past it: k_vscatter2
    (27, 50_000, 100, 64, 12, None, 64),       # 500 maps of 2 tiles: items of one map per range
    (28, 200_000, 200_000, 31, 12, 5, 0),      # 5 distinct keys: hot partitions, long runs
    (29, 3_000, 1_000, 17, 2_000, None, 0),    # rows up to 16 KiB
    (30, 400, 150, 9, 8_189, None, 0),         # rows up to 64 KiB - 4: one or two per chunk
    (31, 100_000, 30_000, 100, 0, None, 64),   # 20-byte rows only
]


@pytest.mark.parametrize("shape", V3_SHAPES, ids=lambda s: f"n{s[1]}-rpm{s[2]}-R{s[3]}-w{s[4]}")
def test_line_image_scatter(gpu_node, tuned, shape):
    seed, n, rpm, R, mw, kmod, tile = shape
    tuned(varlen_kernel=3, varlen_tile=tile)
    data, offs = O.gen_unsafe_rows(seed, n, max_payload_words=mw, key_mod=kmod)
    check(gpu_node, R, data, offs, rpm)


@pytest.mark.parametrize("lead", [4, 8, 12])
def test_line_image_scatter_unaligned_buffers(gpu_node, tuned, lead):
    """Rows and output starting 4, 8 or 12 bytes past a 16-byte boundary: the window's first unit
    holds bytes before the rows, and every line of the output is shifted."""
    tuned(varlen_kernel=3)
    R, rpm = 77, 9_000
    data, offs = O.gen_unsafe_rows(40 + lead, 30_000)
    gp = gpu_node.partitioner(O.MURMUR3_LONG, R, key_offset=12, key_len=8)
    op = O.Partitioner(O.MURMUR3_LONG, R, 12, 8)
    buf = torch.zeros(data.size + 64, dtype=torch.uint8, device="cuda")
    buf[lead:lead + data.size] = to_dev(data)
    obuf = torch.zeros(data.size + 64, dtype=torch.uint8, device="cuda")
    d = buf[lead:lead + data.size]
    o = obuf[lead:lead + data.size]
    out, ix, be = gpu_node.partition_varlen(gp, d, to_dev(offs.astype(np.int64)), rpm, out=o)
    torch.cuda.synchronize()
    eo, eix, ebe, _ = O.varlen_write_maps(op, data, offs, rpm, R=R)
    maps = -(-(offs.size - 1) // rpm)
    assert np.array_equal(ix.cpu().numpy()[: maps * (R + 1)], eix)
    assert obuf.cpu().numpy()[lead:lead + data.size].tobytes() == eo.tobytes()
    assert not obuf[:lead].any() and not obuf[lead + data.size:].any()  # nothing outside


def test_line_image_scatter_full_size(gpu_node, tuned):
    """The bench's shape (1 Mi-row maps, R = 200), 4 maps: bit-exact against the oracle."""
    tuned(varlen_kernel=3)
    data, offs = O.gen_unsafe_rows(50, 4 << 20)
    check(gpu_node, 200, data, offs, 1 << 20)
