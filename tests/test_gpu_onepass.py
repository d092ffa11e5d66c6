"""GPU parity of the one-pass map side (sux_onepass.hip) — map batch held on chip, one launch.

The one-pass kernel is opt-in (sux_tuning.onepass = 1, per node) for 100-byte records when a map
batch fits the grid (<= 256 records per workgroup, 2 workgroups per CU) and R's LDS image fits;
otherwise, and by default, the three-kernel path runs.
Both are checked bit-exact against the oracle (P1-P3: data bytes, native + big-endian index,
pids), and against each other at full map size (131072-record maps, size-independent check).
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


def run(node, opart, drecs, n, rs, rpm, pids=True):
    gp = gpu_part(node, opart)
    pd = torch.full((max(1, n),), -1, dtype=torch.int16, device="cuda") if pids else None
    out, index, index_be = node.partition_maps(gp, drecs, rs, rpm, num_records=n, pids=pd)
    torch.cuda.synchronize()
    gp.close()
    return out, index, index_be, pd


def check(node, opart, recs, rpm, tuned, onepass=True):
    tuned(onepass=1 if onepass else 0)
    n = recs.size // 100
    out, index, index_be, pd = run(node, opart, torch.from_numpy(recs).cuda(), n, 100, rpm)
    want_data, want_index, want_be = O.write_maps(opart, recs, 100, rpm)
    maps = -(-n // rpm)
    assert host(out)[: n * 100].tobytes() == bytes(want_data), "data bytes differ"
    assert host(index)[: maps * (opart.R + 1)].tolist() == want_index.tolist()
    assert host(index_be)[: maps * (opart.R + 1) * 8].tobytes() == want_be
    assert (host(pd)[:n].view(np.uint16) == opart.ids(recs, 100)).all()


@pytest.mark.parametrize("R", [1, 2, 3, 7, 64, 200, 256])
@pytest.mark.parametrize("onepass", [True, False])
def test_range_R(gpu_node, tuned, R, onepass):
    recs = O.gen_terasort(21, 0, 30000)
    check(gpu_node, O.terasort_partitioner(R), recs, 30000, tuned, onepass)


@pytest.mark.parametrize("n,rpm", [(1, 1), (255, 255), (256, 256), (257, 257), (1000, 7),
                                   (5000, 1024), (70000, 65536), (131072, 131072),
                                   (300000, 131071), (262145, 131072)])
def test_map_shapes(gpu_node, tuned, n, rpm):
    """Slices of 1..1024 records, empty slices, ragged last maps, many maps per launch."""
    recs = O.gen_terasort(22, 0, n)
    check(gpu_node, O.terasort_partitioner(200), recs, rpm, tuned)


@pytest.mark.parametrize("kind,key_len,off", [(O.MURMUR3_LONG, 8, 0), (O.MURMUR3_LONG, 8, 92),
                                              (O.MURMUR3_INT, 4, 4), (O.HASH_LONG, 8, 8),
                                              (O.HASH_INT, 4, 0), (O.RANGE_BYTES, 16, 0),
                                              (O.RANGE_BYTES, 5, 4)])
def test_kinds(gpu_node, tuned, kind, key_len, off):
    recs = O.gen_zipf(23, 0, 40000, 1.1, 1 << 16)
    b = O.uniform_range_bounds(200, key_len) if kind == O.RANGE_BYTES else None
    check(gpu_node, O.Partitioner(kind, 200, off, key_len, seed=42, bounds=b), recs, 20000,
          tuned)


def test_skew_one_partition(gpu_node, tuned):
    """Every record in one partition (one run of the whole map), and a Zipf-skewed map."""
    recs = O.gen_terasort(24, 0, 50000).reshape(-1, 100)
    recs[:, :10] = 0xFF
    check(gpu_node, O.terasort_partitioner(200), recs.ravel(), 50000, tuned)
    recs = O.gen_zipf(0x5EED0004, 0, 100000, 1.1, 1 << 24)
    check(gpu_node, O.Partitioner(O.MURMUR3_LONG, 200, 0, 8, seed=42), recs, 100000, tuned)


def test_unaligned_record_base(gpu_node, tuned):
    """The map group starts 4 bytes into a 16-byte unit (record loads straddle units)."""
    n = 9000
    recs = O.gen_terasort(25, 0, n)
    buf = torch.zeros(n * 100 + 16, dtype=torch.uint8, device="cuda")
    buf[4:4 + n * 100] = torch.from_numpy(recs).cuda()
    opart = O.terasort_partitioner(200)
    for onepass in ("1", "0"):
        tuned(onepass=int(onepass))
        out, index, _, _ = run(gpu_node, opart, buf[4:4 + n * 100], n, 100, 4000)
        want_data, want_index, _ = O.write_maps(opart, recs, 100, 4000)
        assert host(out)[: n * 100].tobytes() == bytes(want_data)
        assert host(index).tolist()[: len(want_index)] == want_index.tolist()


@pytest.mark.parametrize("R", [200, 256])
def test_full_size_maps_equal_three_kernel_path(gpu_node, tuned, R):
    """64 maps of 131072 TeraSort records (0.84 GB, the bench map shape): one-pass output,
    index tables and pids identical to the three-kernel path's (both parity-checked above)."""
    n, rpm = 64 * 131072, 131072
    opart = O.terasort_partitioner(R)
    d = gpu_node.generate(N.GEN_TERASORT, 0x5EED0002, 0, n, 100)
    tuned(onepass=1)
    a = run(gpu_node, opart, d, n, 100, rpm)
    tuned(onepass=0)
    b = run(gpu_node, opart, d, n, 100, rpm)
    for x, y in zip(a, b):
        assert torch.equal(x, y)
    idx = a[1].view(-1, R + 1)
    assert int(idx[:, 0].abs().sum()) == 0 and bool((idx[:, R] == rpm * 100).all())
    assert bool((idx[:, 1:] >= idx[:, :-1]).all())


def test_repeated_launches_same_workspace(gpu_node, tuned):
    """The sync words are reset per launch: back-to-back launches on one workspace agree."""
    tuned(onepass=1)
    n, rpm = 3 * 131072, 131072
    opart = O.terasort_partitioner(200)
    gp = gpu_part(gpu_node, opart)
    d = gpu_node.generate(N.GEN_TERASORT, 7, 0, n, 100)
    ws = torch.empty(gpu_node.workspace_size(gp, 100, rpm, n), dtype=torch.uint8, device="cuda")
    outs = []
    for _ in range(4):
        out, index, _ = gpu_node.partition_maps(gp, d, 100, rpm, workspace=ws)
        outs.append((out, index))
    torch.cuda.synchronize()
    for o, i in outs[1:]:
        assert torch.equal(o, outs[0][0]) and torch.equal(i, outs[0][1])
    want_data, want_index, _ = O.write_maps(opart, host(d), 100, rpm)
    assert host(outs[0][0]).tobytes() == bytes(want_data)
    gp.close()


def test_cu_masked_stream(gpu_node, tuned):
    """On a stream masked to 224 CUs the grid is sized to the stream's CUs (448 workgroups, all
    resident) — the same bytes as the oracle."""
    tuned(onepass=1)
    recs = O.gen_terasort(26, 0, 250_000)
    opart = O.terasort_partitioner(200)
    gp = gpu_part(gpu_node, opart)
    st = gpu_node.cu_stream(32, complement=True)
    try:
        ts = torch.cuda.ExternalStream(st)
        drecs = torch.from_numpy(recs).cuda()
        ts.wait_stream(torch.cuda.current_stream())
        out, index, _ = gpu_node.partition_maps(gp, drecs, 100, 100_000, stream=ts)
        ts.synchronize()
        want_data, want_index, _ = O.write_maps(opart, recs, 100, 100_000)
        assert host(out).tobytes() == bytes(want_data)
        assert host(index).tolist() == want_index.tolist()
    finally:
        gpu_node.destroy_stream(st)
        gp.close()
