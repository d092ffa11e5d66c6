"""GPU parity: the reduce-side sort (the reader's ExternalSorter step,
compat/spark_3_0/UcxShuffleReader.scala:138-154) through the C-ABI against the CPU oracle.

Bit-exact output bytes: ascending key order, input order kept for equal keys.
"""
import numpy as np
import pytest
import torch

from oracle import oracle as O
from sparkucx_amd import native as N

pytestmark = pytest.mark.gpu


def to_dev(a: np.ndarray) -> torch.Tensor:
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def gpu_sort(node, recs, rs, kind, off, klen):
    n = recs.size // rs
    d = to_dev(recs) if recs.size else torch.zeros(4, dtype=torch.uint8, device="cuda")
    out = node.sort_records(d, rs, kind, off, klen, num_records=n)
    torch.cuda.synchronize()
    return out.cpu().numpy()[: n * rs]


@pytest.mark.parametrize("n", [0, 1, 63, 1000, 4097, 100_000, 1_000_000])
def test_terasort_keys(gpu_node, n):
    recs = O.gen_terasort(21, 0, n)
    got = gpu_sort(gpu_node, recs, 100, N.SORT_BYTES, 0, 10)
    assert got.tobytes() == O.sort_records(recs, 100, O.SORT_BYTES, 0, 10).tobytes()


def test_duplicate_keys_are_stable(gpu_node):
    """Few distinct keys: the order of equal keys must be the input order (row ids rise)."""
    rng = np.random.default_rng(3)
    recs = O.gen_terasort(22, 0, 200_000).reshape(-1, 100)
    recs[:, :10] = 0
    recs[:, 8:10] = rng.integers(0, 3, (recs.shape[0], 2), dtype=np.uint8)  # 9 distinct keys
    got = gpu_sort(gpu_node, recs.ravel(), 100, N.SORT_BYTES, 0, 10)
    assert got.tobytes() == O.sort_records(recs.ravel(), 100, O.SORT_BYTES, 0, 10).tobytes()


@pytest.mark.parametrize("rs,off,klen", [(20, 3, 7), (16, 0, 12), (8, 4, 1), (4096, 100, 10)])
def test_byte_keys_shapes(gpu_node, rs, off, klen):
    n = 3000 if rs < 1000 else 500
    rng = np.random.default_rng(rs)
    recs = rng.integers(0, 256, n * rs, dtype=np.uint8)
    got = gpu_sort(gpu_node, recs, rs, N.SORT_BYTES, off, klen)
    assert got.tobytes() == O.sort_records(recs, rs, O.SORT_BYTES, off, klen).tobytes()


def test_signed_long_and_int_keys(gpu_node):
    recs = O.gen_small(23, 0, 300_000)  # int64 key (full range, negatives included) + value
    got = gpu_sort(gpu_node, recs, 16, N.SORT_LONG, 0, 8)
    assert got.tobytes() == O.sort_records(recs, 16, O.SORT_LONG, 0, 8).tobytes()
    got = gpu_sort(gpu_node, recs, 16, N.SORT_INT, 8, 4)
    assert got.tobytes() == O.sort_records(recs, 16, O.SORT_INT, 8, 4).tobytes()


def test_validation(gpu_node):
    x = torch.zeros(1600, dtype=torch.uint8, device="cuda")
    for kind, off, klen in [(N.SORT_BYTES, 0, 13), (N.SORT_LONG, 0, 4), (N.SORT_BYTES, 95, 10),
                            (9, 0, 4)]:
        with pytest.raises(N.SuxError) as e:
            gpu_node.sort_records(x, 100, kind, off, klen, num_records=16)
        assert e.value.code == N.SUX_EINVAL
    with pytest.raises(N.SuxError):
        gpu_node.sort_records(x, 100, N.SORT_BYTES, 0, 10, num_records=16, out=x)


def test_fetch_then_sort_one_reduce_partition(gpu_node):
    """Reduce task end to end: map outputs -> fetch one partition's blocks in map order
    (UcxShuffleClient.fetchBlocks) -> sort by key (ExternalSorter)."""
    R, rs, maps, per = 16, 100, 5, 20_000
    recs = O.gen_terasort(24, 0, maps * per)
    opart = O.terasort_partitioner(R)
    part = gpu_node.partitioner(N.PART_RANGE_BYTES, R, key_offset=0, key_len=10,
                                bounds=opart.bounds)
    gpu_node.register_shuffle(77, maps, R, rs)
    d = to_dev(recs)
    for m in range(maps):
        gpu_node.write_map_output(77, m, part, d[m * per * rs:(m + 1) * per * rs], per)
    p = 9
    buf, sizes = gpu_node.fetch_blocks(77, [(m, p) for m in range(maps)])
    fetched = np.frombuffer(buf.to_bytes(), dtype=np.uint8)
    buf.release(maps)
    want_blocks = []
    for m in range(maps):
        data, _, index, _ = O.write_map(opart, recs[m * per * rs:(m + 1) * per * rs], rs)
        want_blocks.append(bytes(data[index[p]:index[p + 1]]))
    assert fetched.tobytes() == b"".join(want_blocks)
    got = gpu_sort(gpu_node, fetched, rs, N.SORT_BYTES, 0, 10)
    assert got.tobytes() == O.sort_records(fetched, rs, O.SORT_BYTES, 0, 10).tobytes()
    gpu_node.unregister_shuffle(77)
    part.close()


def test_large_sort_properties(gpu_node):
    """10^7 records (1 GB): ascending keys and the same multiset of records (column sums)."""
    n = 10_000_000
    d = gpu_node.generate(N.GEN_TERASORT, 25, 0, n, 100)
    out = gpu_node.sort_records(d, 100, N.SORT_BYTES, 0, 10, num_records=n)
    torch.cuda.synchronize()
    a = d.view(n, 100)
    b = out.view(n, 100)
    # keys ascend: compare the first 8 key bytes as big-endian u64, then bytes 8..9
    kb = b[:, :10].cpu().numpy()
    hi = kb[:, :8].copy().view(">u8").ravel().astype(np.uint64)
    lo = (kb[:, 8].astype(np.uint32) << 8) | kb[:, 9]
    assert (hi[1:] >= hi[:-1]).all()
    eq = hi[1:] == hi[:-1]
    assert (lo[1:][eq] >= lo[:-1][eq]).all()
    # multiset: per-column byte sums agree (the generator's row id sits in bytes 10..17)
    assert torch.equal(a.sum(0, dtype=torch.int64), b.sum(0, dtype=torch.int64))


@pytest.mark.parametrize("nseg", [1, 2, 25, 300, 70_000])
def test_segmented_sort(gpu_node, nseg):
    """Every run sorted in place of itself (a reducer's owned partitions in one call); empty
    runs, 1-record runs and segment-id widths of 0..3 bytes."""
    n = 200_000
    rng = np.random.default_rng(nseg)
    cuts = np.sort(rng.integers(0, n + 1, nseg - 1))
    seg = np.concatenate([[0], cuts, [n]]).astype(np.int64)
    recs = O.gen_terasort(24, 0, n)
    key_len = 10 if nseg <= 65536 else 9
    segs = torch.from_numpy(seg).cuda()
    out = gpu_node.sort_segments(to_dev(recs), 100, N.SORT_BYTES, 0, key_len, segs)
    torch.cuda.synchronize()
    exp = O.sort_segments(recs, 100, O.SORT_BYTES, 0, key_len, seg)
    assert out.cpu().numpy()[: n * 100].tobytes() == exp.tobytes()


def test_segmented_sort_long_keys(gpu_node):
    recs = O.gen_small(25, 0, 100_000)
    seg = np.array([0, 10, 10, 50_000, 99_999, 100_000], np.int64)
    out = gpu_node.sort_segments(to_dev(recs), 16, N.SORT_LONG, 0, 8,
                                 torch.from_numpy(seg).cuda())
    torch.cuda.synchronize()
    exp = O.sort_segments(recs, 16, O.SORT_LONG, 0, 8, seg)
    assert out.cpu().numpy()[: recs.size].tobytes() == exp.tobytes()


def _long_recs(keys: np.ndarray) -> np.ndarray:
    recs = np.zeros((keys.size, 16), np.uint8)
    recs[:, :8] = keys.astype("<i8").view(np.uint8).reshape(-1, 8)
    recs[:, 8:] = np.arange(keys.size, dtype="<u8").view(np.uint8).reshape(-1, 8)
    return recs.ravel()


@pytest.mark.parametrize("lo,hi,n", [(0, 1 << 20, 1_500_000),   # top digits constant: skipped
                                     (7, 8, 100_000),            # one key: every pass skipped
                                     (-3, 3, 200_000),           # sign flips: every digit varies
                                     (1 << 40, (1 << 40) + 4096, 600_000)])
def test_long_keys_constant_digits(gpu_node, lo, hi, n):
    """Digit passes whose bits never vary are skipped (k_sort_pairs' AND/OR key span): the
    result must still be the oracle's, including the grid-stride walk past 2048 x 256 records."""
    keys = np.random.default_rng(n).integers(lo, hi, n, dtype=np.int64)
    recs = _long_recs(keys)
    got = gpu_sort(gpu_node, recs, 16, N.SORT_LONG, 0, 8)
    assert got.tobytes() == O.sort_records(recs, 16, O.SORT_LONG, 0, 8).tobytes()


def test_byte_keys_one_varying_middle_byte(gpu_node):
    recs = O.gen_terasort(26, 0, 50_000).reshape(-1, 100)
    recs[:, :10] = 0x5A
    recs[:, 4] = np.random.default_rng(4).integers(0, 256, recs.shape[0], dtype=np.uint8)
    got = gpu_sort(gpu_node, recs.ravel(), 100, N.SORT_BYTES, 0, 10)
    assert got.tobytes() == O.sort_records(recs.ravel(), 100, O.SORT_BYTES, 0, 10).tobytes()


def test_segmented_sort_equal_keys(gpu_node):
    """Keys all equal: only the segment-id digits are sorted; each run keeps its order."""
    recs = _long_recs(np.full(30_000, 42, np.int64))
    seg = np.array([0, 7, 7, 20_000, 30_000], np.int64)
    out = gpu_node.sort_segments(to_dev(recs), 16, N.SORT_LONG, 0, 8,
                                 torch.from_numpy(seg).cuda())
    torch.cuda.synchronize()
    exp = O.sort_segments(recs, 16, O.SORT_LONG, 0, 8, seg)
    assert out.cpu().numpy()[: recs.size].tobytes() == exp.tobytes()
    assert exp.tobytes() == recs.tobytes()


def test_long_sort_long_tiles(gpu_node):
    """17 Mi records: the sort plan grows its tiles to 65536 records (>= 256 tiles remain);
    bit-exact against the oracle."""
    n = 17 << 20
    keys = np.random.default_rng(17).integers(-(1 << 62), 1 << 62, n, dtype=np.int64)
    recs = _long_recs(keys)
    got = gpu_sort(gpu_node, recs, 16, N.SORT_LONG, 0, 8)
    assert got.tobytes() == O.sort_records(recs, 16, O.SORT_LONG, 0, 8).tobytes()


@pytest.mark.parametrize("rs,kind,off,klen", [(12, N.SORT_INT, 4, 4), (8, N.SORT_BYTES, 2, 3),
                                              (16, N.SORT_BYTES, 5, 11), (4, N.SORT_INT, 0, 4),
                                              (16, N.SORT_LONG, 8, 8)])
def test_inline_small_records(gpu_node, rs, kind, off, klen):
    """Records of <= 16 bytes ride inside the sort pairs (no gather): key bytes anywhere in the
    record, signed and unsigned kinds, ties kept in input order."""
    n = 70_000
    rng = np.random.default_rng(rs * 100 + off)
    recs = rng.integers(0, 256, (n, rs), dtype=np.uint8)
    recs[: n // 2, off:off + min(klen, 2)] = 7  # many equal leading key bytes / ties
    got = gpu_sort(gpu_node, recs.ravel(), rs, kind, off, klen)
    assert got.tobytes() == O.sort_records(recs.ravel(), rs, kind, off, klen).tobytes()


@pytest.mark.parametrize("nseg", [3, 300])
def test_segmented_inline_small_records(gpu_node, nseg):
    """8-byte records with a 1-2 byte segment id still fit a pair (inline mode)."""
    n, rs = 50_000, 8
    rng = np.random.default_rng(nseg)
    recs = rng.integers(0, 256, n * rs, dtype=np.uint8)
    seg = np.concatenate([[0], np.sort(rng.integers(0, n + 1, nseg - 1)), [n]]).astype(np.int64)
    out = gpu_node.sort_segments(to_dev(recs), rs, N.SORT_INT, 4, 4, torch.from_numpy(seg).cuda())
    torch.cuda.synchronize()
    exp = O.sort_segments(recs, rs, O.SORT_INT, 4, 4, seg)
    assert out.cpu().numpy()[: n * rs].tobytes() == exp.tobytes()


@pytest.mark.parametrize("msd", [1, 2, 3])
@pytest.mark.parametrize("shape", ["terasort", "skewed_top", "skewed_top9", "long", "int_inline",
                                   "distinct50", "distinct50_k9", "skewed_const_mid"])
def test_msd_finish_and_lsd_agree_with_oracle(gpu_node, tuned, msd, shape):
    """sort_msd 1: the top digit (chunked: each 4096-pair chunk sorted in place, buckets read as
    runs) + every bucket sorted by the lower digits (k_sort_local in LDS; k_sort_bucket_global for
    a bucket above the LDS capacity, copied out of its runs first); 3: the same after a one-pass
    top-digit partition; 2: LSD digit passes only.
    'skewed_top' / 'skewed_top9': 60 % of the keys share their top bytes, so one bucket passes the
    LDS capacity and is sorted through global memory (10- and 9-byte keys: both parities of its
    digit count).  'distinct50*': 50 distinct keys, so every non-empty bucket holds ~6 000 equal
    keys and k_sort_bucket_global skips every digit (its per-bucket key span); 'skewed_const_mid':
    the big bucket's middle key bytes are constant, so it skips some digits and runs others."""
    tuned(sort_msd=msd)
    if shape in ("distinct50", "distinct50_k9"):
        recs = O.gen_terasort(65, 0, 300_000).reshape(-1, 100)
        pick = np.random.default_rng(65).integers(0, 50, recs.shape[0])
        recs[:, :10] = recs[:50, :10][pick]
        klen = 10 if shape == "distinct50" else 9
        recs, rs, kind, off = recs.ravel(), 100, N.SORT_BYTES, 0
    elif shape == "skewed_const_mid":
        recs = O.gen_terasort(66, 0, 300_000).reshape(-1, 100)
        recs[: 180_000, :4] = 9
        recs[: 180_000, 4:7] = 77
        recs, rs, kind, off, klen = recs.ravel(), 100, N.SORT_BYTES, 0, 10
    elif shape == "terasort":
        recs, rs, kind, off, klen = O.gen_terasort(61, 0, 700_000), 100, N.SORT_BYTES, 0, 10
    elif shape in ("skewed_top", "skewed_top9"):
        recs = O.gen_terasort(62, 0, 300_000).reshape(-1, 100)
        recs[: 180_000, :4] = 9
        klen = 10 if shape == "skewed_top" else 9
        recs, rs, kind, off = recs.ravel(), 100, N.SORT_BYTES, 0
    elif shape == "long":
        recs, rs, kind, off, klen = O.gen_small(63, 0, 500_000), 16, N.SORT_LONG, 0, 8
    else:
        recs, rs, kind, off, klen = O.gen_small(64, 0, 400_000), 16, N.SORT_INT, 8, 4
    okind = {N.SORT_BYTES: O.SORT_BYTES, N.SORT_LONG: O.SORT_LONG, N.SORT_INT: O.SORT_INT}[kind]
    got = gpu_sort(gpu_node, recs, rs, kind, off, klen)
    assert got.tobytes() == O.sort_records(recs, rs, okind, off, klen).tobytes()
    gpu_node.check()


@pytest.mark.parametrize("msd", [1, 3])
@pytest.mark.parametrize("n", [1, 4095, 4096, 4097, 70_001, 1_000_000])
@pytest.mark.parametrize("kind", ["terasort", "top_only", "equal"])
def test_chunked_top_digit(gpu_node, tuned, msd, n, kind):
    """The chunked top pass (sort_msd 1) against the one-pass partition (3) and the oracle: chunk
    counts around the 4096-pair chunk (a partial last chunk, one exact chunk), top digits of 8..10
    bits; 'top_only': keys that vary only inside the top digit (no lower digit: every bucket is
    copied out of its runs in order); 'equal': one key (the plan's identity)."""
    tuned(sort_msd=msd)
    recs = O.gen_terasort(70, 0, n).reshape(-1, 100)
    if kind == "top_only":
        recs[:, 1:10] = 0
        recs[:, 0] = np.random.default_rng(70).integers(0, 256, n)
    elif kind == "equal":
        recs[:, :10] = recs[0, :10]
    recs = recs.ravel()
    got = gpu_sort(gpu_node, recs, 100, N.SORT_BYTES, 0, 10)
    assert got.tobytes() == O.sort_records(recs, 100, O.SORT_BYTES, 0, 10).tobytes()
    gpu_node.check()


@pytest.mark.parametrize("kind", ["random", "range_partition"])
def test_chunked_top_digit_4m(gpu_node, kind):
    """4 M records: the chunked top digit at 12 bits (4096 buckets of ~1 000 pairs);
    'range_partition': the keys of one of 200 TeraSort range partitions (first byte 0x80, or 0x81
    with the second below 0x47), whose buckets fill only part of the top digit, so some pass 2048
    pairs and take the side stream's 4096-pair shape."""
    n = 4_000_000
    recs = O.gen_terasort(71, 0, n).reshape(-1, 100)
    if kind == "range_partition":
        rng = np.random.default_rng(71)
        hi = rng.random(n) < 0.22
        recs[:, 0] = np.where(hi, 0x81, 0x80)
        recs[:, 1] = np.where(hi, rng.integers(0, 0x47, n), recs[:, 1])
    recs = recs.ravel()
    got = gpu_sort(gpu_node, recs, 100, N.SORT_BYTES, 0, 10)
    assert got.tobytes() == O.sort_records(recs, 100, O.SORT_BYTES, 0, 10).tobytes()
    gpu_node.check()


@pytest.mark.parametrize("base,width", [(0x7FFF_FFFF_FFF0_1234, 1 << 40),   # crosses 2^63
                                        (0x0123_4567_89AB_CDEF, 1 << 20),   # few blocks
                                        (0x8000_0000_0000_0000, 0x0147_AE14_7AE1_47AE),
                                        (0xFFFF_FFFF_0000_0007, (1 << 32) - 8)])  # ends at 2^64 - 1
def test_ranged_top_digit(gpu_node, base, width):
    """The chunked top digit over the key RANGE (round 5): the bucket of a key is its aligned
    block counted from the smallest key's, so keys that fill only part of the varying bits — a
    range partition's, or ones straddling a power of two, where the bit span put everything in
    two buckets — spread over every bucket.  Keys: 8-byte big-endian prefixes uniform in
    [base, base + width) (with their other two key bytes random), vs the oracle."""
    n = 600_000
    rng = np.random.default_rng(width & 0xFFFF)
    recs = O.gen_terasort(73, 0, n).reshape(-1, 100)
    k = (np.uint64(base) + (rng.random(n) * width).astype(np.uint64)).astype(">u8")
    recs[:, :8] = k.view(np.uint8).reshape(n, 8)
    recs = recs.ravel()
    got = gpu_sort(gpu_node, recs, 100, N.SORT_BYTES, 0, 10)
    assert got.tobytes() == O.sort_records(recs, 100, O.SORT_BYTES, 0, 10).tobytes()
    gpu_node.check()


@pytest.mark.parametrize("shape", ["tie_runs", "long_tie_runs"])
def test_lds_sort_tie_fixup_and_redo(gpu_node, shape):
    """k_sort_local sorts a bucket by its two most significant varying digits, then finishes the
    runs whose two digits tie with a stable insertion sort: 'tie_runs' leaves ~512 top-digit
    combinations per 781-pair bucket (short runs, fixed in place); 'long_tie_runs' leaves 4
    (runs of ~200 > 16: the bucket runs every digit pass instead).  Bytes vs the oracle."""
    rng = np.random.default_rng(91)
    n = 200_000
    recs = O.gen_terasort(92, 0, n).reshape(-1, 100)
    recs[:, :10] = 0
    recs[:, 0] = rng.integers(0, 256, n, dtype=np.uint8)           # the bucket digit
    if shape == "tie_runs":
        recs[:, 1] = rng.integers(0, 256, n, dtype=np.uint8)
        recs[:, 2] = rng.integers(0, 2, n, dtype=np.uint8)
        recs[:, 4] = rng.integers(0, 256, n, dtype=np.uint8)
    else:
        recs[:, 1] = rng.integers(0, 2, n, dtype=np.uint8)
        recs[:, 2] = rng.integers(0, 2, n, dtype=np.uint8)
        recs[:, 4] = rng.integers(0, 256, n, dtype=np.uint8)
        recs[:, 6] = rng.integers(0, 256, n, dtype=np.uint8)
    recs = recs.ravel()
    got = gpu_sort(gpu_node, recs, 100, N.SORT_BYTES, 0, 10)
    assert got.tobytes() == O.sort_records(recs, 100, O.SORT_BYTES, 0, 10).tobytes()
    gpu_node.check()


@pytest.mark.parametrize("shape", ["terasort", "skewed_top", "equal", "top_only", "long_small"])
def test_sort_records_captured_in_a_graph(gpu_node, shape):
    """sux_sort_records on a stream being captured into a HIP graph: the plan is made on the
    device (make_sort_plan, in the span reduction), so there is no host wait and no host allocation
    mid-capture, and every branch runs inside the graph — the LDS finish ('terasort'), the LSD
    fallback of a bucket above the LDS capacity ('skewed_top'), the identity of equal keys
    ('equal'), a key whose varying bits all sit in the top digit ('top_only': the result stays in
    the second pair buffer), int64 keys with constant top digits ('long_small').  Replays equal
    the oracle."""
    rng = np.random.default_rng(81)
    rs, kind, off, klen = 100, N.SORT_BYTES, 0, 10
    if shape == "terasort":
        h = O.gen_terasort(77, 0, 200_000)
    elif shape == "skewed_top":
        h = O.gen_terasort(78, 0, 150_000).reshape(-1, 100)
        h[:90_000, :4] = 5
        h = h.ravel()
    elif shape == "equal":
        h = O.gen_terasort(79, 0, 50_000).reshape(-1, 100)
        h[:, :10] = 7
        h = h.ravel()
    elif shape == "top_only":
        h = O.gen_terasort(80, 0, 60_000).reshape(-1, 100)
        h[:, :10] = 0
        h[:, 3] = rng.integers(0, 256, h.shape[0], dtype=np.uint8)  # 8 varying bits: one digit
        h = h.ravel()
    else:
        rows = np.zeros((300_000, 2), dtype=np.int64)
        rows[:, 0] = rng.integers(0, 1 << 20, rows.shape[0])
        rows[:, 1] = np.arange(rows.shape[0])
        h, rs, kind, off, klen = rows.view(np.uint8).ravel(), 16, N.SORT_LONG, 0, 8
    okind = {N.SORT_BYTES: O.SORT_BYTES, N.SORT_LONG: O.SORT_LONG}[kind]
    want = O.sort_records(h, rs, okind, off, klen)
    n = h.size // rs
    recs = to_dev(h)
    out = torch.empty_like(recs)
    ws = torch.empty(gpu_node.sort_workspace_size(n, rs), dtype=torch.uint8, device=recs.device)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        gpu_node.sort_records(recs, rs, kind, off, klen, out=out, workspace=ws, stream=s)
    for _ in range(2):  # two replays of the same graph
        out.zero_()
        g.replay()
        torch.cuda.synchronize()
        assert out.cpu().numpy().tobytes() == want.tobytes()
    gpu_node.check()


@pytest.mark.parametrize("gk", [1, 2, 3])
@pytest.mark.parametrize("rs,n", [(100, 300_000), (20, 50_000), (36, 7777), (44, 123_457), (1024, 3000),
                                  (1028, 3000), (4096, 500)])
def test_record_gather_kernels(gpu_node, tuned, gk, rs, n):
    """Every record gather (tuning gather_kernel: 1 = its own launch in 16-byte units with L lanes
    per record, 2 = one dword per lane, 3 = fused into the LDS bucket sort, records <= 1024 B)
    over record sizes with 0..3 tail dwords and L from 2 to 64."""
    tuned(gather_kernel=gk)
    rng = np.random.default_rng(rs + n)
    recs = rng.integers(0, 256, n * rs, dtype=np.uint8)
    got = gpu_sort(gpu_node, recs, rs, N.SORT_BYTES, 0, 10)
    assert got.tobytes() == O.sort_records(recs, rs, O.SORT_BYTES, 0, 10).tobytes()
