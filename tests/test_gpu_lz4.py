"""GPU parity: compressed map outputs (spark.shuffle.compress=true with the
lz4 codec) — sux_compress_map_outputs against oracle/lz4.c and against the system liblz4.

Bit-exact: the framed streams (headers, XXH32 checksums, LZ4 blocks, raw chunks, end marks) and
the index tables vs the oracle, whose compressor restates liblz4's LZ4_compress_default; and,
independently of the oracle, every chunk the GPU compressed is byte-for-byte the system
liblz4.so.1.9.3's LZ4_compress_default of that chunk (every raw chunk one liblz4 could not
shrink) — the bytes lz4-java's JNI compressor gives Spark's LZ4BlockOutputStream.
"""
import numpy as np
import pytest
import torch

from oracle import oracle as O

pytestmark = pytest.mark.gpu


def to_dev(a: np.ndarray) -> torch.Tensor:
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def run_gpu(node, data, index, maps, R, bs):
    d = to_dev(data) if data.size else torch.zeros(16, dtype=torch.uint8, device="cuda")
    out, oix, obe, nbytes = node.compress_map_outputs(d, to_dev(index), maps, R, bs,
                                                      data_bytes=data.size)
    torch.cuda.synchronize()
    n = int(nbytes.item())
    return out[:n].cpu().numpy().tobytes(), oix.cpu().numpy(), obe.cpu().numpy().tobytes()


def check(node, data, index, maps, R, bs):
    got, gix, gbe = run_gpu(node, data, index, maps, R, bs)
    exp, eix, ebe = O.lz4_map_outputs(data, index, maps, R, bs)
    assert np.array_equal(gix, eix)
    assert gbe == ebe
    assert len(got) == len(exp)
    if got != exp:
        i = next(k for k in range(len(got)) if got[k] != exp[k])
        raise AssertionError(f"first differing byte at {i} of {len(got)}")
    # decode every run back (independent of the compressor)
    base_in = base_out = 0
    for m in range(maps):
        im = index[m * (R + 1):(m + 1) * (R + 1)]
        om = gix[m * (R + 1):(m + 1) * (R + 1)]
        for p in range(R):
            raw = data[base_in + im[p]:base_in + im[p + 1]].tobytes()
            assert O.lz4_unframe(got[base_out + om[p]:base_out + om[p + 1]], len(raw)) == raw
        base_in += int(im[R])
        base_out += int(om[R])
    return got


def partitioned(recs, rs, R, rpm, kind="tera"):
    part = O.terasort_partitioner(R) if kind == "tera" else O.Partitioner(O.MURMUR3_LONG, R, 0, 8)
    data, index, _ = O.write_maps(part, recs, rs, rpm)
    return data, index, index.size // (R + 1)


@pytest.fixture(autouse=True, params=["grid", "queue"])
def deal(request, tuned):
    """Every test runs under both chunk deals of the compressor (tuning lz4_queue: 2 the fixed
    grid-stride deal, 1 the device work queue); the bytes must not depend on the deal."""
    tuned(lz4_queue=1 if request.param == "queue" else 2)
    return request.param


@pytest.mark.parametrize("bs", [1024, 32768, 65536])
def test_terasort_map_outputs(gpu_node, bs):
    data, index, maps = partitioned(O.gen_terasort(31, 0, 40_000), 100, 200, 10_000)
    check(gpu_node, data, index, maps, 200, bs)


def test_zipf_and_small_records(gpu_node):
    data, index, maps = partitioned(O.gen_zipf(32, 0, 30_000), 100, 64, 30_000, kind="hash")
    check(gpu_node, data, index, maps, 64, 32768)
    data, index, maps = partitioned(O.gen_small(33, 0, 100_000), 16, 1000, 50_000, kind="hash")
    check(gpu_node, data, index, maps, 1000, 32768)


def test_unsafe_rows(gpu_node):
    d, o = O.gen_unsafe_rows(34, 60_000, key_mod=1000)
    part = O.Partitioner(O.MURMUR3_LONG, 50, 12, 8)
    out, ix, _, _ = O.varlen_write_maps(part, d, o, 20_000)
    check(gpu_node, out, ix, 3, 50, 32768)


@pytest.mark.parametrize("pattern", ["zeros", "period7", "lowent", "random", "mixed"])
def test_synthetic_runs(gpu_node, pattern):
    """Arbitrary run boundaries (any byte alignment), long matches, raw chunks, empty runs."""
    rng = np.random.default_rng(hash(pattern) % 1000)
    maps, R = 3, 37
    lens = rng.integers(0, 9000, (maps, R))
    lens[:, ::5] = 0                       # empty runs
    lens[0, 1], lens[1, 2], lens[2, 3] = 32768, 32769, 65536 * 2 + 13  # chunk edges
    lens[0, 2] = 12                        # shorter than LZ4's minimum block
    n = int(lens.sum())
    if pattern == "zeros":
        data = np.zeros(n, np.uint8)
    elif pattern == "period7":
        data = np.tile(np.arange(7, dtype=np.uint8), n // 7 + 1)[:n]
    elif pattern == "lowent":
        data = rng.integers(0, 3, n, dtype=np.uint8)
    elif pattern == "random":
        data = rng.integers(0, 256, n, dtype=np.uint8)
    else:
        data = rng.integers(0, 256, n, dtype=np.uint8)
        data[rng.random(n) < 0.7] = 0
    index = np.zeros((maps, R + 1), np.int64)
    index[:, 1:] = np.cumsum(lens, axis=1)
    check(gpu_node, data, index.ravel(), maps, R, 32768)


def _liblz4():
    import ctypes as C
    import ctypes.util
    name = ctypes.util.find_library("lz4") or "liblz4.so.1"
    try:
        L = C.CDLL(name)
    except OSError:
        pytest.skip("system liblz4 not present")
    L.LZ4_compress_default.argtypes = [C.c_char_p, C.c_char_p, C.c_int, C.c_int]
    L.LZ4_decompress_safe.argtypes = [C.c_char_p, C.c_char_p, C.c_int, C.c_int]
    return L


def _workload(kind):
    if kind == "terasort":
        return partitioned(O.gen_terasort(35, 0, 30_000), 100, 16, 15_000) + (16,)
    if kind == "zipf":
        return partitioned(O.gen_zipf(35, 0, 30_000), 100, 8, 15_000, kind="hash") + (8,)
    if kind == "small":
        return partitioned(O.gen_small(36, 0, 200_000), 16, 32, 100_000, kind="hash") + (32,)
    if kind == "rows":
        d, o = O.gen_unsafe_rows(37, 40_000, key_mod=500)
        out, ix, _, _ = O.varlen_write_maps(O.Partitioner(O.MURMUR3_LONG, 10, 12, 8), d, o, 20_000)
        return out, ix, 2, 10
    rng = np.random.default_rng(5)
    n = 300_000
    data = rng.integers(0, 256, n, dtype=np.uint8)
    data[rng.random(n) < (0.9 if kind == "sparse" else 0.5)] = 0
    return data, np.array([0, n // 3, n // 3, n], np.int64), 1, 3


@pytest.mark.parametrize("kind", ["terasort", "zipf", "small", "rows", "sparse", "half"])
def test_gpu_chunks_are_liblz4_compress_default(gpu_node, kind):
    """Every chunk of every GPU stream vs the system liblz4, not via the oracle."""
    import ctypes as C
    L = _liblz4()
    data, index, maps, R = _workload(kind)
    bs = 32768
    got, gix, _ = run_gpu(gpu_node, data, index, maps, R, bs)
    base_in = base_out = 0
    compressed = 0
    for m in range(maps):
        im = index[m * (R + 1):(m + 1) * (R + 1)]
        om = gix[m * (R + 1):(m + 1) * (R + 1)]
        for p in range(R):
            raw = data[base_in + im[p]:base_in + im[p + 1]].tobytes()
            enc = got[base_out + om[p]:base_out + om[p + 1]]
            i = 0
            for a in range(0, len(raw), bs):
                chunk = raw[a:a + bs]
                method = enc[i + 8] & 0xF0
                clen = int.from_bytes(enc[i + 9:i + 13], "little")
                cap = len(chunk) + len(chunk) // 255 + 16
                buf = C.create_string_buffer(cap)
                nw = L.LZ4_compress_default(chunk, buf, len(chunk), cap)
                want = buf.raw[:nw]
                if len(want) < len(chunk):
                    assert method == 0x20 and enc[i + 21:i + 21 + clen] == want, (kind, m, p, a)
                    compressed += 1
                else:
                    assert method == 0x10 and enc[i + 21:i + 21 + clen] == chunk, (kind, m, p, a)
                i += 21 + clen
        base_in += int(im[R])
        base_out += int(om[R])
    assert compressed > 0


def test_empty_and_single(gpu_node):
    index = np.zeros(2 * 5, np.int64)
    check(gpu_node, np.zeros(0, np.uint8), index, 2, 4, 32768)
    data = np.arange(100, dtype=np.uint8)
    check(gpu_node, data, np.array([0, 100], np.int64), 1, 1, 64)
