"""CPU: the compressed-map-output oracle (oracle/lz4.c) pinned against
independent implementations present in this image: XXH32 against the python xxhash module, and
the LZ4 compressor against the system liblz4 1.9.3 — o_lz4_compress_default must produce
LZ4_compress_default's bytes exactly (the compressor lz4-java's JNI instance runs for Spark), on
every input below, including the shapes the GPU kernel finds hardest (no match at all, matches
from the never-written table entries that read as position 0, overlapping matches, long runs)."""
import ctypes as C
import ctypes.util

import numpy as np
import pytest
import xxhash

from oracle import oracle as O


def _liblz4():
    name = ctypes.util.find_library("lz4") or "liblz4.so.1"
    try:
        L = C.CDLL(name)
    except OSError:
        return None
    L.LZ4_decompress_safe.restype = C.c_int
    L.LZ4_decompress_safe.argtypes = [C.c_char_p, C.c_char_p, C.c_int, C.c_int]
    L.LZ4_compress_default.restype = C.c_int
    L.LZ4_compress_default.argtypes = [C.c_char_p, C.c_char_p, C.c_int, C.c_int]
    return L


LZ4 = _liblz4()
needs_lz4 = pytest.mark.skipif(LZ4 is None, reason="system liblz4 not present")


def samples():
    rng = np.random.default_rng(7)
    yield np.frombuffer(b"abcdabcdabcdabcd" * 3, np.uint8)                # 48 B, overlap
    yield np.frombuffer(b"x" * 12 + b"y", np.uint8)                        # min length
    yield np.frombuffer(bytes(range(200)) + bytes(range(200)), np.uint8)   # one far match
    z = rng.integers(0, 256, 5000, dtype=np.uint8)
    z[:4] = z[4000:4004]                                                   # hit via entry 0
    yield z
    yield np.concatenate([rng.integers(0, 256, 3000, dtype=np.uint8), np.zeros(3000, np.uint8),
                          rng.integers(0, 256, 3000, dtype=np.uint8)])
    yield np.zeros(0, np.uint8)
    yield np.zeros(13, np.uint8)
    yield np.zeros(40_000, np.uint8)
    yield rng.integers(0, 256, 32768, dtype=np.uint8)                     # incompressible
    yield np.tile(np.arange(7, dtype=np.uint8), 5000)                      # period 7
    yield rng.integers(0, 4, 30_000, dtype=np.uint8)                       # low entropy
    yield O.gen_terasort(1, 0, 300)                                        # records
    yield O.gen_unsafe_rows(3, 500, key_mod=17)[0]                         # SQL rows
    w = rng.integers(0, 256, 64, dtype=np.uint8)
    yield np.concatenate([w, rng.integers(0, 256, 70_000, dtype=np.uint8), w])  # far repeat


@pytest.mark.parametrize("n", [0, 1, 3, 4, 15, 16, 17, 33, 1000, 32768])
def test_xxh32_matches_xxhash(n):
    b = np.random.default_rng(n).integers(0, 256, n, dtype=np.uint8)
    assert O.xxh32(b) == xxhash.xxh32(b.tobytes(), seed=0x9747B28C).intdigest()
    assert O.xxh32(b, 0) == xxhash.xxh32(b.tobytes(), seed=0).intdigest()


@needs_lz4
def test_blocks_decode_with_liblz4():
    for s in samples():
        for a in range(0, max(1, s.size), 65536):
            chunk = s[a:a + 65536]
            blk = O.lz4_compress_block(chunk)
            if blk is None:
                assert chunk.size < 13 or len(blk or b"") == 0
                continue
            assert len(blk) < chunk.size
            out = C.create_string_buffer(chunk.size)
            n = LZ4.LZ4_decompress_safe(blk, out, len(blk), chunk.size)
            assert n == chunk.size and out.raw == chunk.tobytes()
            assert O.lz4_decompress_block(blk, chunk.size) == chunk.tobytes()


def _liblz4_compress(s: np.ndarray) -> bytes:
    cap = s.size + s.size // 255 + 16
    out = C.create_string_buffer(cap)
    n = LZ4.LZ4_compress_default(s.tobytes(), out, s.size, cap)
    assert n > 0
    return out.raw[:n]


@needs_lz4
def test_compress_default_is_liblz4_bit_exact():
    for s in samples():
        for a in range(0, max(1, s.size), 65536):
            chunk = s[a:a + 65536]
            assert O.lz4_compress_default(chunk) == _liblz4_compress(chunk), (s.size, a)


@needs_lz4
@pytest.mark.parametrize("kind", ["terasort", "zipf", "small", "rows", "text", "runs"])
def test_compress_default_is_liblz4_bit_exact_on_workloads(kind):
    """32 KiB chunks (Spark's spark.io.compression.lz4.blockSize) of every workload's bytes."""
    rng = np.random.default_rng(11)
    if kind == "terasort":
        data = O.gen_terasort(3, 0, 4000)
    elif kind == "zipf":
        data = O.gen_zipf(3, 0, 4000)
    elif kind == "small":
        data = O.gen_small(3, 0, 30000)
    elif kind == "rows":
        data = O.gen_unsafe_rows(5, 6000, key_mod=101)[0]
    elif kind == "text":
        words = [b"shuffle", b"spark", b"partition", b"record", b"the", b"of", b"GPU", b" ", b"\n"]
        data = np.frombuffer(b"".join(words[i] for i in rng.integers(0, len(words), 60000)), np.uint8)
    else:
        data = np.repeat(rng.integers(0, 256, 4000, dtype=np.uint8), rng.integers(1, 40, 4000))
    for a in range(0, data.size, 32768):
        chunk = data[a:a + 32768]
        assert O.lz4_compress_default(chunk) == _liblz4_compress(chunk), (kind, a)


@needs_lz4
def test_decoder_reads_liblz4_blocks():
    for s in samples():
        if s.size == 0:
            continue
        cap = s.size + s.size // 255 + 16
        out = C.create_string_buffer(cap)
        n = LZ4.LZ4_compress_default(s.tobytes(), out, s.size, cap)
        assert n > 0
        assert O.lz4_decompress_block(out.raw[:n], s.size) == s.tobytes()


def test_compresses_repetitive_data():
    assert len(O.lz4_compress_block(np.zeros(32768, np.uint8))) < 200
    assert O.lz4_compress_block(np.random.default_rng(1).integers(0, 256, 32768,
                                                                  dtype=np.uint8)) is None


@pytest.mark.parametrize("bs", [1024, 32768, 65536])
def test_map_outputs_round_trip(bs):
    """Per-(map, partition) streams: framing, empty runs, index, and decode back to the runs."""
    R, rpm = 13, 700
    recs = O.gen_terasort(5, 0, 2000)
    part = O.terasort_partitioner(R)
    data, index, _ = O.write_maps(part, recs, 100, rpm)
    maps = index.size // (R + 1)
    out, oix, obe = O.lz4_map_outputs(data, index, maps, R, bs)
    assert obe == oix.astype(">i8").tobytes()
    in_base = out_base = 0
    for m in range(maps):
        im, om = index[m * (R + 1):(m + 1) * (R + 1)], oix[m * (R + 1):(m + 1) * (R + 1)]
        for p in range(R):
            raw = data[in_base + im[p]:in_base + im[p + 1]].tobytes()
            enc = out[out_base + om[p]:out_base + om[p + 1]]
            assert (len(enc) == 0) == (len(raw) == 0)
            if raw:
                assert enc[:8] == b"LZ4Block" and enc[-21:-13] == b"LZ4Block"
                assert O.lz4_unframe(enc, len(raw)) == raw
        in_base += int(im[R])
        out_base += int(om[R])
    assert out_base == len(out)
