"""CPU: the compressed-map-output oracle (oracle/lz4.c) pinned against
independent implementations present in this image: XXH32 against the python xxhash module, the
LZ4 block format against the system liblz4 (LZ4_decompress_safe decodes the oracle's blocks;
the oracle's decoder decodes LZ4_compress_default's blocks)."""
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
