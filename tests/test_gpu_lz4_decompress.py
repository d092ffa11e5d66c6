"""GPU parity: the reader's side of spark.shuffle.compress=true — sux_decompress_blocks (lz4-java's
LZ4BlockInputStream over every fetched block) against the bytes the streams were made from.

The compressed inputs come from the CPU oracle (oracle/lz4.c, whose compressor is pinned to the
system liblz4's LZ4_compress_default) and from the system liblz4 itself (its fast and HC
compressors, framed here), so the decoder is checked against streams the GPU compressor never
touched; the GPU compressor's own outputs round-trip too.  Every decoded block is compared byte
for byte with its source run; corrupted, truncated and oversized inputs must set the node's error
word and never write outside the output.
"""
import ctypes as C
import ctypes.util

import numpy as np
import pytest
import torch

from oracle import oracle as O
from sparkucx_amd import native as N

pytestmark = pytest.mark.gpu


def to_dev(a) -> torch.Tensor:
    a = np.frombuffer(a, np.uint8) if isinstance(a, (bytes, bytearray)) else a
    a = np.ascontiguousarray(a)
    return torch.from_numpy(a.copy() if a.size else np.zeros(16, a.dtype)).cuda()


def blocks_of(oix: np.ndarray, maps: int, R: int) -> np.ndarray:
    """Start offsets of every (map, partition) compressed run, maps consecutive (+ the end)."""
    offs, base = [], 0
    for m in range(maps):
        om = oix[m * (R + 1):(m + 1) * (R + 1)]
        offs.extend(base + int(om[p]) for p in range(R))
        base += int(om[R])
    offs.append(base)
    return np.array(offs, np.int64)


def runs_of(data: np.ndarray, index: np.ndarray, maps: int, R: int) -> list:
    out, base = [], 0
    for m in range(maps):
        im = index[m * (R + 1):(m + 1) * (R + 1)]
        out.extend(data[base + im[p]:base + im[p + 1]].tobytes() for p in range(R))
        base += int(im[R])
    return out


def decode(node, stream: bytes, offs: np.ndarray, max_bs=32768, out=None):
    d = to_dev(stream)
    out, oo = node.decompress_blocks(d, to_dev(offs), max_bs, out=out, in_bytes=len(stream))
    torch.cuda.synchronize()
    return out, oo.cpu().numpy()


def check_roundtrip(node, data, index, maps, R, bs, stream=None, oix=None):
    if stream is None:
        stream, oix, _ = O.lz4_map_outputs(data, index, maps, R, bs)
    offs = blocks_of(oix, maps, R)
    out, oo = decode(node, stream, offs, max(bs, 64))
    node.check()
    want = runs_of(data, index, maps, R)
    assert oo[0] == 0 and oo[-1] == sum(len(w) for w in want)
    got = out[:int(oo[-1])].cpu().numpy().tobytes()
    for k, w in enumerate(want):
        assert got[oo[k]:oo[k + 1]] == w, (k, len(w))


def partitioned(recs, rs, R, rpm, kind="tera"):
    part = O.terasort_partitioner(R) if kind == "tera" else O.Partitioner(O.MURMUR3_LONG, R, 0, 8)
    data, index, _ = O.write_maps(part, recs, rs, rpm)
    return data, index, index.size // (R + 1)


@pytest.mark.parametrize("bs", [1024, 32768, 65536])
def test_terasort_streams_from_the_oracle(gpu_node, bs):
    data, index, maps = partitioned(O.gen_terasort(41, 0, 40_000), 100, 200, 10_000)
    check_roundtrip(gpu_node, data, index, maps, 200, bs)


@pytest.mark.parametrize("pattern", ["zeros", "period7", "lowent", "random", "mixed"])
def test_synthetic_runs(gpu_node, pattern):
    """Any byte alignment of the blocks in the input and output, long matches overlapping
    themselves (period 1 and 7), long literal runs, raw chunks, empty blocks, chunk edges."""
    rng = np.random.default_rng(abs(hash(pattern)) % 1000)
    maps, R = 3, 37
    lens = rng.integers(0, 9000, (maps, R))
    lens[:, ::5] = 0
    lens[0, 1], lens[1, 2], lens[2, 3] = 32768, 32769, 65536 * 2 + 13
    lens[0, 2] = 12
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
    check_roundtrip(gpu_node, data, index.ravel(), maps, R, 32768)


def test_the_gpu_compressors_streams_round_trip(gpu_node):
    data, index, maps = partitioned(O.gen_zipf(42, 0, 30_000), 100, 64, 10_000, kind="hash")
    d = to_dev(data)
    out, oix, _, nbytes = gpu_node.compress_map_outputs(d, to_dev(index), maps, 64, 32768)
    torch.cuda.synchronize()
    stream = out[:int(nbytes.item())].cpu().numpy().tobytes()
    check_roundtrip(gpu_node, data, index, maps, 64, 32768, stream, oix.cpu().numpy())


def _liblz4():
    name = ctypes.util.find_library("lz4") or "liblz4.so.1"
    try:
        L = C.CDLL(name)
    except OSError:
        pytest.skip("system liblz4 not present")
    for f in ("LZ4_compress_default", "LZ4_compress_HC"):
        getattr(L, f).restype = C.c_int
    L.LZ4_compress_default.argtypes = [C.c_char_p, C.c_char_p, C.c_int, C.c_int]
    L.LZ4_compress_HC.argtypes = [C.c_char_p, C.c_char_p, C.c_int, C.c_int, C.c_int]
    return L


def frame(L, raw: bytes, bs: int, hc: int) -> bytes:
    """One LZ4BlockOutputStream stream of `raw` with liblz4's fast (hc = 0) or HC compressor."""
    level = max(0, (bs - 1).bit_length() - 10)
    out = bytearray()
    for a in range(0, len(raw), bs):
        chunk = raw[a:a + bs]
        cap = len(chunk) + len(chunk) // 255 + 16
        buf = C.create_string_buffer(cap)
        n = (L.LZ4_compress_HC(chunk, buf, len(chunk), cap, hc) if hc else
             L.LZ4_compress_default(chunk, buf, len(chunk), cap))
        comp = n > 0 and n < len(chunk)
        payload = buf.raw[:n] if comp else chunk
        out += b"LZ4Block" + bytes([(0x20 if comp else 0x10) | level])
        out += len(payload).to_bytes(4, "little") + len(chunk).to_bytes(4, "little")
        out += (O.xxh32(np.frombuffer(chunk, np.uint8)) & 0x0FFFFFFF).to_bytes(4, "little")
        out += payload
    out += b"LZ4Block" + bytes([0x10 | level]) + bytes(12)
    return bytes(out)


@pytest.mark.parametrize("hc", [0, 9])
def test_streams_from_the_system_liblz4(gpu_node, hc):
    """liblz4's fast and HC (level 9: longer matches, other offsets) blocks, framed as lz4-java
    frames them, several streams concatenated in one block (a ShuffleBlockBatchId's range)."""
    L = _liblz4()
    rng = np.random.default_rng(7 + hc)
    raws, streams = [], []
    for k in range(24):
        n = int(rng.integers(0, 70_000))
        kind = k % 4
        if kind == 0:
            raw = O.gen_terasort(50 + k, 0, n // 100 + 1).tobytes()[:n]
        elif kind == 1:
            raw = np.repeat(rng.integers(0, 256, n // 13 + 1, dtype=np.uint8), 13)[:n].tobytes()
        elif kind == 2:
            raw = rng.integers(0, 4, n, dtype=np.uint8).tobytes()
        else:
            raw = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        raws.append(raw)
        streams.append(frame(L, raw, 32768, hc) if raw else b"")
    # blocks: singles, then pairs of streams back to back (concatenation)
    groups = [[k] for k in range(12)] + [[k, k + 1] for k in range(12, 24, 2)]
    blob, offs, want = b"", [0], []
    for g in groups:
        blob += b"".join(streams[k] for k in g)
        offs.append(len(blob))
        want.append(b"".join(raws[k] for k in g))
    out, oo = decode(gpu_node, blob, np.array(offs, np.int64))
    gpu_node.check()
    got = out.cpu().numpy().tobytes()
    for k, w in enumerate(want):
        assert got[oo[k]:oo[k + 1]] == w, k
        assert O.lz4_unframe(blob[offs[k]:offs[k + 1]], len(w) + 1) == w  # the oracle agrees


def _one_stream(raw: bytes, bs=32768):
    stream, oix, _ = O.lz4_map_outputs(np.frombuffer(raw, np.uint8),
                                       np.array([0, len(raw)], np.int64), 1, 1, bs)
    return bytearray(stream)


def _expect_error(node, stream: bytes, what: str, out_cap=None):
    offs = np.array([0, len(stream)], np.int64)
    out = None if out_cap is None else torch.zeros(out_cap + 64, dtype=torch.uint8, device="cuda")
    guard = None
    if out is not None:
        view = out[:out_cap]
        guard = out[out_cap:].clone()
    else:
        view = torch.zeros(1 << 20, dtype=torch.uint8, device="cuda")
    d = to_dev(bytes(stream))
    node.decompress_blocks(d, to_dev(offs), 32768, out=view, in_bytes=len(stream))
    torch.cuda.synchronize()
    with pytest.raises(N.SuxError) as e:
        node.check()
    assert e.value.code == N.SUX_EHIP and what in str(e.value), str(e.value)
    if guard is not None:  # nothing written past the capacity
        assert torch.equal(out[out_cap:], guard)


def test_corrupted_truncated_and_oversized_blocks_set_the_error_word(gpu_node):
    raw = O.gen_terasort(60, 0, 2000).tobytes()  # 200 KB: 7 chunks, LZ4 and raw
    good = _one_stream(raw)
    bad = bytearray(good)
    bad[21 + 100] ^= 0x40                    # a payload byte of the first chunk
    _expect_error(gpu_node, bad, "")         # a wrong sequence or a wrong checksum
    bad = bytearray(good)
    bad[0] = ord("X")                        # magic
    _expect_error(gpu_node, bad, "corrupted")
    _expect_error(gpu_node, good[:len(good) - 30], "corrupted")  # truncated mid-chunk
    bad = bytearray(good)
    bad[13:17] = (40000).to_bytes(4, "little")  # original length > the 32 KiB block size
    _expect_error(gpu_node, bad, "corrupted")
    _expect_error(gpu_node, good, "capacity", out_cap=len(raw) - 1)
    # the error word was cleared by each check: a good stream decodes cleanly afterwards
    out, oo = decode(gpu_node, bytes(good), np.array([0, len(good)], np.int64))
    gpu_node.check()
    assert out[:len(raw)].cpu().numpy().tobytes() == raw


def test_empty_and_no_blocks(gpu_node):
    out, oo = decode(gpu_node, b"", np.array([0], np.int64))
    gpu_node.check()
    assert list(oo) == [0]
    end_only = b"LZ4Block" + bytes([0x10 | 5]) + bytes(12)
    out, oo = decode(gpu_node, end_only * 2, np.array([0, 0, 21, 42], np.int64))
    gpu_node.check()
    assert list(oo) == [0, 0, 0, 0]


def test_sizes_only_call(gpu_node):
    raw = bytes(range(256)) * 300
    s = bytes(_one_stream(raw, 1024))
    d = to_dev(s)
    offs = to_dev(np.array([0, len(s)], np.int64))
    oo = torch.empty(2, dtype=torch.int64, device="cuda")
    ws = torch.empty(gpu_node.decompress_workspace_size(len(s), 1, 1024), dtype=torch.uint8,
                     device="cuda")
    lib = N.load()
    N.check(lib.sux_decompress_blocks(gpu_node.h, d.data_ptr(), len(s), offs.data_ptr(), 1, 1024,
                                      None, 0, oo.data_ptr(), ws.data_ptr(), ws.numel(), None))
    torch.cuda.synchronize()
    gpu_node.check()
    assert oo.cpu().tolist() == [0, len(raw)]


def test_fuzzed_blocks_never_write_outside_the_output(gpu_node):
    """300 corrupted variants of a multi-chunk stream (a flipped byte anywhere — header, lengths,
    tokens, offsets, literals — or a cut at any length) decoded as 300 blocks of one call: the
    call completes, nothing past the output capacity changes, and the decoder decodes a good
    stream afterwards.  (Which variants are rejected is the error word's business; a variant that
    still parses decodes to bytes of its own.)"""
    rng = np.random.default_rng(11)
    raw = np.concatenate([O.gen_terasort(70, 0, 600).ravel(),
                          np.tile(np.arange(9, dtype=np.uint8), 4000)]).tobytes()
    good = bytes(_one_stream(raw, 4096))
    variants = []
    for k in range(300):
        v = bytearray(good)
        if k % 5 == 4:
            v = v[:int(rng.integers(0, len(v)))]
        else:
            pos = int(rng.integers(0, len(v)))
            v[pos] ^= int(rng.integers(1, 256))
        variants.append(bytes(v))
    blob = b"".join(variants)
    offs = np.concatenate([[0], np.cumsum([len(v) for v in variants])]).astype(np.int64)
    cap = 300 * len(raw) + 4096
    out = torch.zeros(cap + 4096, dtype=torch.uint8, device="cuda")
    guard = out[cap:].clone()
    gpu_node.decompress_blocks(to_dev(blob), to_dev(offs), 4096, out=out[:cap],
                               in_bytes=len(blob))
    torch.cuda.synchronize()
    try:
        gpu_node.check()
    except N.SuxError as e:
        assert e.code == N.SUX_EHIP
    assert torch.equal(out[cap:], guard)
    got, oo = decode(gpu_node, good, np.array([0, len(good)], np.int64), 4096)
    gpu_node.check()
    assert got[:len(raw)].cpu().numpy().tobytes() == raw


def test_overlapping_block_ranges_cannot_overrun_the_chunk_table(gpu_node):
    """non-monotone in_offsets let good blocks overlap, so they can hold more chunk
    headers than the input — the chunk table (sized for the input) would overflow if the count
    wrapped or went unchecked.  The walk counts chunks in 64 bits: 400 blocks that all re-read the
    same 64-chunk stream (offsets 0, L, 0, L, ...: every other block is a reversed, corrupted range)
    exceed the table, the call reports a corrupted input and nothing is decoded or written."""
    raw = bytes(range(256)) * 64  # 16 KiB -> 64 raw-ish 256-byte chunks
    s = bytes(_one_stream(raw, 256))
    L = len(s)
    offs = np.array([0 if k % 2 == 0 else L for k in range(801)], np.int64)
    out = torch.zeros(400 * len(raw) + 4096, dtype=torch.uint8, device="cuda")
    gpu_node.decompress_blocks(to_dev(s), to_dev(offs), 256, out=out[:400 * len(raw)], in_bytes=L)
    torch.cuda.synchronize()
    with pytest.raises(N.SuxError) as e:
        gpu_node.check()
    assert e.value.code == N.SUX_EHIP and "corrupted" in str(e.value), str(e.value)
    assert int(out.count_nonzero()) == 0  # nothing decoded anywhere
    got, _ = decode(gpu_node, s, np.array([0, L], np.int64), 256)  # the decoder is fine afterwards
    gpu_node.check()
    assert got[:len(raw)].cpu().numpy().tobytes() == raw
