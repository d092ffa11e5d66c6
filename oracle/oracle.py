"""numpy/ctypes wrapper of oracle/liboracle.so — TEST INFRASTRUCTURE ONLY.

The CPU restatement of the reference path (see oracle.c's header for the file:line map and the
pinning status).  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this module; the product path (sparkucx_amd) never does.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")

RANGE_BYTES, MURMUR3_LONG, MURMUR3_INT, MURMUR3_BYTES, HASH_LONG, HASH_INT = 1, 2, 3, 4, 5, 6


class Part(C.Structure):
    _fields_ = [("kind", C.c_int32), ("num_partitions", C.c_int32), ("key_offset", C.c_int32),
                ("key_len", C.c_int32), ("seed", C.c_int32), ("ascending", C.c_int32),
                ("range_bounds", C.c_void_p)]


class CpuResult(C.Structure):
    _fields_ = [("map_s", C.c_double), ("fetch_s", C.c_double), ("total_s", C.c_double),
                ("bytes_in", C.c_uint64), ("bytes_fetched", C.c_uint64),
                ("checksum", C.c_uint64)]


_lib = None


def build() -> None:
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        P, U64, I32, U32 = C.c_void_p, C.c_uint64, C.c_int32, C.c_uint32
        sig = {
            "o_mix64": (U64, [U64]),
            "o_gen_terasort": (None, [U64, U64, U64, P]),
            "o_gen_small": (None, [U64, U64, U64, P]),
            "o_gen_zipf": (None, [U64, U64, U64, C.c_double, U64, P]),
            "o_zipf_table_size": (C.c_int, [U64]),
            "o_zipf_table": (None, [C.c_double, U64, P, P]),
            "o_murmur3_hash_int": (I32, [I32, I32]),
            "o_murmur3_hash_long": (I32, [C.c_int64, I32]),
            "o_murmur3_hash_unsafe_bytes": (I32, [P, I32, I32]),
            "o_pmod": (I32, [I32, I32]),
            "o_non_negative_mod": (I32, [I32, I32]),
            "o_range_bounds_uniform": (None, [I32, I32, P]),
            "o_get_partition": (I32, [C.POINTER(Part), P]),
            "o_partition_ids": (None, [C.POINTER(Part), P, U64, U32, P]),
            "o_write_map": (None, [C.POINTER(Part), P, U64, U32, P, P, P, P]),
            "o_index_from_lengths": (None, [P, I32, P, P]),
            "o_fetch_blocks": (C.c_int64, [P, P, I32, I32, P, I32, P, P]),
            "o_owner_start": (I32, [I32, I32, I32]),
            "o_cpu_shuffle": (C.c_int, [C.POINTER(Part), P, U64, U32, I32, I32, C.c_char_p,
                                        C.POINTER(CpuResult), P]),
            "o_checksum": (U64, [P, U64]),
            "o_xxh32": (U32, [P, U64, U32]),
            "o_lz4_compress_default": (I32, [P, I32, P]),
            "o_lz4_compress_block": (I32, [P, I32, P]),
            "o_lz4_decompress_block": (I32, [P, I32, P, I32]),
            "o_lz4_stream": (U64, [P, U64, U32, P]),
            "o_lz4_map_outputs": (U64, [P, P, I32, I32, U32, P, P]),
            "o_lz4_unframe": (C.c_int64, [P, U64, P, U64]),
        }
        for k, (r, a) in sig.items():
            f = getattr(L, k)
            f.restype, f.argtypes = r, a
        _lib = L
    return _lib


def _p(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


# ---- generators --------------------------------------------------------------------------
def gen_terasort(seed: int, first: int, n: int) -> np.ndarray:
    out = np.empty(n * 100, np.uint8)
    lib().o_gen_terasort(seed, first, n, _p(out))
    return out


def gen_small(seed: int, first: int, n: int) -> np.ndarray:
    out = np.empty(n * 16, np.uint8)
    lib().o_gen_small(seed, first, n, _p(out))
    return out


def gen_zipf(seed: int, first: int, n: int, s: float = 1.1, zipf_n: int = 1 << 24) -> np.ndarray:
    out = np.empty(n * 100, np.uint8)
    lib().o_gen_zipf(seed, first, n, s, zipf_n, _p(out))
    return out


def zipf_table(s: float, zipf_n: int):
    nb = lib().o_zipf_table_size(zipf_n)
    b = np.empty(nb + 1, np.uint64)
    t = np.empty(nb + 1, np.uint64)
    lib().o_zipf_table(s, zipf_n, _p(b), _p(t))
    return b, t


# ---- hashing ----------------------------------------------------------------------------------
def murmur3_int(v: int, seed: int) -> int:
    return lib().o_murmur3_hash_int(v, seed)


def murmur3_long(v: int, seed: int) -> int:
    return lib().o_murmur3_hash_long(v, seed)


def murmur3_bytes(b: bytes, seed: int) -> int:
    arr = np.frombuffer(bytes(b) or b"\0", np.uint8).copy()
    return lib().o_murmur3_hash_unsafe_bytes(_p(arr), len(b), seed)


def pmod(a: int, n: int) -> int:
    return lib().o_pmod(a, n)


# ---- partitioners / map write ------------------------------------------------------------------
class Partitioner:
    def __init__(self, kind: int, R: int, key_offset: int = 0, key_len: int = 8, seed: int = 42,
                 ascending: bool = True, bounds: bytes | None = None):
        self.kind, self.R, self.key_offset, self.key_len = kind, R, key_offset, key_len
        self.seed, self.ascending = seed, ascending
        self._b = None if bounds is None else np.frombuffer(bytes(bounds) or b"\0", np.uint8).copy()
        self.bounds = bounds
        self.c = Part(kind, R, key_offset, key_len, seed, int(ascending),
                      None if self._b is None else self._b.ctypes.data)

    def ids(self, recs: np.ndarray, rec_size: int) -> np.ndarray:
        n = recs.size // rec_size
        out = np.empty(max(n, 1), np.uint16)
        lib().o_partition_ids(C.byref(self.c), _p(recs), n, rec_size, _p(out))
        return out[:n]


def uniform_range_bounds(R: int, key_len: int = 10) -> bytes:
    out = np.zeros(max(1, (R - 1) * key_len), np.uint8)
    lib().o_range_bounds_uniform(R, key_len, _p(out))
    return out[: (R - 1) * key_len].tobytes()


def terasort_partitioner(R: int) -> Partitioner:
    return Partitioner(RANGE_BYTES, R, 0, 10, bounds=uniform_range_bounds(R, 10))


def write_map(part: Partitioner, recs: np.ndarray, rec_size: int):
    """Returns (data bytes, lengths[R] i64, index[R+1] i64, index_be bytes)."""
    n = recs.size // rec_size
    out = np.empty(max(1, n * rec_size), np.uint8)
    lengths = np.empty(part.R, np.int64)
    index = np.empty(part.R + 1, np.int64)
    index_be = np.empty((part.R + 1) * 8, np.uint8)
    lib().o_write_map(C.byref(part.c), _p(recs), n, rec_size, _p(out), _p(lengths), _p(index),
                      _p(index_be))
    return out[: n * rec_size], lengths, index, index_be.tobytes()


def write_maps(part: Partitioner, recs: np.ndarray, rec_size: int, rpm: int):
    """Concatenated map-major outputs of consecutive maps (what sux_partition_maps produces)."""
    n = recs.size // rec_size
    datas, idxs, bes = [], [], []
    for m0 in range(0, n, rpm):
        d, _, ix, be = write_map(part, recs[m0 * rec_size:min(n, m0 + rpm) * rec_size], rec_size)
        datas.append(d)
        idxs.append(ix)
        bes.append(be)
    if not datas:
        return np.empty(0, np.uint8), np.zeros(part.R + 1, np.int64), b""
    return np.concatenate(datas), np.concatenate(idxs), b"".join(bes)


def owner_start(h: int, R: int, G: int) -> int:
    return (h * R) // G


def plan_ownership(world: int, partition_bytes) -> list[int]:
    """Oracle of sux_plan_ownership, by dynamic programming (not the library's binary search):
    the contiguous split of R partitions into `world` non-empty ranges minimising the largest
    range's bytes; of the optimal splits, the one whose owners end as early as possible (the
    library's greedy fill).  Returns world + 1 bounds.  O(world R^2): test sizes only."""
    b = [int(x) for x in partition_bytes]
    R = len(b)
    pre = [0]
    for x in b:
        pre.append(pre[-1] + x)
    INF = float("inf")
    # best[h][p]: smallest possible largest range when owners h.. cover partitions p..R-1
    best = [[INF] * (R + 1) for _ in range(world + 1)]
    best[world][R] = 0
    for h in range(world - 1, -1, -1):
        for p in range(R - (world - h) + 1):
            for q in range(p + 1, R - (world - h - 1) + 1):
                v = max(pre[q] - pre[p], best[h + 1][q])
                if v < best[h][p]:
                    best[h][p] = v
    cap = best[0][0]
    # the greedy fill at the optimal cap: each owner as long as the cap allows, leaving one
    # partition per later owner
    bounds, p = [0], 0
    for h in range(world - 1):
        s = b[p]
        p += 1
        while p < R - (world - 1 - h) and s + b[p] <= cap:
            s += b[p]
            p += 1
        bounds.append(p)
    bounds.append(R)
    return bounds


def peer_major(part: Partitioner, recs: np.ndarray, rec_size: int, rpm: int, world: int,
               own=None):
    """Oracle of sux_partition_maps_peer_major: [peer h][map m][partitions owned by h]; `own`:
    the ownership bounds (world + 1; None = the equal split)."""
    n = recs.size // rec_size
    maps = []
    for m0 in range(0, n, rpm):
        d, _, ix, _ = write_map(part, recs[m0 * rec_size:min(n, m0 + rpm) * rec_size], rec_size)
        maps.append((d, ix))
    chunks, peer_bytes = [], []
    for h in range(world):
        lo, hi = ((owner_start(h, part.R, world), owner_start(h + 1, part.R, world))
                  if own is None else (int(own[h]), int(own[h + 1])))
        b = 0
        for d, ix in maps:
            chunks.append(d[ix[lo]:ix[hi]])
            b += int(ix[hi] - ix[lo])
        peer_bytes.append(b)
    data = np.concatenate(chunks) if chunks else np.empty(0, np.uint8)
    index = np.concatenate([ix for _, ix in maps]) if maps else np.zeros(0, np.int64)
    return data, index, np.array(peer_bytes, np.int64)


def fetch_blocks(map_data: list[np.ndarray], map_index_be: list[bytes], R: int, blocks):
    """UcxShuffleClient.fetchBlocks restated: returns (contiguous bytes, sizes)."""
    nm = len(map_data)
    datas = [np.ascontiguousarray(d) if d.size else np.zeros(1, np.uint8) for d in map_data]
    idx = [np.frombuffer(b, np.uint8).copy() for b in map_index_be]
    dp = (C.c_void_p * max(1, nm))(*[d.ctypes.data for d in datas])
    ip = (C.c_void_p * max(1, nm))(*[i.ctypes.data for i in idx])
    flat = []
    for b in blocks:
        flat += [b[0], b[1], b[2] if len(b) > 2 else b[1] + 1]
    bl = np.array(flat or [0], np.int32)
    sizes = np.zeros(max(1, len(blocks)), np.int64)
    total = lib().o_fetch_blocks(dp, ip, nm, R, _p(bl), len(blocks), _p(sizes), None)
    if total < 0:
        raise ValueError("invalid block")
    dst = np.empty(max(1, total), np.uint8)
    lib().o_fetch_blocks(dp, ip, nm, R, _p(bl), len(blocks), _p(sizes), _p(dst))
    return dst[:total].tobytes(), sizes[:len(blocks)].tolist()


def checksum(a: np.ndarray) -> int:
    return int(lib().o_checksum(_p(a), a.size))


def cpu_shuffle(part: Partitioner, recs: np.ndarray, rec_size: int, num_maps: int, threads: int,
                directory: str = "/dev/shm", index_out: np.ndarray | None = None) -> CpuResult:
    """CPU baseline shuffle; index_out (int64[num_maps * (R+1)], optional) receives the
    committed index files (native order) for a parity check."""
    res = CpuResult()
    rc = lib().o_cpu_shuffle(C.byref(part.c), _p(recs), recs.size // rec_size, rec_size, num_maps,
                             threads, directory.encode(), C.byref(res),
                             None if index_out is None else _p(index_out))
    if rc != 0:
        raise RuntimeError("cpu shuffle failed")
    return res


SORT_BYTES, SORT_LONG, SORT_INT = 1, 2, 3


def sort_records(recs: np.ndarray, rec_size: int, kind: int, key_offset: int,
                 key_len: int) -> np.ndarray:
    """Reduce-side sort: the reader's ExternalSorter step when the
    dependency has a key ordering (compat/spark_3_0/UcxShuffleReader.scala:138-154).  Stable in
    input order for equal keys — the canonical answer for a map-ordered concatenation (Spark's
    own order for equal keys depends on the fetch order, quirk Q4).  Keys: unsigned byte
    lexicographic (TeraSort's comparator), or signed little-endian int64 / int32 (Spark's
    LongType / IntegerType orderings)."""
    rows = np.ascontiguousarray(recs).reshape(-1, rec_size)
    n = rows.shape[0]
    if n == 0:
        return rows.reshape(-1).copy()
    key = np.ascontiguousarray(rows[:, key_offset:key_offset + key_len])
    if kind == SORT_BYTES:
        order = np.argsort(key.view(np.dtype((np.void, key_len))).ravel(), kind="stable")
    elif kind == SORT_LONG:
        order = np.argsort(key.view("<i8").ravel(), kind="stable")
    elif kind == SORT_INT:
        order = np.argsort(key.view("<i4").ravel(), kind="stable")
    else:
        raise ValueError(f"unknown sort key kind {kind}")
    return rows[order].reshape(-1)


def sort_segments(recs: np.ndarray, rec_size: int, kind: int, key_offset: int, key_len: int,
                  seg_offsets) -> np.ndarray:
    """sort_records applied to every run [seg_offsets[k], seg_offsets[k+1]) of records."""
    rows = np.ascontiguousarray(recs).reshape(-1, rec_size)
    parts = [sort_records(rows[a:b].reshape(-1), rec_size, kind, key_offset, key_len)
             for a, b in zip(seg_offsets[:-1], seg_offsets[1:])]
    return np.concatenate(parts) if parts else rows.reshape(-1).copy()


# ---- variable-length rows -----------------------------------------------
def gen_unsafe_rows(seed: int, n: int, max_payload_words: int = 12,
                    key_mod: int | None = None) -> tuple[np.ndarray, np.ndarray]:
    """n rows in Spark SQL's UnsafeRowSerializer framing [ext: spark-sql UnsafeRowSerializer
    writeValue = writeInt(row.getSizeInBytes) + row.writeToStream]: a 4-byte big-endian length L,
    then an UnsafeRow of L bytes = 8-byte null bitset (0) | int64 key (little-endian, the row's
    first fixed-width field) | k payload words, k uniform in [0, max_payload_words].  The key sits
    at byte 12 of each framed row.  Returns (data u8, offsets i64[n + 1])."""
    rng = np.random.default_rng(seed)
    k = rng.integers(0, max_payload_words + 1, n)
    L = 8 * (2 + k)
    offs = np.zeros(n + 1, np.int64)
    np.cumsum(4 + L, out=offs[1:])
    data = rng.integers(0, 256, int(offs[-1]), dtype=np.uint8)
    keys = rng.integers(-(1 << 63), (1 << 63) - 1, n, dtype=np.int64, endpoint=True)
    if key_mod:
        keys %= key_mod
    starts = offs[:-1]
    data[starts[:, None] + np.arange(4)] = L.astype(">u4").view(np.uint8).reshape(n, 4)
    data[starts[:, None] + 4 + np.arange(8)] = 0
    data[starts[:, None] + 12 + np.arange(8)] = keys.astype("<i8").view(np.uint8).reshape(n, 8)
    return data, offs


def varlen_ids(part: Partitioner, data: np.ndarray, offs: np.ndarray) -> np.ndarray:
    """P1 on each row's key: the key bytes [key_offset, +key_len) of every row gathered into a
    fixed-width array, then the same partitioner (oracle.c o_partition_ids) at key_offset 0."""
    n = offs.size - 1
    if n == 0:
        return np.empty(0, np.uint16)
    kl = part.key_len
    keys = np.ascontiguousarray(data[(offs[:-1] - offs[0] + part.key_offset)[:, None]
                                     + np.arange(kl)])
    p0 = Partitioner(part.kind, part.R, 0, kl, part.seed, part.ascending, part.bounds)
    return p0.ids(keys.reshape(-1), kl)


def varlen_write_maps(part: Partitioner | None, data: np.ndarray, offs: np.ndarray, rpm: int,
                      R: int | None = None, pids: np.ndarray | None = None):
    """P2+P3 for variable-length rows: per map (runs of rpm rows), a stable regroup of the rows by
    pid — the serialized rows of partition 0, then 1, ..., R-1, each in input order (what Spark's
    UnsafeShuffleWriter emits for UnsafeRowSerializer output with compression off) — written at
    the map's own byte range, and its (R+1) cumulative BYTE offsets (the index file,
    IndexShuffleBlockResolver.writeIndexFileAndCommit via compat/spark_3_0/
    UcxShuffleBlockResolver.scala:35).  Returns (out, index i64[maps*(R+1)], index_be, pids)."""
    n = offs.size - 1
    R = part.R if R is None else R
    if pids is None:
        pids = varlen_ids(part, data, offs)
    pids = pids.astype(np.int64)
    base = offs - offs[0]
    lens = np.diff(offs)
    out = np.empty(int(base[-1]), np.uint8)
    idx, be = [], []
    for m0 in range(0, n, rpm):
        m1 = min(n, m0 + rpm)
        order = m0 + np.argsort(pids[m0:m1], kind="stable")
        ln = lens[order]
        src = np.repeat(base[order], ln) + (np.arange(int(ln.sum())) -
                                            np.repeat(np.cumsum(ln) - ln, ln))
        out[base[m0]:base[m1]] = data[src]
        sizes = np.bincount(pids[m0:m1], weights=lens[m0:m1], minlength=R).astype(np.int64)
        ix = np.zeros(R + 1, np.int64)
        np.cumsum(sizes, out=ix[1:])
        idx.append(ix)
        be.append(ix.astype(">i8").tobytes())
    if not idx:
        return out, np.zeros(0, np.int64), b"", pids.astype(np.uint16)
    return out, np.concatenate(idx), b"".join(be), pids.astype(np.uint16)


# ---- compressed map outputs (oracle/lz4.c) -------------------------------
def xxh32(b: np.ndarray, seed: int = 0x9747B28C) -> int:
    b = np.ascontiguousarray(b, np.uint8)
    return int(lib().o_xxh32(_p(b), b.size, seed))


def lz4_compress_default(b: np.ndarray) -> bytes:
    """liblz4 1.9.3 LZ4_compress_default restated (oracle/lz4.c): the LZ4 block, always."""
    b = np.ascontiguousarray(b, np.uint8)
    out = np.empty(b.size + b.size // 255 + 16, np.uint8)
    n = lib().o_lz4_compress_default(_p(b) if b.size else None, b.size, _p(out))
    return out[:n].tobytes()


def lz4_compress_block(b: np.ndarray) -> bytes | None:
    """One LZ4BlockOutputStream chunk's payload: the LZ4 block, or None = stored raw (the block
    would not be shorter, lz4-java's rule)."""
    b = np.ascontiguousarray(b, np.uint8)
    out = np.empty(max(16, b.size), np.uint8)
    n = lib().o_lz4_compress_block(_p(b) if b.size else None, b.size, _p(out))
    return None if n == 0 else out[:n].tobytes()


def lz4_decompress_block(src: bytes, size: int) -> bytes:
    s = np.frombuffer(src, np.uint8).copy() if src else np.zeros(1, np.uint8)
    out = np.empty(max(1, size), np.uint8)
    n = lib().o_lz4_decompress_block(_p(s), len(src), _p(out), size)
    if n != size:
        raise ValueError(f"malformed LZ4 block ({n})")
    return out[:size].tobytes()


def lz4_map_outputs(data: np.ndarray, index: np.ndarray, maps: int, R: int, block_size: int):
    """Compressed map outputs: (out bytes, index i64[maps*(R+1)], index_be bytes)."""
    data = np.ascontiguousarray(data, np.uint8)
    index = np.ascontiguousarray(index, np.int64)
    runs = maps * R
    cap = data.size + (data.size // block_size + runs + 1) * 21 + runs * 21 + 64
    out = np.empty(cap, np.uint8)
    oix = np.empty(maps * (R + 1), np.int64)
    n = lib().o_lz4_map_outputs(_p(data) if data.size else None, _p(index), maps, R, block_size,
                                _p(out), _p(oix))
    return out[:n].tobytes(), oix, oix.astype(">i8").tobytes()


def lz4_unframe(stream: bytes, cap: int) -> bytes:
    """Decode concatenated LZ4BlockOutputStream streams (checks magic, lengths, checksums)."""
    s = np.frombuffer(stream, np.uint8).copy() if stream else np.zeros(1, np.uint8)
    out = np.empty(max(1, cap), np.uint8)
    n = lib().o_lz4_unframe(_p(s), len(stream), _p(out), cap)
    if n < 0:
        raise ValueError("malformed LZ4Block stream")
    return out[:n].tobytes()
