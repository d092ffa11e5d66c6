"""CPU: the oracle against Spark's known answers, its own invariants and the golden fixtures."""
import hashlib
import json
import os

import numpy as np
import pytest

from oracle import oracle as O

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def load(name):
    with open(os.path.join(GOLD, name)) as f:
        return json.load(f)


def sha(b):
    return hashlib.sha256(bytes(b)).hexdigest()


# ---- Murmur3: pinned to Spark's Murmur3_x86_32Suite -----------------------------------------
def test_murmur3_known_answers():
    kat = load("murmur3_kat.json")
    for v, want in kat["hashInt_seed0"].items():
        assert O.murmur3_int(int(v), 0) == want
    for v, want in kat["hashLong_seed0"].items():
        assert O.murmur3_long(int(v), 0) == want
    assert O.murmur3_int(0, 42) == kat["hashInt_seed42"]["0"]
    assert O.murmur3_long(0, 42) == kat["hashLong_seed42"]["0"]


def test_hash_unsafe_bytes_word_aligned_equals_hash_int():
    # for a 4-byte input the legacy bytes hash is one word round + fmix(len=4) == hashInt
    for v in (0, 1, -1, 123456789, -2**31):
        b = int(v & 0xFFFFFFFF).to_bytes(4, "little")
        assert O.murmur3_bytes(b, 42) == O.murmur3_int(v, 42)


def test_hash_unsafe_bytes_tail_is_sign_extended():
    # tail bytes are mixed one at a time, sign-extended: 0x80 differs from 0x00000080 word
    a = O.murmur3_bytes(b"\x80", 42)
    b = O.murmur3_bytes(b"\x7f", 42)
    assert a != b
    assert O.murmur3_bytes(b"abcde", 42) != O.murmur3_bytes(b"abcd", 42)


def test_pmod_matches_java():
    for a in (-7, -1, 0, 1, 7, -2**31, 2**31 - 1):
        for n in (1, 3, 200, 10000):
            r = a % n  # python floor-mod == Java Pmod result for positive n
            assert O.pmod(a, n) == r


# ---- partitioners ---------------------------------------------------------------------------
def test_range_partition_counts_bounds_below_key():
    R = 5
    bounds = O.uniform_range_bounds(R, 10)
    part = O.Partitioner(O.RANGE_BYTES, R, 0, 10, bounds=bounds)
    recs = np.zeros((R - 1) * 3 * 100, np.uint8).reshape(-1, 100)
    bs = [bounds[i * 10:(i + 1) * 10] for i in range(R - 1)]
    rows = []
    for i, b in enumerate(bs):
        key = np.frombuffer(b, np.uint8)
        below = key.copy()
        below[9] = 0  # bounds end with zero bytes; decrement the 8-byte prefix instead
        v = int.from_bytes(b[:8], "big") - 1
        below[:8] = np.frombuffer(v.to_bytes(8, "big"), np.uint8)
        above = key.copy()
        above[9] = 1
        rows += [(below, i), (key, i), (above, i + 1)]  # equal to a bound -> lower partition
    recs = np.zeros(len(rows) * 100, np.uint8)
    for j, (k, _) in enumerate(rows):
        recs[j * 100:j * 100 + 10] = k
    assert part.ids(recs, 100).tolist() == [p for _, p in rows]


def test_range_descending_flips():
    R = 9
    recs = O.gen_terasort(3, 0, 2000)
    a = O.Partitioner(O.RANGE_BYTES, R, 0, 10, bounds=O.uniform_range_bounds(R, 10))
    d = O.Partitioner(O.RANGE_BYTES, R, 0, 10, ascending=False, bounds=O.uniform_range_bounds(R, 10))
    assert (d.ids(recs, 100) == (R - 1) - a.ids(recs, 100)).all()


def test_hash_long_partitioner_matches_java_long_hashcode():
    recs = O.gen_small(9, 0, 1000)
    part = O.Partitioner(O.HASH_LONG, 37, 0, 8)
    keys = recs.reshape(-1, 16)[:, :8].copy().view(np.int64).ravel()
    want = []
    for k in keys.tolist():
        u = k & 0xFFFFFFFFFFFFFFFF
        h = (u ^ (u >> 32)) & 0xFFFFFFFF
        h = h - (1 << 32) if h >= 1 << 31 else h
        r = int(np.fmod(h, 37))
        want.append(r + 37 if r < 0 else r)
    assert part.ids(recs, 16).tolist() == want


def test_murmur3_long_partitioner_is_pmod_of_hash():
    recs = O.gen_zipf(5, 0, 500)
    part = O.Partitioner(O.MURMUR3_LONG, 200, 0, 8, seed=42)
    keys = recs.reshape(-1, 100)[:, :8].copy().view(np.int64).ravel().tolist()
    assert part.ids(recs, 100).tolist() == [O.murmur3_long(k, 42) % 200 for k in keys]


# ---- sort-shuffle write -----------------------------------------------------------------------
def test_write_map_is_stable_group_by_pid():
    recs = O.gen_terasort(2, 0, 3000)
    part = O.terasort_partitioner(13)
    data, lengths, index, index_be = O.write_map(part, recs, 100)
    pids = part.ids(recs, 100)
    order = np.argsort(pids, kind="stable")
    assert bytes(data) == recs.reshape(-1, 100)[order].tobytes()
    assert index[0] == 0 and index[-1] == recs.size
    assert (np.diff(index) == lengths).all()
    assert index_be == b"".join(int(v).to_bytes(8, "big") for v in index)


def test_empty_and_single_partition():
    part = O.Partitioner(O.MURMUR3_LONG, 1, 0, 8)
    recs = O.gen_small(1, 0, 100)
    data, lengths, index, _ = O.write_map(part, recs, 16)
    assert bytes(data) == recs.tobytes() and index.tolist() == [0, 1600]
    data, lengths, index, be = O.write_map(O.terasort_partitioner(4), np.empty(0, np.uint8), 100)
    assert index.tolist() == [0] * 5 and be == bytes(40)


# ---- golden fixtures ----------------------------------------------------------------------------
GEN = {"gen_terasort": O.gen_terasort, "gen_zipf": O.gen_zipf, "gen_small": O.gen_small}


@pytest.mark.parametrize("name", ["terasort_4096_R7.json", "terasort_4096_R200.json",
                                  "zipf_4096_R200.json", "small_65536_R10000.json",
                                  "terasort_10000_rpm3000_R200.json"])
def test_golden_map_fixtures(name):
    g = load(name)
    recs = GEN[g["generator"]](*g["gen_args"])
    assert sha(recs) == g["input_sha256"]
    kw = dict(g["partitioner"])
    if "bounds" in kw:
        kw["bounds"] = bytes.fromhex(kw["bounds"])
    part = O.Partitioner(**kw)
    pids = part.ids(recs, g["record_size"])
    assert sha(pids.astype("<u2").tobytes()) == g["pids_sha256"]
    assert np.bincount(pids, minlength=part.R).tolist() == g["pid_counts"]
    data, index, index_be = O.write_maps(part, recs, g["record_size"], g["records_per_map"])
    assert sha(data) == g["data_sha256"]
    assert sha(index_be) == g["index_be_sha256"]
    if "index_be_hex" in g:
        assert index_be.hex() == g["index_be_hex"]


def test_golden_exchange_fixture():
    ex = load("exchange_3maps_G2.json")
    part = O.terasort_partitioner(ex["R"])
    rpm = ex["records_per_map"]
    for r in ex["ranks"]:
        recs = O.gen_terasort(r["seed"], 0, 3 * rpm)
        data, index, peer = O.peer_major(part, recs, 100, rpm, ex["world"])
        assert sha(data) == r["send_sha256"] and peer.tolist() == r["peer_bytes"]
        assert index.tolist() == r["index"]


# ---- fetch restatement ----------------------------------------------------------------------------
def test_fetch_blocks_packs_in_request_order_and_batches():
    part = O.terasort_partitioner(10)
    maps = []
    for m in range(3):
        d, _, ix, be = O.write_map(part, O.gen_terasort(20 + m, 0, 700), 100)
        maps.append((d, ix, be))
    blocks = [(2, 3), (0, 0), (1, 2, 7), (0, 9), (2, 0, 10)]
    buf, sizes = O.fetch_blocks([m[0] for m in maps], [m[2] for m in maps], 10, blocks)
    want, want_sizes = b"", []
    for b in blocks:
        m, s = b[0], b[1]
        e = b[2] if len(b) > 2 else s + 1
        d, ix, _ = maps[m]
        want += bytes(d[ix[s]:ix[e]])
        want_sizes.append(int(ix[e] - ix[s]))
    assert buf == want
    assert sizes == want_sizes and sum(sizes) == len(buf)
    with pytest.raises(ValueError):
        O.fetch_blocks([m[0] for m in maps], [m[2] for m in maps], 10, [(3, 0)])


def test_zipf_table_and_generator_are_deterministic():
    b, t = O.zipf_table(1.1, 1 << 24)
    assert b[0] == 1 and b[-1] == (1 << 24) + 1 and (np.diff(b.astype(np.int64)) > 0).all()
    assert t[0] == 0 and (np.diff(t[:-1].astype(np.float64)) >= 0).all()
    a = O.gen_zipf(4, 1000, 50)
    c = O.gen_zipf(4, 0, 1050)[1000 * 100:]
    assert (a == c).all()
    keys = O.gen_zipf(4, 0, 20000).reshape(-1, 100)[:, :8].copy().view(np.int64).ravel()
    assert keys.min() >= 1 and keys.max() <= 1 << 24
    assert (keys == 1).mean() > 0.08  # Zipf(1.1) head: ~11.5% of draws are key 1


def test_cpu_baseline_runs_and_fetches_everything(tmp_path):
    recs = O.gen_terasort(5, 0, 20000)
    part = O.terasort_partitioner(16)
    res = O.cpu_shuffle(part, recs, 100, num_maps=4, threads=4, directory=str(tmp_path))
    assert res.bytes_in == recs.size and res.bytes_fetched == recs.size
    # the fetched multiset equals the input: compare the per-reducer checksum sum
    want = 0
    for p in range(16):
        blob = b""
        for m in range(4):
            sub = recs[m * 5000 * 100:(m + 1) * 5000 * 100]
            d, _, ix, _ = O.write_map(part, sub, 100)
            blob += bytes(d[ix[p]:ix[p + 1]])
        want = (want + O.checksum(np.frombuffer(blob, np.uint8).copy() if blob else np.zeros(0, np.uint8))) % (1 << 64)
    assert res.checksum == want
