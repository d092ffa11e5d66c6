"""Generate the committed golden fixtures under tests/golden/ (run: python tests/golden/make_golden.py).

Provenance.  The reference (SparkUCX, JVM-only, no unit tests or fixtures — SURVEY.md §4/§8c)
cannot be run in this image, so two kinds of fixtures exist:
  * murmur3_kat.json — known answers of Spark's Murmur3_x86_32Suite (seed 0) and the Spark SQL
    seed-42 values quoted in SURVEY.md §8c: these pin the hash primitive to Spark itself;
  * every other file — outputs of the CPU restatement (oracle/oracle.c) frozen at the time of
    writing, so that the GPU path and later rounds are checked against fixed bytes.  They are
    "parity unpinned" against the reference itself (no JVM).
Inputs are not stored: they are regenerated from the counter-based generators, and each fixture
stores the sha256 of its input so a generator drift is caught too.
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from oracle import oracle as O  # noqa: E402


def sha(b) -> str:
    return hashlib.sha256(bytes(b)).hexdigest()


def dump(name, obj):
    with open(os.path.join(HERE, name), "w") as f:
        json.dump(obj, f, indent=1, sort_keys=True)
        f.write("\n")


def map_fixture(name, gen, gen_args, rec_size, part_kw, rpm=None):
    recs = gen(*gen_args)
    n = recs.size // rec_size
    part = O.Partitioner(**part_kw)
    pids = part.ids(recs, rec_size)
    rpm = rpm or n
    data, index, index_be = O.write_maps(part, recs, rec_size, rpm)
    obj = {
        "generator": gen.__name__, "gen_args": list(gen_args), "record_size": rec_size,
        "records_per_map": rpm, "num_records": n,
        "partitioner": {k: (v.hex() if isinstance(v, bytes) else v) for k, v in part_kw.items()},
        "input_sha256": sha(recs), "pids_sha256": sha(pids.astype("<u2").tobytes()),
        "pid_counts": np.bincount(pids, minlength=part.R).tolist(),
        "data_sha256": sha(data), "index_be_sha256": sha(index_be),
    }
    if len(index_be) <= 4096 * 8:
        obj["index_be_hex"] = index_be.hex()
    if n <= 4096:
        obj["pids_head"] = pids[:64].tolist()
    dump(name, obj)
    return recs, part, data, index, index_be


def main():
    # 1. Murmur3 known answers (Spark Murmur3_x86_32Suite, seed 0; Spark SQL seed 42)
    kat = {
        "source": "Spark Murmur3_x86_32Suite (seed 0) + SURVEY.md §8c seed-42 values",
        "hashInt_seed0": {"0": 593689054, "-42": -189366624, "42": -1134849565,
                          "-2147483648": -1718298732, "2147483647": -1653689534},
        "hashLong_seed0": {"0": 1669671676, "-42": -846261623, "42": 1871679806,
                           "-9223372036854775808": 1366273829,
                           "9223372036854775807": -2106506049},
        "hashInt_seed42": {"0": 933211791},
        "hashLong_seed42": {"0": -1670924195},
    }
    for k, tab in [("hashInt_seed0", kat["hashInt_seed0"]), ("hashLong_seed0", kat["hashLong_seed0"])]:
        f = O.murmur3_int if "Int" in k else O.murmur3_long
        for v, want in tab.items():
            assert f(int(v), 0) == want, (k, v)
    dump("murmur3_kat.json", kat)

    # 2. TeraSort, 4096 x 100 B, seed 1, range bounds, R in {7, 200}
    for R in (7, 200):
        map_fixture(f"terasort_4096_R{R}.json", O.gen_terasort, (1, 0, 4096), 100,
                    dict(kind=O.RANGE_BYTES, R=R, key_offset=0, key_len=10,
                         bounds=O.uniform_range_bounds(R, 10)))
    # 3. Zipf int64 keys, 4096 x 100 B, R=200, Spark SQL murmur3 hash
    map_fixture("zipf_4096_R200.json", O.gen_zipf, (0x5EED0004, 0, 4096, 1.1, 1 << 24), 100,
                dict(kind=O.MURMUR3_LONG, R=200, key_offset=0, key_len=8, seed=42))
    # 4. small records, 65536 x 16 B, R=10000 (index includes empty partitions)
    map_fixture("small_65536_R10000.json", O.gen_small, (0x5EED0005, 0, 65536), 16,
                dict(kind=O.MURMUR3_LONG, R=10000, key_offset=0, key_len=8, seed=42))
    # 5. multi-map TeraSort (ragged last map), R=200
    map_fixture("terasort_10000_rpm3000_R200.json", O.gen_terasort, (7, 0, 10000), 100,
                dict(kind=O.RANGE_BYTES, R=200, key_offset=0, key_len=10,
                     bounds=O.uniform_range_bounds(200, 10)), rpm=3000)
    # 6. exchange: 3 maps x 2 ranks, R=8 — expected per-(map, reduce) block hashes and the
    #    receive layout of each rank
    R, G, rpm = 8, 2, 500
    ex = {"R": R, "world": G, "records_per_map": rpm, "record_size": 100, "ranks": []}
    part = O.terasort_partitioner(R)
    for g in range(G):
        recs = O.gen_terasort(11 + g, 0, 3 * rpm)
        data, index, peer = O.peer_major(part, recs, 100, rpm, G)
        blocks = {}
        for m in range(3):
            d, _, ix, _ = O.write_map(part, recs[m * rpm * 100:(m + 1) * rpm * 100], 100)
            for p in range(R):
                blocks[f"{m}_{p}"] = sha(d[ix[p]:ix[p + 1]])
        ex["ranks"].append({"seed": 11 + g, "send_sha256": sha(data), "peer_bytes": peer.tolist(),
                            "index": index.tolist(), "blocks": blocks})
    dump("exchange_3maps_G2.json", ex)
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    main()
