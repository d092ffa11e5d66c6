"""CPU: the variable-length oracle against independent per-row Python
restatements — frame parsing, the Spark SQL Murmur3 hash of the key field, stable grouping."""
import numpy as np

from oracle import oracle as O


def parse(buf: bytes):
    rows, pos = [], 0
    while pos < len(buf):
        L = int.from_bytes(buf[pos:pos + 4], "big")
        rows.append(buf[pos:pos + 4 + L])
        pos += 4 + L
    assert pos == len(buf)
    return rows


def test_framing():
    data, offs = O.gen_unsafe_rows(1, 500, max_payload_words=5)
    rows = parse(data.tobytes())
    assert len(rows) == 500
    assert [len(r) for r in rows] == list(np.diff(offs))
    assert all(len(r) % 8 == 4 and r[4:12] == b"\0" * 8 for r in rows)


def test_varlen_maps_match_per_row_restatement():
    R, rpm = 13, 170
    data, offs = O.gen_unsafe_rows(2, 1000)
    part = O.Partitioner(O.MURMUR3_LONG, R, 12, 8)
    out, ix, be, pids = O.varlen_write_maps(part, data, offs, rpm)
    rows = parse(data.tobytes())
    key = [int.from_bytes(r[12:20], "little", signed=True) for r in rows]
    pid = [O.pmod(O.murmur3_long(k, 42), R) for k in key]
    assert list(pids) == pid
    exp, eix = b"", []
    for m0 in range(0, len(rows), rpm):
        mrows = list(range(m0, min(len(rows), m0 + rpm)))
        ix_m, off = [0], 0
        for p in range(R):
            for i in mrows:
                if pid[i] == p:
                    exp += rows[i]
                    off += len(rows[i])
            ix_m.append(off)
        eix += ix_m
    assert out.tobytes() == exp
    assert list(ix) == eix
    assert be == np.array(eix, ">i8").tobytes()


def test_caller_pids_and_empty():
    data, offs = O.gen_unsafe_rows(3, 0)
    out, ix, be, _ = O.varlen_write_maps(None, data, offs, 4, R=3, pids=np.zeros(0, np.uint16))
    assert out.size == 0 and ix.size == 0
    data, offs = O.gen_unsafe_rows(4, 9)
    pids = np.array([2, 0, 2, 1, 0, 0, 2, 1, 1], np.uint16)
    out, ix, _, _ = O.varlen_write_maps(None, data, offs, 9, R=3, pids=pids)
    rows = parse(data.tobytes())
    assert out.tobytes() == b"".join(rows[i] for i in [1, 4, 5, 3, 7, 8, 0, 2, 6])
