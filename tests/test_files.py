"""CPU: Spark's on-disk commit (IndexShuffleBlockResolver.writeIndexFileAndCommit [ext], the super
call at compat/spark_3_0/UcxShuffleBlockResolver.scala:35) through sux_index_file_commit —
host-only, against a Python restatement of the same rules."""
import os

import numpy as np

from sparkucx_amd.shuffle import index_file_commit


def be_index(lengths):
    return np.concatenate([[0], np.cumsum(lengths)]).astype(">i8").tobytes()


def test_fresh_commit(tmp_path):
    d, i, t = str(tmp_path / "s.data"), str(tmp_path / "s.index"), str(tmp_path / "s.tmp")
    open(t, "wb").write(b"x" * 60)
    lengths, reused = index_file_commit(i, d, t, [10, 0, 50])
    assert not reused and list(lengths) == [10, 0, 50]
    assert open(i, "rb").read() == be_index([10, 0, 50])
    assert open(d, "rb").read() == b"x" * 60 and not os.path.exists(t)
    assert sorted(os.listdir(tmp_path)) == ["s.data", "s.index"]  # no index temp left behind


def test_existing_consistent_pair_wins(tmp_path):
    d, i, t = str(tmp_path / "s.data"), str(tmp_path / "s.index"), str(tmp_path / "s.tmp")
    open(d, "wb").write(b"a" * 30)
    open(i, "wb").write(be_index([30, 0]))
    open(t, "wb").write(b"b" * 7)
    lengths, reused = index_file_commit(i, d, t, [3, 4])
    assert reused and list(lengths) == [30, 0]
    assert open(d, "rb").read() == b"a" * 30 and not os.path.exists(t)


def test_inconsistent_pair_is_replaced(tmp_path):
    d, i, t = str(tmp_path / "s.data"), str(tmp_path / "s.index"), str(tmp_path / "s.tmp")
    open(d, "wb").write(b"a" * 29)              # data length != index sum
    open(i, "wb").write(be_index([30, 0]))
    open(t, "wb").write(b"b" * 7)
    lengths, reused = index_file_commit(i, d, t, [3, 4])
    assert not reused and list(lengths) == [3, 4]
    assert open(d, "rb").read() == b"b" * 7 and open(i, "rb").read() == be_index([3, 4])
    # wrong size, nonzero first offset: replaced too
    open(i, "wb").write(be_index([3, 4])[:-8])
    assert not index_file_commit(i, d, None, [3, 4])[1]
    open(i, "wb").write(np.array([1, 4, 7], ">i8").tobytes())
    assert not index_file_commit(i, d, None, [3, 4])[1]


def test_missing_data_file_counts_as_empty(tmp_path):
    """java.io.File.length() of a missing file is 0: an all-empty index with no data file is a
    committed pair."""
    d, i = str(tmp_path / "s.data"), str(tmp_path / "s.index")
    open(i, "wb").write(be_index([0, 0, 0]))
    lengths, reused = index_file_commit(i, d, None, [1, 2, 3])
    assert reused and list(lengths) == [0, 0, 0]
