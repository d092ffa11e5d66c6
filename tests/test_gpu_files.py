"""GPU: Spark's on-disk shuffle files from device map outputs (data + BE
index files for the local-disk fallback) — sux_write_map_files / sux_read_file_blocks against
the oracle's map outputs."""
import os

import numpy as np
import pytest
import torch

from oracle import oracle as O

pytestmark = pytest.mark.gpu


def test_write_and_read_map_files(gpu_node, tmp_path):
    R, rpm, n = 200, 30_000, 100_000
    recs = O.gen_terasort(41, 0, n)
    gp = gpu_node.partitioner(O.RANGE_BYTES, R, key_offset=0, key_len=10,
                              bounds=O.uniform_range_bounds(R, 10))
    d = torch.from_numpy(recs).cuda()
    out, index, _ = gpu_node.partition_maps(gp, d, 100, rpm)
    maps = -(-n // rpm)
    exp_data, exp_index, exp_be = O.write_maps(O.terasort_partitioner(R), recs, 100, rpm)
    dps = [str(tmp_path / f"shuffle_0_{m}_0.data") for m in range(maps)]
    ips = [str(tmp_path / f"shuffle_0_{m}_0.index") for m in range(maps)]
    lengths = gpu_node.write_map_files(out, index, maps, R, dps, ips)
    base = 0
    for m in range(maps):
        ix = exp_index[m * (R + 1):(m + 1) * (R + 1)]
        assert np.array_equal(lengths[m], np.diff(ix))
        assert open(ips[m], "rb").read() == exp_be[m * (R + 1) * 8:(m + 1) * (R + 1) * 8]
        assert open(dps[m], "rb").read() == exp_data[base:base + ix[R]].tobytes()
        for a, e in [(0, R), (0, 1), (17, 18), (50, 150), (199, 200), (80, 80)]:
            got = gpu_node.read_file_blocks(dps[m], ips[m], R, a, e)
            torch.cuda.synchronize()
            assert got.cpu().numpy().tobytes() == exp_data[base + ix[a]:base + ix[e]].tobytes()
        base += int(ix[R])
    # a second attempt of the same maps keeps the committed pair (and its lengths)
    again = gpu_node.write_map_files(out, index, maps, R, dps, ips)
    assert np.array_equal(again, lengths)
    assert sorted(os.listdir(tmp_path)) == sorted([os.path.basename(p) for p in dps + ips])


def test_read_rejects_bad_ranges(gpu_node, tmp_path):
    from sparkucx_amd.native import SuxError
    i, d = str(tmp_path / "x.index"), str(tmp_path / "x.data")
    open(i, "wb").write(np.array([0, 4, 8], ">i8").tobytes())
    open(d, "wb").write(b"abcdefgh")
    assert gpu_node.read_file_blocks(d, i, 2, 1, 2).cpu().numpy().tobytes() == b"efgh"
    with pytest.raises(SuxError):
        gpu_node.read_file_blocks(d, i, 2, 2, 1)
    with pytest.raises(SuxError):
        gpu_node.read_file_blocks(d, i, 3, 0, 1)  # index holds 2 partitions, not 3
