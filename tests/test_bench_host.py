"""CPU: bench.py's host-side pieces — the PMC traffic lookup, the host-core count, the launch-group
sizing, and the untimed self-check every bench line carries (it must pass on a correct map-side
output and reject a corrupted one).  The self-check runs here on CPU tensors, with the CPU oracle
standing in for the device's k_pids kernel (test infrastructure only)."""
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

import bench
from oracle import oracle as O


def test_traffic_lookup_is_keyed_by_workload_and_kernel():
    t = bench.load_traffic("terasort", "k_scatter8")
    assert t is not None and 200 < t["bytes_per_record"] < 210
    assert t["source"].endswith("terasort/k_scatter8")
    assert bench.load_traffic("terasort", "k_no_such_kernel") is None
    assert bench.load_traffic("no_such_workload", "k_scatter8") is None
    # a slot running two kernels sums them
    a = bench.load_traffic("small", "k_msd16a")["bytes_per_record"]
    b = bench.load_traffic("small", "k_msd16b")["bytes_per_record"]
    ab = bench.load_traffic("small", "k_msd16a+k_msd16b")["bytes_per_record"]
    assert ab == pytest.approx(a + b)


def test_host_cores_reports_a_usable_count():
    hc = bench.host_cores()
    assert hc["nproc"] >= 1 and 1 <= hc["use"] <= hc["affinity"] <= hc["nproc"]


@pytest.mark.parametrize("workload,want", [("terasort", 32), ("zipf", 32), ("small", 200)])
def test_default_launch_group_is_about_3_4_gb(workload, want):
    rs = bench.WORKLOADS[workload][0]
    assert max(1, round(bench.GROUP_BYTES / ((1 << 20) * rs))) == want


class _OracleNode:
    """partition_ids of the oracle, shaped like Node.partition_ids (int16 tensor)."""

    def __init__(self, opart):
        self.opart = opart

    def partition_ids(self, part, records, rs):
        ids = self.opart.ids(records.numpy(), rs).astype(np.int16)
        return torch.from_numpy(ids)


def _maps(R=16, n=5000, rpm=1200, rs=100):
    opart = O.terasort_partitioner(R)
    recs = O.gen_terasort(77, 0, n)
    data, index, _ = O.write_maps(opart, recs, rs, rpm)
    return (opart, torch.from_numpy(recs.copy()), torch.from_numpy(np.frombuffer(bytes(data), np.uint8).copy()),
            torch.from_numpy(index.astype(np.int64)), n, rs, rpm, R)


def test_self_check_accepts_the_oracle_output():
    opart, data, out, index, n, rs, rpm, R = _maps()
    res = bench.self_check(_OracleNode(opart), None, data, out, index, n, rs, rpm, R,
                           group_recs=2 * rpm, dev=torch.device("cpu"))
    assert res["ok"] and res["maps"] == -(-n // rpm)


def _expect_reject(mutate):
    opart, data, out, index, n, rs, rpm, R = _maps()
    mutate(out, index, rs, rpm)
    with pytest.raises(RuntimeError, match="self-check"):
        bench.self_check(_OracleNode(opart), None, data, out, index, n, rs, rpm, R,
                         group_recs=2 * rpm, dev=torch.device("cpu"))


def test_self_check_rejects_a_missing_record():
    _expect_reject(lambda out, index, rs, rpm: out[rs * 10:rs * 11].zero_())


def test_self_check_rejects_records_out_of_partition_order():
    def swap(out, index, rs, rpm):
        a = out[0:rs].clone()  # the first record (partition 0) and the map's last one
        out[0:rs] = out[(rpm - 1) * rs:rpm * rs]
        out[(rpm - 1) * rs:rpm * rs] = a
    _expect_reject(swap)


def test_self_check_rejects_a_wrong_index_table():
    def shift(out, index, rs, rpm):
        index[3] += rs
    _expect_reject(shift)


def _bench_cmd(*args):
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    return [sys.executable, os.path.join(root, "bench.py"), *args]


def test_bench_refuses_a_world_size_other_than_gpus():
    """A rank whose launcher started a different number of ranks than --gpus stops before it
    touches a GPU: its line would misreport n_gpus."""
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run(_bench_cmd("--gpus", "2"), capture_output=True, text=True, env=env,
                       timeout=120)
    assert r.returncode != 0 and "WORLD_SIZE=1" in r.stderr
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]


def test_bench_without_a_launcher_starts_its_ranks():
    """--gpus 2 and no WORLD_SIZE: bench.py becomes the parent of two ranks (torch.distributed.run
    child processes).  Without a GPU the ranks fail; the parent reports their status and prints
    no result line."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run(_bench_cmd("--gpus", "2", "--records", "1000"), capture_output=True,
                       text=True, env=env, timeout=300)
    assert "starting 2 ranks" in r.stderr and "torch.distributed.run" in r.stderr
    assert r.returncode != 0 and "ranks exited with status" in r.stderr
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]


def test_map_side_floor_follows_the_launched_design():
    """floor_frac: K1 read + K3 copy of 100-B records at the measured ceilings
    is ~0.49 of 8 TB/s; the MSD small-record path copies twice; a one-pass design once."""
    two = bench.map_side_floor({"hist": "k_hist4", "scatter": "k_scatter8"}, 100)
    assert 0.48 < two["floor_frac"] < 0.50
    msd = bench.map_side_floor({"hist": "k_msd16a", "scatter": "k_msd16b"}, 16)
    assert msd["floor_frac"] == pytest.approx(bench.COPY_CEIL_GBS / 2 / bench.HBM_PEAK_GBS, abs=1e-4)
    one = bench.map_side_floor({"hist": "", "scatter": "k_onepass"}, 100)
    assert one["floor_frac"] == pytest.approx(bench.COPY_CEIL_GBS / bench.HBM_PEAK_GBS, abs=1e-4)


def test_first_mismatch_is_chunked_and_exact():
    """The exchange diagnostic's first-differing-byte search in bounded chunks."""
    a = torch.zeros(10_000, dtype=torch.uint8)
    b = a.clone()
    assert bench.first_mismatch(a, b, chunk=1024) == (-1, 0)
    b[5000] = 1
    b[9999] = 7
    i, k = bench.first_mismatch(a, b, chunk=1024)
    assert i == 5000 and k == 1
    assert bench.first_mismatch(a, b, chunk=1 << 20) == (5000, 2)
