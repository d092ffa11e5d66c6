"""GPU, multi-process: bench.py's N>1 pipeline (ipc transport) rehearsed with several ranks on
cuda:0, TeraSort and Zipf keys, with --verify: every received (source, map, partition) block of
every launch group is compared with the CPU oracle inside the run."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(world, *args, timeout=300):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={world}", "--master-addr=127.0.0.1", f"--master-port={_free_port()}",
           os.path.join(ROOT, "bench.py"), "--gpus", str(world), "--rehearse-one-gpu", *args]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout,
                       env=dict(os.environ, OMP_NUM_THREADS="1"))
    if r.returncode != 0:  # the ranks' own exceptions first (the launcher's summary is long)
        errs = [l for l in r.stderr.splitlines() if "Error" in l and "amdgpu.ids" not in l]
        raise AssertionError("\n".join(errs[:20]) + "\n" + r.stderr[-2000:])
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def test_bench_two_ranks_one_gpu():
    res = _run(2, "--records", "3000000", "--map-records", "262144", "--group-maps", "2",
               "--steps", "2", "--warmup", "1")
    assert res["n_gpus"] == 2 and res["value"] > 0
    ex = res["roofline_exchange"]
    # uniform keys: about half of each rank's bytes leave it
    assert 0.4 < ex["remote_bytes_per_rank"] / (3_000_000 * 100) < 0.6
    # the N>1 device self-check ran over every launch group, and the plugin leg (write ->
    # windowed sux_exchange_maps -> wait -> fetch) passed its own device check
    assert res["self_check"]["ok"] and res["self_check"]["groups"] == 6
    assert res["plugin"]["self_check"] == "ok" and res["plugin"]["maps"] == 5 * 2 * 2
    # the same shuffle also ran map stage first, exchange after: both phases were timed
    assert res["plugin"]["serial_ms"]["writes"] > 0 and res["plugin"]["serial_ms"]["then_exchange"] > 0
    assert 0.0 <= res["plugin"]["exchange_hidden"] <= 1.0
    # the peer-read probe ran before the pipeline (flagged: both ranks share one GPU)
    probe = ex["probe"]
    assert probe["ok"] and probe["GB/s"] > 0 and "one_gpu" in probe
    assert ex["measured_peak"] > 0 and ex["frac_of_measured"] is not None


@pytest.mark.parametrize("workload", ["terasort", "zipf"])
def test_bench_eight_ranks_verified(workload):
    # 3 launch groups of 2 maps (the last one short), every block of every group checked
    n, rpm = 100_000, 20_000
    res = _run(8, "--workload", workload, "--records", str(n), "--map-records", str(rpm),
               "--group-maps", "2", "--steps", "1", "--warmup", "0", "--verify")
    assert res["n_gpus"] == 8
    assert res["verified_groups"] == 3
    ex = res["roofline_exchange"]
    assert ex["remote_bytes_per_rank"] > 0
    assert res["self_check"]["ok"] and res["self_check"]["groups"] == 3
    assert res["plugin"]["self_check"] == "ok" and res["plugin"]["maps"] == 2 * 8 * 2


def test_bench_eight_ranks_plugin_leg_after_the_pipeline():
    """100 MB batches at W = 8: the plugin leg runs after the stateless pipeline freed its IPC-
    shared send buffers, whose addresses come back for the plugin's slabs.  Each rank unmaps
    its peers' buffers (and all agree) before any is freed; a stale mapping handed out for a
    reused address used to feed the exchange the old bytes (its device check failed)."""
    res = _run(8, "--records", "4194304", "--map-records", "524288", "--group-maps", "2",
               "--plugin-groups", "4", "--steps", "1", "--warmup", "0", "--self-check", "0")
    assert res["plugin"]["self_check"] == "ok" and res["plugin"]["maps"] == 4 * 8 * 2


def test_bench_starts_its_own_ranks():
    """`python bench.py --gpus 2` with no launcher: bench.py starts its two ranks itself (child
    processes of torch.distributed.run), relays rank 0's line, and that line carries the N > 1
    self-check, the exchange roofline and the CPU baseline beside it."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--rehearse-one-gpu",
           "--records", "3000000", "--map-records", "262144", "--group-maps", "2", "--steps", "1",
           "--warmup", "0", "--plugin-groups", "0", "--cpu-records", "1000000", "--cpu-reps", "1"]
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300,
                       env=dict(env, OMP_NUM_THREADS="1"))
    assert r.returncode == 0, r.stderr[-3000:]
    assert "starting 2 ranks" in r.stderr
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["value"] > 0
    assert res["self_check"]["ok"]
    assert res["roofline_exchange"]["remote_bytes_per_rank"] > 0
    cb = res["cpu_baseline"]
    assert cb and cb["value"] > 0 and cb["cores"] >= 1
    assert cb["parity"]["index_tables_equal"] and cb["parity"]["fetch_checksum_equal"]


def _rccl_at_one(*args, timeout=300):
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--rccl-at-one", "--no-cpu-baseline",
           *args]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    return subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=env)


@pytest.mark.parametrize("mode", ["one-call", "post-issue"])
def test_bench_rccl_at_one(mode):
    """The N > 1 RCCL pipeline on a one-rank communicator (every byte to self), every group
    self-checked: 'one-call' (the default: all-gather + plan + all-to-all in one
    sux_exchange_group call) and 'post-issue' (the index all-gather of group k posted on its own
    stream, the all-to-all of group k - 1 issued after it over the split communicator)."""
    r = _rccl_at_one("--exchange", mode, "--records", "3000000", "--map-records", "262144",
                     "--group-maps", "2", "--steps", "2", "--warmup", "1")
    assert r.returncode == 0, r.stderr[-3000:]
    res = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    assert res["n_gpus"] == 1 and res["self_check"]["ok"] and res["self_check"]["groups"] == 6
    assert res["roofline_exchange"]["exchange_ms"] > 0
    assert res["roofline_exchange"]["exchange"] == mode
    probe = res["roofline_exchange"]["probe"]  # the RCCL probe ran through the library
    assert probe["ok"] and probe["transport"] == "rccl" and probe["GB/s"] > 0


def test_forced_mismatch_on_a_3_gb_group_reports_its_first_byte():
    """the self-check's diagnostic on a 3.36 GB group (32 maps of 2^20 TeraSort
    records) finds the first differing byte in bounded chunks instead of a whole-buffer
    nonzero() that asked torch for tens of exabytes."""
    r = _rccl_at_one("--records", str(32 << 20), "--map-records", str(1 << 20), "--group-maps",
                     "32", "--steps", "1", "--warmup", "0", "--force-mismatch", timeout=400)
    assert r.returncode != 0
    assert "first differing byte at" in r.stderr, r.stderr[-3000:]
    assert "Tried to allocate" not in r.stderr
    # the corrupted byte: the first key byte of the group's middle record
    want = (32 << 20) // 2 * 100
    assert f"first differing byte at {want} " in r.stderr, r.stderr[-3000:]
