"""GPU, multi-process: the exchange's RCCL code path at W > 1 on one GPU, through the loopback
build of the library (tests/loopback_rccl: every RCCL call of sux_api.cpp goes to a stand-in whose
messages travel through files, each receive checked against its matching send's size).  RCCL
itself refuses two ranks on one GPU, so before this the path — the index all-gather, the split
communicator of post/issue, the grouped ncclSend/ncclRecv pieces of <= 256 MiB and their pairing
between ranks — had only ever run with one rank.  Every run is bench.py's
N > 1 pipeline with its device self-check (and --verify against the CPU oracle where noted)."""
import ctypes as C
import json
import os
import re
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LOOP_LIB = os.path.join(ROOT, "sparkucx_amd", "libsparkucx_amd_loop.so")
PIECE = 256 << 20  # kA2aPiece, sux_api.cpp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(world, tmp_path, *args, timeout=400):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={world}", "--master-addr=127.0.0.1", f"--master-port={_free_port()}",
           os.path.join(ROOT, "bench.py"), "--gpus", str(world), "--loopback-rccl",
           "--no-cpu-baseline", *args]
    env = dict(os.environ, OMP_NUM_THREADS="1", SUX_LOOPBACK_DIR=str(tmp_path),
               SUX_LOOPBACK_LOG="1", SUX_LOOPBACK_TIMEOUT="150")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=env)
    if r.returncode != 0:
        errs = [l for l in r.stderr.splitlines()
                if ("Error" in l or "loopback rccl: rank" in l and "waited" in l
                    or "expects" in l) and "amdgpu.ids" not in l]
        raise AssertionError("\n".join(errs[:20]) + "\n" + r.stderr[-2000:])
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    msgs = [(m.group(1), int(m.group(2)), int(m.group(3)), int(m.group(5))) for m in re.finditer(
        r"loopback rccl: (\S+) rank (\d+) -> (\d+) #(\d+) (\d+) bytes", r.stderr)]
    # every message was received: a receive unlinks its file, and no comm directory keeps one
    left = [os.path.join(d, f) for d, _, fs in os.walk(tmp_path) for f in fs]
    assert not left, left[:5]
    return json.loads(lines[0]), msgs


def test_loopback_pairs_messages_in_order_and_rejects_a_size_mismatch(tmp_path, monkeypatch):
    """The stand-in itself, two communicators of one id in one process: messages of an ordered
    pair match in posting order, bytes intact; a receive whose size differs from its send's is
    ncclInvalidUsage (real RCCL would hang or corrupt), so a mispaired piece cannot pass."""
    import torch

    from sparkucx_amd import native as N

    N.load()  # torch's HIP runtime first (native._init_torch_hip_first), then the loop build
    monkeypatch.setenv("SUX_LOOPBACK_DIR", str(tmp_path))
    monkeypatch.setenv("SUX_LOOPBACK_TIMEOUT", "5")
    lib = C.CDLL(LOOP_LIB)

    class UniqueId(C.Structure):  # ncclUniqueId, passed by value to ncclCommInitRank
        _fields_ = [("internal", C.c_char * 128)]
    lib.sux_loop_ncclCommInitRank.argtypes = [C.POINTER(C.c_void_p), C.c_int, UniqueId, C.c_int]
    uid = UniqueId()
    assert lib.sux_loop_ncclGetUniqueId(C.byref(uid)) == 0
    comms = [C.c_void_p(), C.c_void_p()]
    for r in range(2):
        assert lib.sux_loop_ncclCommInitRank(C.byref(comms[r]), 2, uid, r) == 0
    a = torch.arange(3000, dtype=torch.int32, device="cuda").view(torch.uint8)
    b = torch.randint(0, 255, (500,), dtype=torch.uint8, device="cuda")
    s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    u8 = 1  # ncclUint8
    assert lib.sux_loop_ncclSend(C.c_void_p(a.data_ptr()), C.c_size_t(a.numel()), u8, 1,
                                 comms[0], s) == 0
    assert lib.sux_loop_ncclSend(C.c_void_p(b.data_ptr()), C.c_size_t(b.numel()), u8, 1,
                                 comms[0], s) == 0
    ra = torch.zeros_like(a)
    assert lib.sux_loop_ncclRecv(C.c_void_p(ra.data_ptr()), C.c_size_t(ra.numel()), u8, 0,
                                 comms[1], s) == 0
    assert torch.equal(ra, a)
    rb = torch.zeros(250, dtype=torch.uint8, device="cuda")
    rc = lib.sux_loop_ncclRecv(C.c_void_p(rb.data_ptr()), C.c_size_t(rb.numel()), u8, 0,
                               comms[1], s)
    assert rc == 5  # ncclInvalidUsage: 500 bytes sent, 250 expected
    for c in comms:
        assert lib.sux_loop_ncclCommDestroy(c) == 0


@pytest.mark.parametrize("mode", ["one-call", "post-issue"])
def test_two_ranks_through_the_rccl_path(tmp_path, mode):
    """W = 2, 6 launch groups per step, every group self-checked on the device; the plugin leg's
    windowed sux_exchange_maps runs through the same communicator."""
    res, msgs = _run(2, tmp_path, "--exchange", mode, "--records", "3000000", "--map-records",
                     "262144", "--group-maps", "2", "--steps", "2", "--warmup", "1")
    assert res["n_gpus"] == 2
    assert res["self_check"]["ok"] and res["self_check"]["groups"] == 6
    assert res["plugin"]["self_check"] == "ok"
    ex = res["roofline_exchange"]
    assert ex["exchange"] == mode
    assert 0.4 < ex["remote_bytes_per_rank"] / (3_000_000 * 100) < 0.6
    assert ex["probe"]["ok"] and ex["probe"]["transport"] == "rccl"
    # both ranks sent to each other, through one communicator (one-call) or the all-gathers on
    # the first and the all-to-alls on its split (post-issue)
    pairs = {(r, p) for _, r, p, _ in msgs}
    assert {(0, 1), (1, 0)} <= pairs
    dirs = {d for d, _, _, _ in msgs}
    assert any("split" in d for d in dirs) == (mode == "post-issue")


def test_pieces_of_256_mib_pair_up_between_ranks(tmp_path):
    """One 600 MB launch group per rank: each rank sends ~300 MB to its peer, cut into a full
    256 MiB piece and the rest (RCCL 2.26.6 loses data past 1 GiB in one count; sux_api.cpp
    all_to_all_pieces).  Both sides cut the same count the same way and the stand-in checks each
    piece's size against its receive; the device self-check checks the bytes."""
    res, msgs = _run(2, tmp_path, "--records", "6000000", "--map-records", str(1 << 20),
                     "--group-maps", "6", "--steps", "1", "--warmup", "0", "--plugin-groups", "0",
                     "--xgmi-probe-mib", "0")
    assert res["self_check"]["ok"] and res["self_check"]["groups"] == 1
    for src, dst in ((0, 1), (1, 0)):
        sizes = [n for _, r, p, n in msgs if (r, p) == (src, dst)]
        assert PIECE in sizes, (src, dst, sizes)  # a full piece, then the remainder
    assert max(n for *_, n in msgs) <= PIECE


def test_four_ranks_zipf_balanced_ownership_verified(tmp_path):
    """W = 4, Zipf keys (C4) with skew-balanced ownership: every received (source, map,
    partition) block compared with the CPU oracle inside the run (--verify)."""
    res, msgs = _run(4, tmp_path, "--workload", "zipf", "--records", "100000", "--map-records",
                     "20000", "--group-maps", "2", "--steps", "1", "--warmup", "0", "--verify",
                     "--ownership", "balanced", "--plugin-groups", "0")
    assert res["n_gpus"] == 4 and res["verified_groups"] == 3
    assert res["self_check"]["ok"]
    own = res["roofline_exchange"]["ownership"]
    assert own and own["plan"] == "balanced"
    assert {(r, p) for _, r, p, _ in msgs} >= {(r, p) for r in range(4) for p in range(4) if r != p}


def test_eight_ranks_verified_with_the_plugin_leg(tmp_path):
    """W = 8 (C3's rank count): 3 launch groups, every received block checked against the CPU
    oracle, then the plugin leg's windowed sux_exchange_maps over the same communicator."""
    res, msgs = _run(8, tmp_path, "--records", "100000", "--map-records", "20000", "--group-maps",
                     "2", "--steps", "1", "--warmup", "0", "--verify")
    assert res["n_gpus"] == 8 and res["verified_groups"] == 3
    assert res["self_check"]["ok"] and res["self_check"]["groups"] == 3
    assert res["plugin"]["self_check"] == "ok" and res["plugin"]["maps"] == 2 * 8 * 2
    assert len({(r, p) for _, r, p, _ in msgs}) == 64  # every ordered pair, self included


def test_three_ranks_uneven_partitions_verified(tmp_path):
    """W = 3 over R = 10 (owners of 3, 3 and 4 partitions), post-issue, every block checked
    against the CPU oracle: an odd world and an uneven split through the RCCL path."""
    res, msgs = _run(3, tmp_path, "--exchange", "post-issue", "--partitions", "10", "--records",
                     "120000", "--map-records", "20000", "--group-maps", "2", "--steps", "1",
                     "--warmup", "0", "--verify", "--plugin-groups", "0")
    assert res["n_gpus"] == 3 and res["verified_groups"] == 3
    assert res["self_check"]["ok"]
    assert {(r, p) for _, r, p, _ in msgs} >= {(r, p) for r in range(3) for p in range(3) if r != p}


def test_eight_ranks_default_line_explains_itself(tmp_path):
    """the N = 8 line (bench.py's defaults; sizes cut to fit one GPU, the RCCL
    calls through the loopback stand-in) carries everything the first 8-GPU driver run needs to
    explain itself: the measured peer peak and frac against it and against 7 x 153 GB/s, the
    busiest owner's ingress over the mean, exchange_hidden, and the device self-check — and every
    probe phase's duration."""
    res, _ = _run(8, tmp_path, "--records", "200000", "--map-records", "20000", "--group-maps",
                  "2", "--steps", "2", "--warmup", "1", "--plugin-groups", "0")
    ex = res["roofline_exchange"]
    for k in ("measured_peak", "frac", "frac_of_measured", "ingress_max_over_mean",
              "exchange_hidden", "device_self_check", "peak", "achieved"):
        assert ex.get(k) is not None, (k, ex)
    assert ex["peak"] == 7 * 153.0 and 0.0 <= ex["exchange_hidden"] <= 1.0
    assert ex["device_self_check"] == "ok" and res["self_check"]["ok"]
    assert {"buffers", "barrier", "first_exchange"} <= set(ex["probe"]["phases_ms"])


def test_eight_ranks_forced_mismatch_names_source_map_partition(tmp_path):
    """A received record corrupted on every rank: the device self-check fails the run (non-zero
    exit) and names the first mismatching (source, map, partition)."""
    with pytest.raises(AssertionError) as e:
        _run(8, tmp_path, "--records", "100000", "--map-records", "20000", "--group-maps", "2",
             "--steps", "1", "--warmup", "0", "--plugin-groups", "0", "--xgmi-probe-mib", "0",
             "--force-mismatch")
    msg = str(e.value)
    assert "first mismatch at source" in msg and "partition" in msg, msg[-3000:]
