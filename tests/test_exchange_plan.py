"""CPU model of sux_exchange_maps' all-to-all (no GPU): the plan every rank computes from the
gathered directory (sux_plan_exchange, the same host function the exchange runs) is checked by
executing it — as ncclAllToAllv semantics (RCCL transport) and as one-sided pulls (IPC transport)
— over byte-exact peer-major batch slabs, and comparing every received block with the map's data
(OnOffsetsFetchCallback.java:53-87: a block is [off[start], off[end]) of the map's data file).

This is how the multi-rank RCCL branch is covered here: several ranks cannot share one GPU's RCCL
clique, so the arithmetic that feeds ncclAllToAllv is verified on the CPU for W = 2..8, and the
RCCL call itself runs on one GPU through the loopback (tests/test_gpu_exchange_maps.py)."""
import numpy as np
import pytest

from sparkucx_amd.shuffle import plan_exchange


def owner_lo(h, R, W):
    return (h * R) // W


def make_shuffle(rng, W, R, M, max_batch, drop):
    """Maps 0..M-1 dealt to ranks in batches of consecutive maps; each batch slab is peer-major
    [peer h][map][h's partitions].  Some written maps are not committed (another attempt won):
    they occupy slab bytes but are absent from the directory."""
    maps = {}      # map -> (owner, batch, data bytes, index)
    slabs = {}     # (owner, batch) -> bytes
    entries, seg, length = [], [], []
    m = 0
    batch_of_rank = [0] * W
    while m < M:
        g = int(rng.integers(W))
        nb = int(rng.integers(1, max_batch + 1))
        ids = list(range(m, min(M, m + nb)))
        m += len(ids)
        b = batch_of_rank[g] * 3 + int(rng.integers(3))  # batch ids need not be dense
        batch_of_rank[g] += 1
        datas = {}
        for mm in ids:
            sizes = rng.integers(0, 40, R) * int(rng.integers(0, 2) or 1)
            if rng.random() < 0.1:
                sizes[:] = 0  # empty map
            ix = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
            datas[mm] = (rng.integers(0, 256, int(ix[-1]), dtype=np.uint8), ix)
        slab = bytearray()
        segs = {mm: [0] * W for mm in ids}
        for h in range(W):
            lo, hi = owner_lo(h, R, W), owner_lo(h + 1, R, W)
            for mm in ids:
                d, ix = datas[mm]
                segs[mm][h] = len(slab)
                slab += d[ix[lo]:ix[hi]].tobytes()
        slabs[(g, b)] = bytes(slab)
        for mm in ids:
            if rng.random() < drop:
                continue  # written but not committed here
            d, ix = datas[mm]
            maps[mm] = (g, b, d, ix)
            entries.append((mm, g, b))
            seg.append(segs[mm])
            length.append([int(ix[owner_lo(h + 1, R, W)] - ix[owner_lo(h, R, W)])
                           for h in range(W)])
    return maps, slabs, entries, np.array(seg, np.uint64).reshape(-1, W), \
        np.array(length, np.uint64).reshape(-1, W)


def run_alltoall(W, slabs, entries, plans):
    """ncclAllToAllv semantics per round: rank h's receive region for source g in round k is
    filled from rank g's send buffer (its k-th batch slab) at g's sdispls[h]."""
    recv = [bytearray(int(p["round_base"][-1])) for p in plans]
    for k in range(plans[0]["rounds"]):
        for g in range(W):
            pe = plans[g]["piece"][k][g]
            for h in range(W):
                sc = int(plans[g]["sendcounts"][k][h])
                rc = int(plans[h]["recvcounts"][k][g])
                assert sc == rc, f"round {k}: {g}->{h} sends {sc}, receiver expects {rc}"
                if sc == 0:
                    continue
                mm, o, b = entries[pe]
                src = slabs[(o, b)]
                sd = int(plans[g]["sdispls"][k][h])
                dst = int(plans[h]["round_base"][k] + plans[h]["rdispls"][k][g])
                recv[h][dst:dst + sc] = src[sd:sd + sc]
    return recv


def run_pulls(W, slabs, entries, seg, plans):
    """The IPC transport: rank h pulls, per (round, source g), recvcounts bytes from g's piece
    slab at seg[piece entry][h]."""
    recv = [bytearray(int(p["round_base"][-1])) for p in plans]
    for h, p in enumerate(plans):
        for k in range(p["rounds"]):
            for g in range(W):
                pe = p["piece"][k][g]
                rc = int(p["recvcounts"][k][g])
                if pe < 0 or rc == 0:
                    continue
                mm, o, b = entries[pe]
                src = slabs[(o, b)]
                a = int(seg[pe][h])
                dst = int(p["round_base"][k] + p["rdispls"][k][g])
                recv[h][dst:dst + rc] = src[a:a + rc]
    return recv


def check_blocks(W, R, maps, entries, plans, recv, loopback):
    for h in range(W):
        lo, hi = owner_lo(h, R, W), owner_lo(h + 1, R, W)
        for i, (mm, g, b) in enumerate(entries):
            off = int(plans[h]["recv_off"][i])
            if g == h and not loopback:
                assert off == np.iinfo(np.uint64).max
                continue
            _, _, d, ix = maps[mm]
            for p in range(lo, hi):
                want = d[ix[p]:ix[p + 1]].tobytes()
                a = off + int(ix[p] - ix[lo])
                assert bytes(recv[h][a:a + len(want)]) == want, (h, mm, p)


@pytest.mark.parametrize("W", [2, 3, 5, 8])
@pytest.mark.parametrize("loopback", [False, True])
def test_plan_alltoall_and_pulls_move_every_owned_block(W, loopback):
    rng = np.random.default_rng(W * 7 + loopback)
    R = int(rng.integers(W, 4 * W + 9))
    maps, slabs, entries, seg, length = make_shuffle(rng, W, R, M=60, max_batch=7, drop=0.15)
    plans = [plan_exchange(W, h, entries, seg, length, loopback=loopback) for h in range(W)]
    assert len({p["rounds"] for p in plans}) == 1  # every rank runs the same number of rounds
    # the receive buffer is exact: owned bytes of every map received by the rank (+ gaps of
    # uncommitted maps inside a piece)
    for h in range(W):
        lo, hi = owner_lo(h, R, W), owner_lo(h + 1, R, W)
        own = sum(int(maps[mm][3][hi] - maps[mm][3][lo]) for mm, g, _ in entries
                  if g != h or loopback)
        assert int(plans[h]["round_base"][-1]) >= own
    check_blocks(W, R, maps, entries, plans, run_alltoall(W, slabs, entries, plans), loopback)
    check_blocks(W, R, maps, entries, plans, run_pulls(W, slabs, entries, seg, plans), loopback)


def test_plan_without_gaps_is_exact_and_one_round_per_batch():
    W, R = 4, 16
    rng = np.random.default_rng(3)
    maps, slabs, entries, seg, length = make_shuffle(rng, W, R, M=40, max_batch=5, drop=0.0)
    per_rank = [len({b for _, g, b in entries if g == h}) for h in range(W)]
    for h in range(W):
        p = plan_exchange(W, h, entries, seg, length)
        assert p["rounds"] == max(per_rank)
        lo, hi = owner_lo(h, R, W), owner_lo(h + 1, R, W)
        own = sum(int(maps[mm][3][hi] - maps[mm][3][lo]) for mm, g, _ in entries if g != h)
        assert int(p["round_base"][-1]) == own  # no gaps: exactly the owned bytes


def test_plan_empty_directory():
    p = plan_exchange(3, 1, [], np.zeros((0, 3)), np.zeros((0, 3)))
    assert p["rounds"] == 0 and int(p["round_base"][-1]) == 0
