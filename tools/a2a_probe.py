"""Exchange copies at one rank (GPU box diagnostic): does a 1.68 GB / 3.36 GB self exchange
arrive whole?  The --rccl-at-one self-check found the second half of every 32- and 16-map
group's received bytes zero (round 4).  Cases: sux_exchange_group on a one-rank RCCL
communicator, the same node's device-copy path (no communicator), torch's own all_to_all_single
over RCCL at world 1, and a plain tensor copy.
Then torch's all_to_all_single at world 1 over a sweep of sizes (where the loss starts).
usage: python tools/a2a_probe.py [maps=16] [sweep=0]
"""
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sparkucx_amd import native as N  # noqa: E402
from sparkucx_amd.shuffle import Node  # noqa: E402

MAP = 104857600  # one 2^20-record TeraSort map, bytes
R = 200


def table(maps):
    t = torch.empty(maps, R + 1, dtype=torch.int64)
    for m in range(maps):
        t[m] = torch.div(torch.arange(R + 1) * MAP, R, rounding_mode="floor")
    return t.reshape(-1)


def report(name, recv, send, nbytes):
    torch.cuda.synchronize()
    eq = torch.equal(recv[:nbytes], send[:nbytes])
    msg = f"{name}: {nbytes} bytes, equal {eq}"
    if not eq:
        # chunked so that no elementwise op spans more than 2^30 elements
        first, zeros = -1, 0
        for c0 in range(0, nbytes, 1 << 28):
            c1 = min(nbytes, c0 + (1 << 28))
            d = (recv[c0:c1] != send[c0:c1]).nonzero()
            if first < 0 and d.numel():
                first = c0 + int(d[0])
            zeros += int((recv[c0:c1] == 0).sum())
        msg += f"; first difference at byte {first} ({first / nbytes:.4f} of it), zero bytes {zeros}"
    print(msg, flush=True)


def main():
    maps = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    nbytes = maps * MAP
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    g = torch.Generator(device=dev)
    g.manual_seed(7)
    send = torch.randint(1, 256, (nbytes,), dtype=torch.uint8, device=dev, generator=g)
    idx = table(maps).to(dev)

    node = Node(device=0, rank=0, world_size=1, comm_id=N.unique_id())
    gath = torch.empty(maps * (R + 1), dtype=torch.int64, device=dev)
    recv = torch.zeros(nbytes, dtype=torch.uint8, device=dev)
    t0 = time.perf_counter()
    rb = node.exchange_group(send, idx, maps, R, gath, recv)
    report(f"sux_exchange_group, one-rank RCCL (recv_bytes {int(rb.sum())}, "
           f"{time.perf_counter() - t0:.3f} s)", recv, send, nbytes)
    recv.zero_()
    t = node.exchange_group_post(idx, maps, R, gath)
    rb = node.exchange_group_issue(t, send, recv)
    report(f"post/issue, one-rank RCCL (recv_bytes {int(rb.sum())})", recv, send, nbytes)
    node.close()

    plain = Node(device=0)
    recv.zero_()
    rb = plain.exchange_group(send, idx, maps, R, gath, recv)
    report(f"sux_exchange_group, device copy (recv_bytes {int(rb.sum())})", recv, send, nbytes)
    plain.close()

    recv.zero_()
    recv.copy_(send)
    report("torch copy_", recv, send, nbytes)

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    recv.zero_()
    dist.all_to_all_single(recv, send)
    report("torch all_to_all_single (RCCL, world 1)", recv, send, nbytes)
    if len(sys.argv) > 2 and sys.argv[2] == "1":
        G = 1 << 30
        for sz in (G - 256, G, G + 256, G + (G >> 1), 2 * G - 256, 2 * G, 2 * G + 256, 3 * G):
            if sz > nbytes:
                break
            recv.zero_()
            dist.all_to_all_single(recv[:sz], send[:sz])
            report(f"  all_to_all_single {sz} bytes", recv, send, sz)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
