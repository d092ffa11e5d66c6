"""Diagnostic: which library call leaves a HIP error in the calling thread's last-error slot, and
does a torch kernel launch then fail?  Run on the GPU box: python3 tools/diag_hip.py"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.getcwd())
from sparkucx_amd import native as N  # noqa: E402
from sparkucx_amd.shuffle import Node  # noqa: E402

hip = ctypes.CDLL("libamdhip64.so.7")
hip.hipGetLastError.restype = ctypes.c_int
hip.hipPeekAtLastError.restype = ctypes.c_int
dev = ctypes.c_int(-1)


def state(what):
    hip.hipGetDevice(ctypes.byref(dev))
    print(f"{what:55s} peek={hip.hipPeekAtLastError()} device={dev.value}", flush=True)


def launch(what):
    try:
        torch.randint(0, 256, (16,), dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
        print(f"{what:55s} torch launch ok", flush=True)
    except Exception as e:  # noqa: BLE001
        print(f"{what:55s} torch launch FAILED: {str(e).splitlines()[0]}", flush=True)
        hip.hipGetLastError()


maps = open("/proc/self/maps").read()
print(sorted(set(l.split()[-1] for l in maps.splitlines()
                 if "amdhip" in l or "rccl" in l or "hsa-runtime" in l)), flush=True)
launch("baseline")
state("baseline")
uid = N.unique_id()
state("after unique_id")
launch("after unique_id")
node = Node(device=0, rank=0, world_size=1, comm_id=uid)
state("after Node(comm_id)")
launch("after Node(comm_id)")
R, maps_, MAP = 8, 2, 4096
index = (torch.arange(R + 1, dtype=torch.int64) * MAP // R).repeat(maps_).to("cuda")
gathered = torch.empty_like(index)
t = node.exchange_group_post(index, maps_, R, gathered)
state("after post")
launch("after post")
node.exchange_group_discard(t)
state("after discard")
launch("after discard")
node.close()
state("after close")
launch("after close")
node = Node(device=0)
state("after Node()")
launch("after Node()")
node.close()
state("after close 2")
launch("after close 2")
