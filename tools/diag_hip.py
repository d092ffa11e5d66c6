import torch, sys, os
sys.path.insert(0, os.getcwd())
print("avail before:", torch.cuda.is_available(), torch.cuda.device_count(), flush=True)
from sparkucx_amd import native as N
lib = N.load()
maps = open("/proc/self/maps").read()
print(sorted(set(l.split()[-1] for l in maps.splitlines() if "amdhip" in l or "rccl" in l or "hsa-runtime" in l)))
from sparkucx_amd.shuffle import Node
n = Node(device=0)
print("node ok", flush=True)
x = torch.empty(10, device="cuda")
print("torch alloc ok", flush=True)
