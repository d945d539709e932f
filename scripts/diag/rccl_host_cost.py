"""Host-side cost of the ZeRO-1 step's collectives (diagnostic): a world-1
RCCL process group on the one GPU (the collectives are trivial copies there,
but every call pays torch.distributed's and RCCL's full host path) --
reduce_scatter_tensor / all_gather_into_tensor of bucket-sized tensors issued
back to back from the host, host time per call while the GPU runs ahead, then
the GPU time per call once it has drained.  Also the trainer's eager per-bucket
ops in emulation (copy_ + the Adam shard launch).  Prints one JSON line."""
import json
import os
import time

import torch
import torch.distributed as dist

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29533")
torch.cuda.set_device(0)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
out = {}
for mb in (4, 16):
    n = mb * 2 ** 20 // 4
    full = torch.zeros(n, device="cuda")
    shard = torch.zeros(n, device="cuda")
    h16 = torch.zeros(n, dtype=torch.float16, device="cuda")
    s16 = torch.zeros(n, dtype=torch.float16, device="cuda")
    for name, fn in (("reduce_scatter", lambda: dist.reduce_scatter_tensor(shard, full)),
                     ("all_gather", lambda: dist.all_gather_into_tensor(h16, s16)),
                     ("copy", lambda: shard.copy_(full))):
        for _ in range(20):
            fn()
        torch.cuda.synchronize()
        k = 300
        t0 = time.perf_counter()
        for _ in range(k):
            fn()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        out[f"{name}_{mb}MB_host_us"] = round((t1 - t0) / k * 1e6, 1)
        out[f"{name}_{mb}MB_total_us"] = round((t2 - t0) / k * 1e6, 1)
dist.destroy_process_group()
print(json.dumps(out))
