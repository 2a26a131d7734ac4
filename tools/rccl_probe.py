"""Probe: can two ranks share one GPU in an RCCL (torch "nccl") group?  Run under
python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 tools/rccl_probe.py"""
import os

import torch
import torch.distributed as dist

rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
dev = int(os.environ.get("LOCAL_RANK", "0")) % torch.cuda.device_count()
torch.cuda.set_device(dev)
dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
x = torch.full((4,), float(rank + 1), device=f"cuda:{dev}", dtype=torch.int64)
dist.all_reduce(x)
torch.cuda.synchronize()
print(f"rank {rank}/{world} on cuda:{dev}: {x.tolist()}", flush=True)
dist.destroy_process_group()
