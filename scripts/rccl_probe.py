"""Probe: can RCCL (torch "nccl" backend) run 2 ranks on ONE GPU?  Each rank all-reduces an int64
vector and all-gathers a slice; prints the outcome.  Launched by scripts/rccl_probe.sh."""
import os
import sys

import torch
import torch.distributed as dist

rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
x = torch.arange(8, dtype=torch.int64, device="cuda") + 100 * rank
dist.all_reduce(x)
g = [torch.empty(4, dtype=torch.int64, device="cuda") for _ in range(world)]
dist.all_gather(g, x[:4].clone())
torch.cuda.synchronize()
print(f"rank {rank}: all_reduce {x.tolist()} all_gather {[t.tolist() for t in g]}", flush=True)
dist.destroy_process_group()
sys.exit(0)
