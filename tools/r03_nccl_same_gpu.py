"""Probe: can two RCCL ranks share one GPU? (a graph-captured multi-rank step could then be
rehearsed on the 1-GPU box). Launched by torch.distributed.run with 2 ranks, both on cuda:0."""
import os
import torch
import torch.distributed as dist

torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
x = torch.full((4,), float(dist.get_rank() + 1), device="cuda")
dist.all_reduce(x)
torch.cuda.synchronize()
print("rank", dist.get_rank(), "all_reduce ->", x.tolist(), flush=True)
dist.destroy_process_group()
