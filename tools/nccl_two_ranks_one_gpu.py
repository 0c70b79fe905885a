"""Probe: can two RCCL ranks share one GPU on this box? (torchrun --nproc-per-node 2)"""
import os
import torch
import torch.distributed as dist
torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
t = torch.full((4,), float(dist.get_rank()), device="cuda")
out = torch.empty(8, device="cuda")
dist.all_gather_into_tensor(out, t)
torch.cuda.synchronize()
print("rank", dist.get_rank(), out.tolist(), flush=True)
dist.destroy_process_group()
