"""Probe: can two processes share one GPU in an RCCL communicator?"""
import os
import sys
import torch
import torch.distributed as dist

rank = int(os.environ["RANK"])
dist.init_process_group("nccl", device_id=torch.device("cuda:0"))
x = torch.ones(4, device="cuda:0") * (rank + 1)
dist.all_reduce(x)
torch.cuda.synchronize()
y = torch.zeros(4, device="cuda:0")
if rank == 0:
    dist.send(x, 1)
else:
    dist.recv(y, 0)
torch.cuda.synchronize()
print(f"rank {rank} allreduce {x.tolist()} recv {y.tolist()}", flush=True)
dist.destroy_process_group()
