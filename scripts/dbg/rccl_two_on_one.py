"""Can two ranks share one GPU under RCCL (torch.distributed 'nccl')?  Launch with
torch.distributed.run --nproc-per-node 2; both ranks use cuda:0."""
import os

import torch
import torch.distributed as dist

rank = int(os.environ["RANK"])
torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
x = torch.full((4,), float(rank + 1), device="cuda")
dist.all_reduce(x)
y = torch.empty(4, device="cuda")
if rank == 0:
    dist.send(x * 10, 1)
else:
    dist.recv(y, 0)
torch.cuda.synchronize()
print(f"rank {rank}: allreduce {x.tolist()} recv {y.tolist() if rank == 1 else '-'}", flush=True)
dist.destroy_process_group()
