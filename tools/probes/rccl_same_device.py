"""Can two ranks share one GPU under RCCL?  torchrun --nproc-per-node 2 tools/probes/rccl_same_device.py: each
rank binds cuda:0, initialises the nccl (RCCL) backend and gathers a small tensor to rank 0."""
import os

import torch
import torch.distributed as dist

rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
x = torch.full((4,), float(rank), device="cuda:0")
out = [torch.empty_like(x) for _ in range(world)] if rank == 0 else None
dist.gather(x, out, dst=0)
if rank == 0:
    print("gathered", [t.tolist() for t in out], flush=True)
dist.barrier()
dist.destroy_process_group()
