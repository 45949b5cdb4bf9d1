"""Probe: can two RCCL ranks share one GPU on this box (for testing the in-library
RCCL exchange on a 1-GPU machine)?  torchrun --nproc-per-node 2 ..."""
import os
import torch
import torch.distributed as dist

rank = int(os.environ["RANK"])
dist.init_process_group("nccl", rank=rank, world_size=int(os.environ["WORLD_SIZE"]),
                        device_id=torch.device("cuda:0"))
torch.cuda.set_device(0)
x = torch.full((4,), rank, dtype=torch.int32, device="cuda:0")
out = [torch.empty_like(x) for _ in range(2)]
dist.all_gather(out, x)
torch.cuda.synchronize()
print(rank, [o.tolist() for o in out], flush=True)
dist.destroy_process_group()
