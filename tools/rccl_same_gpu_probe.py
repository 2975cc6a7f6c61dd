"""Probe: can two RCCL ranks share one GPU on this pool (so the pipeline's nccl path can be
rehearsed on a 1-GPU box)?  Run: python -m torch.distributed.run --nproc-per-node 2
--master-addr 127.0.0.1 --master-port 29511 tools/rccl_same_gpu_probe.py"""
import os

import torch
import torch.distributed as dist

rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
torch.cuda.set_device(0)
dev = torch.device("cuda", 0)
dist.init_process_group("nccl", device_id=dev)
x = torch.full((4,), float(rank), device=dev)
y = torch.empty(4, device=dev)
ops = [dist.P2POp(dist.isend, x, (rank + 1) % world), dist.P2POp(dist.irecv, y, (rank - 1) % world)]
for w in dist.batch_isend_irecv(ops):
    w.wait()
torch.cuda.synchronize()
print(f"rank {rank}: received {y.tolist()}", flush=True)
dist.barrier()
dist.destroy_process_group()
