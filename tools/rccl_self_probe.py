"""Probe: does RCCL on this stack run a p2p send/recv from a rank to itself (world size 1)?  If
so, the pipeline's nccl hand-off (PipelineStage._exchange) can execute on a 1-GPU box as a
self-loop.  usage: MASTER_ADDR=127.0.0.1 MASTER_PORT=<p> python tools/rccl_self_probe.py"""
import os
from datetime import timedelta

import torch
import torch.distributed as dist

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29533")
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", rank=0, world_size=1, timeout=timedelta(seconds=60), device_id=dev)
x = torch.arange(8, dtype=torch.float32, device=dev)
y = torch.zeros(8, device=dev)
for w in dist.batch_isend_irecv([dist.P2POp(dist.isend, x, 0), dist.P2POp(dist.irecv, y, 0)]):
    w.wait()
torch.cuda.synchronize()
print("self p2p:", y.tolist(), "ok" if torch.equal(x, y) else "MISMATCH", flush=True)
dist.destroy_process_group()
