"""The pipeline's RCCL hand-off on one GPU.

RCCL refuses two ranks on one device, so a 1-GPU box cannot run a 2-stage pipeline over
nccl; it does run a rank's p2p send/recv to itself (tools/rccl_self_probe.py).  This test
drives the real `PipelineStage._exchange` (the nccl branch: `batch_isend_irecv` on RCCL, the
stream wait, the one-tick lifetime of transient tensors, the first-exchange log) as a
self-loop in a world-size-1 nccl process group, in a subprocess so the test process keeps no
process group.  Shapes: the decode hand-off (B = 16 hidden rows of Qwen3-8B, bf16, plus the
int32 ids) and a prefill chunk (2 x 2048 rows)."""
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import sys, types, torch, torch.distributed as dist
from datetime import timedelta
sys.path.insert(0, sys.argv[1])
from inferd_amd.pipeline import PipelineStage
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", rank=0, world_size=1, timeout=timedelta(seconds=60), device_id=dev)
st = types.SimpleNamespace(group=None, rank=0, S=1, device=dev, first_layer=0, n_layers=36,
                           _exchanged=False, _inflight=None, _global=lambda r: r)
g = torch.Generator(device=dev).manual_seed(3)
ok = True
# decode ticks: fixed buffers (send h_out / ids_out, receive into h_in / ids)
h_out = torch.randn(16, 4096, device=dev, generator=g).to(torch.bfloat16)
h_in = torch.zeros_like(h_out)
ids_out = torch.randint(0, 151936, (16,), device=dev, dtype=torch.int32, generator=g)
ids_in = torch.zeros_like(ids_out)
for tick in range(4):
    h_out.add_(1.0)                      # the next graph replay rewrites the buffer
    PipelineStage._exchange(st, h_out, 0, h_in, 0)
    PipelineStage._exchange(st, ids_out, 0, ids_in, 0)
    torch.cuda.synchronize()
    ok &= torch.equal(h_in, h_out) and torch.equal(ids_in, ids_out)
# prefill ticks: a transient send per chunk and a fresh receive tensor, kept one tick
for tick in range(3):
    send = torch.randn(2 * 2048, 4096, device=dev, generator=g).to(torch.bfloat16)
    ref = send.clone()
    recv = torch.empty_like(send)
    PipelineStage._exchange(st, send, 0, recv, 0)
    del send
    torch.cuda.synchronize()
    ok &= torch.equal(recv, ref) and st._inflight is not None
# prefill ticks with NO synchronisation in between (ADVICE r04): each tick's send tensor is freed
# right after its exchange and a same-size tensor is allocated and overwritten at once -- the
# caching allocator may hand it the freed block; the one-tick lifetime (_inflight) and the
# stream wait must keep the in-flight send intact.  One synchronisation at the end.
refs, recvs = [], []
for tick in range(4):
    send = torch.randn(2 * 2048, 4096, device=dev, generator=g).to(torch.bfloat16)
    refs.append(send.clone())
    recvs.append(torch.empty_like(send))
    PipelineStage._exchange(st, send, 0, recvs[-1], 0)
    del send
    junk = torch.empty(2 * 2048, 4096, device=dev, dtype=torch.bfloat16)
    junk.fill_(7.0)
    del junk
torch.cuda.synchronize()
ok &= all(torch.equal(a, b) for a, b in zip(recvs, refs))
# a gate/up-boundary record: only its head travels (pipeline.handoff_elems), as a view
from inferd_amd.pipeline import handoff_elems, record_elems
from inferd_amd.runtime import MODELS
d = MODELS["qwen3-8b"]
rec_out = torch.randn(record_elems(d, 16), device=dev, generator=g).to(torch.bfloat16)
rec_in = torch.zeros_like(rec_out)
n = handoff_elems(d, 16, 4096)
PipelineStage._exchange(st, rec_out[:n], 0, rec_in[:n], 0)
torch.cuda.synchronize()
ok &= torch.equal(rec_in[:n], rec_out[:n]) and int(rec_in[n:].abs().sum()) == 0
dist.destroy_process_group()
print("RCCL_EXCHANGE_OK" if ok else "RCCL_EXCHANGE_MISMATCH", flush=True)
'''


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.gpu
@pytest.mark.timeout(240)
def test_pipeline_exchange_over_rccl_self_loop():
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    r = subprocess.run([sys.executable, "-c", CHILD, ROOT], env=env, capture_output=True, text=True, timeout=200)
    print(r.stdout[-2000:], r.stderr[-2000:])
    assert r.returncode == 0
    assert "RCCL_EXCHANGE_OK" in r.stdout
    assert "first exchange done over nccl" in r.stderr
