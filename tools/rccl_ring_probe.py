"""Hand-off costs of the asynchronous decode ring (pipeline.PipelineStage), measured on ONE GPU.

A 1-GPU box cannot run two RCCL ranks (RCCL refuses two ranks on one device), so the cross-device
xGMI hop is not measurable here.  What is measured, as proxies (DESIGN.md §6 uses them):
  1. self_loop: a world-size-1 nccl group sending a record to itself (batch_isend_irecv of one send
     and one receive): the GPU time of the exchange (HIP events on the current stream, which waits
     on RCCL's stream), mean over 200, for the ring's record sizes -- the ids (64 B), the decode
     hidden rows of B = 16 (128 KiB), the head record (128 KiB + keys), a q/k/v-boundary record
     (320 KiB) and 1 MiB.  A local copy through RCCL's p2p machinery: kernel launch, protocol and
     a copy inside one HBM -- a lower bound for the xGMI hop, which adds bytes / link bandwidth.
  2. host_enqueue: host microseconds per batch_isend_irecv call (1 op) -- what the ring's host loop
     pays per hand-off post (the device never waits for it while the host runs ahead).
  3. queues: whether a kernel on one HIP stream runs while a resident waiting kernel (the stand-in
     for a receive posted before its data, tools/queue_lab.hip) sits on another stream: for each of
     n pool streams and the default stream, at GPU_MAX_HW_QUEUES as set in the environment.
  4. resident: how much k resident polling workgroups (a posted receive's channels) slow a 1 GiB
     device copy.
usage: python tools/rccl_ring_probe.py [out.json]"""
import ctypes as C
import json
import os
import sys
import time
from datetime import timedelta

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
out = {"gpu": torch.cuda.get_device_name(0), "GPU_MAX_HW_QUEUES": os.environ.get("GPU_MAX_HW_QUEUES", "(default)")}


def ev_time(fn, reps=200, warm=20):
    s = torch.cuda.current_stream()
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        fn()
    e1.record(s)
    e1.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


# ---- 3 / 4: queues and resident waiters (lab kernels)
lab = C.CDLL(os.path.join(ROOT, "tools", "labbin", "queue_lab.so"))
lab.lab_wait.argtypes = [C.c_void_p, C.c_double, C.c_int, C.c_int, C.c_void_p]
lab.lab_set.argtypes = [C.c_void_p, C.c_int, C.c_void_p]
flag = torch.zeros(64, dtype=torch.int32, device=dev)
small = torch.zeros(1024, device=dev)
streams = [torch.cuda.Stream() for _ in range(8)]
TIMEOUT_US = 30000.0
res = {}
for i, x in enumerate([torch.cuda.default_stream()] + streams[1:]):
    torch.cuda.synchronize()
    flag.zero_()
    torch.cuda.synchronize()
    lab.lab_wait(flag.data_ptr(), TIMEOUT_US, 1, 64, streams[0].cuda_stream)
    e = torch.cuda.Event()
    t0 = time.perf_counter()
    with torch.cuda.stream(x):
        small.add_(1.0)
        e.record(x)
    e.synchronize()
    dt = (time.perf_counter() - t0) * 1e6
    res["default" if i == 0 else f"pool{i}"] = round(dt, 1)
    torch.cuda.synchronize()
out["queues"] = {"waiter_on": "pool0", "waiter_timeout_us": TIMEOUT_US, "probe_done_after_us": res,
                 "blocked": [k for k, v in res.items() if v > TIMEOUT_US * 0.5]}
print("queues:", out["queues"], flush=True)

# a CU-masked stream over every CU (HIP gives such streams a hardware queue of their own, outside the
# GPU_MAX_HW_QUEUES pool): is it ever blocked by a waiter on the default stream or any pool stream?
hip = C.CDLL("libamdhip64.so")
ncu = torch.cuda.get_device_properties(0).multi_processor_count
mask = (C.c_uint32 * ((ncu + 31) // 32))(*([0xFFFFFFFF] * ((ncu + 31) // 32)))
if ncu % 32:
    mask[-1] = (1 << (ncu % 32)) - 1
sp = C.c_void_p()
rc = hip.hipExtStreamCreateWithCUMask(C.byref(sp), C.c_uint32(len(mask)), mask)
masked = torch.cuda.ExternalStream(sp.value, device=dev) if rc == 0 else None
mres = {}
if masked is not None:
    for i, wst in enumerate([torch.cuda.default_stream()] + streams):
        torch.cuda.synchronize()
        flag.zero_()
        torch.cuda.synchronize()
        lab.lab_wait(flag.data_ptr(), TIMEOUT_US, 1, 64, wst.cuda_stream)
        e = torch.cuda.Event()
        t0 = time.perf_counter()
        with torch.cuda.stream(masked):
            small.add_(1.0)
            e.record(masked)
        e.synchronize()
        mres["default" if i == 0 else f"pool{i - 1}"] = round((time.perf_counter() - t0) * 1e6, 1)
        torch.cuda.synchronize()
out["cu_masked_stream"] = {"create_rc": rc, "cus": ncu, "probe_done_after_us_by_waiter_stream": mres,
                           "blocked_by": [k for k, v in mres.items() if v > TIMEOUT_US * 0.5]}
print("cu-masked stream:", out["cu_masked_stream"], flush=True)
# and the reverse: a waiter ON the masked stream, probes on the default and pool streams
rres = {}
if masked is not None:
    for i, x in enumerate([torch.cuda.default_stream()] + streams):
        torch.cuda.synchronize()
        flag.zero_()
        torch.cuda.synchronize()
        lab.lab_wait(flag.data_ptr(), TIMEOUT_US, 1, 64, masked.cuda_stream)
        e = torch.cuda.Event()
        t0 = time.perf_counter()
        with torch.cuda.stream(x):
            small.add_(1.0)
            e.record(x)
        e.synchronize()
        rres["default" if i == 0 else f"pool{i - 1}"] = round((time.perf_counter() - t0) * 1e6, 1)
        torch.cuda.synchronize()
out["cu_masked_stream"]["waiter_on_masked_probe_us"] = rres
print("waiter on masked:", rres, flush=True)

big = torch.empty(1 << 29, dtype=torch.int16, device=dev)    # 1 GiB
dst = torch.empty_like(big)
cur = torch.cuda.current_stream()
resident = {}
for k in (0, 1, 4, 16, 64):
    ts = []
    for _ in range(6):
        torch.cuda.synchronize()
        flag.zero_()
        torch.cuda.synchronize()
        if k:
            lab.lab_wait(flag.data_ptr(), 20000.0, k, 256, streams[0].cuda_stream)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(cur)
        dst.copy_(big)
        e1.record(cur)
        lab.lab_set(flag.data_ptr(), 1, cur.cuda_stream)
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    torch.cuda.synchronize()
    resident[k] = round(sorted(ts)[len(ts) // 2], 1)
out["resident"] = {"copy_bytes": 2 * big.numel() * 2, "copy_us_by_waiting_workgroups": resident}
print("resident:", out["resident"], flush=True)
del big, dst

# ---- 1 / 2: RCCL self loop
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29547")
dist.init_process_group("nccl", rank=0, world_size=1, timeout=timedelta(seconds=60), device_id=dev)
loop = {}
for nbytes in (64, 131072, 131072 + 128, 327680, 1 << 20):
    a = torch.randint(0, 100, (nbytes,), dtype=torch.uint8, device=dev)
    b = torch.zeros_like(a)

    def ex():
        for w in dist.batch_isend_irecv([dist.P2POp(dist.isend, a, 0), dist.P2POp(dist.irecv, b, 0)]):
            w.wait()
    gpu_us = ev_time(ex)
    torch.cuda.synchronize()
    assert torch.equal(a, b)
    t0 = time.perf_counter()
    for _ in range(100):
        ex()
    host = (time.perf_counter() - t0) / 100 * 1e6
    torch.cuda.synchronize()
    loop[nbytes] = {"gpu_us": round(gpu_us, 2), "host_us_per_exchange": round(host, 1),
                    "host_us_per_op": round(host / 2, 1)}
    print(nbytes, loop[nbytes], flush=True)
out["self_loop"] = loop
out["note"] = ("self_loop: world-size-1 nccl send + receive of one record to itself, HIP events on the current "
               "stream around batch_isend_irecv + wait (a proxy: one GPU, no xGMI); host_us: the host's cost of "
               "the call (2 ops); queues: microseconds until a tiny kernel on each stream completed while a "
               "30 ms waiter sat on pool stream 0; resident: a 1 GiB device copy with k waiting 256-thread "
               "workgroups resident on another stream")
dist.destroy_process_group()
path = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "rccl_ring_probe.json")
os.makedirs(os.path.dirname(path), exist_ok=True)
with open(path, "w") as f:
    json.dump(out, f, indent=1)
print("wrote", path)
