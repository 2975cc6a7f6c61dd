"""Attention kernel timing on the GPU box through the C-ABI (inferd_attention).

prefill: Qwen3-32B dims (H=64, KV=8), B x T causal prompt (BASELINE config 5)
decode : Qwen3-8B dims (H=32, KV=8), B=16 single tokens at ctx 2048 (BASELINE config 3)
Random bf16 q and K/V (uniform, rule 25); algorithmic flops count T(T+1)/2 keys per row.
The library is the span library (a lab build is selected with INFERD_LIB; tools/attn_ab.py
compares several builds in one process).

usage: python tools/attn_bench.py [--mode prefill|decode]
"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from inferd_amd import _lib  # noqa: E402
from inferd_amd.runtime import KvTable  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--mode", default="prefill")
    p.add_argument("--T", type=int, default=8192)
    p.add_argument("--B", type=int, default=1)
    p.add_argument("--ctx", type=int, default=2048)
    p.add_argument("--rounds", type=int, default=5)
    p.add_argument("--reps", type=int, default=3)
    args = p.parse_args()
    L = _lib.load()
    dev = torch.device("cuda", 0)
    if args.mode == "prefill":
        H, KV, B, T, P = 64, 8, args.B, args.T, 0
    else:
        H, KV, B, T, P = 32, 8, 16, 1, args.ctx - 1
    n = T + P
    pages_per = (n + 63) // 64
    table = KvTable(B * pages_per)
    for b in range(B):
        table.reserve(b, n)
        table.advance(b, P)
    bd = table.build_batch([(b, T) for b in range(B)], dev)
    batch = _lib.batch_struct(bd.words, bd.shape)
    pool_pages = (B * pages_per + 15) // 16 * 16  # whole KV super-pages (common.h KV_SUPER)
    kv = (torch.rand(pool_pages * 2 * KV * 64 * 128, device=dev) * 2 - 1).to(torch.bfloat16)
    q = (torch.rand(B * T, H, 128, device=dev) * 4 - 2).to(torch.bfloat16)
    out = torch.empty(B * T, H * 128, dtype=torch.bfloat16, device=dev)
    ws_bytes = L.inferd_attention_workspace_bytes(B, H, n)
    ws = torch.zeros(max(ws_bytes, 256), dtype=torch.uint8, device=dev)
    st = _lib.stream_ptr()
    if args.mode == "prefill":
        flops = B * 4.0 * H * 128 * T * (T + 1) / 2
        bytes_ = None
    else:
        flops = B * 4.0 * H * 128 * n
        bytes_ = B * n * KV * 128 * 2 * 2
    times = []

    def call():
        _lib.check(L.inferd_attention(q.data_ptr(), kv.data_ptr(), batch, H, KV,
                                      out.data_ptr(), ws.data_ptr(), ws_bytes, st))
    for _ in range(args.rounds):
        call()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.reps):
            call()
        e1.record()
        torch.cuda.synchronize()
        times.append(e0.elapsed_time(e1) / args.reps)
    t = sorted(times)
    med = t[len(t) // 2]
    line = f"{args.mode}: {med * 1e3:9.1f} us  {flops / med / 1e9:7.1f} TF/s"
    if bytes_:
        line += f"  {bytes_ / med / 1e6:7.1f} GB/s"
    print(line, flush=True)


if __name__ == "__main__":
    main()
