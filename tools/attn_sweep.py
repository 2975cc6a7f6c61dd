"""Decode-attention micro-benchmark (GPU): B sequences x ctx tokens x KV heads of random
bf16 K/V in the paged pool, one query token per sequence.  Prints achieved GB/s of the
KV stream.  INFERD_DECODE_PPW (env) overrides the pages-per-wave choice."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from inferd_amd import _lib  # noqa: E402
from inferd_amd.runtime import PagePool, SeqState, build_batch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=16)
    ap.add_argument("--ctx", type=int, default=2100)
    ap.add_argument("--H", type=int, default=32)
    ap.add_argument("--KV", type=int, default=8)
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    L = _lib.load()
    pages = (a.ctx + 63) // 64
    pool = PagePool(a.B * pages + 1)
    kv = torch.randn(pool.n_pages * 2 * a.KV * 64 * 128, device="cuda").to(torch.bfloat16)
    seqs = []
    for _ in range(a.B):
        st = SeqState(pages=pool.alloc(pages), length=a.ctx - 1)
        seqs.append((st, 1))
    batch, keep = build_batch(seqs, "cuda")
    q = torch.randn(a.B, a.H, 128, device="cuda").to(torch.bfloat16)
    out = torch.empty(a.B, a.H * 128, dtype=torch.bfloat16, device="cuda")
    wsb = L.inferd_attention_workspace_bytes(a.B, a.H, a.ctx)
    ws = torch.zeros(wsb, dtype=torch.uint8, device="cuda")
    args = (q.data_ptr(), kv.data_ptr(), batch, a.H, a.KV, out.data_ptr(), ws.data_ptr(), wsb, _lib.stream_ptr())
    for _ in range(5):
        _lib.check(L.inferd_attention(*args))
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters):
        _lib.check(L.inferd_attention(*args))
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / a.iters * 1e3
    byts = a.B * a.ctx * a.KV * 128 * 2 * 2
    print(f"ppw={os.environ.get('INFERD_DECODE_PPW', 'auto')} B={a.B} ctx={a.ctx} H={a.H} KV={a.KV}: "
          f"{us:.2f} us  {byts / us / 1e3:.1f} GB/s")


if __name__ == "__main__":
    main()
