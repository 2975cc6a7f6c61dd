"""Lab: do two decode microbatches replayed CONCURRENTLY on one GPU (two streams) fill each
other's kernel boundaries (launch ramp, tail, grid-wide gaps: the decode layer's ~17 us per
layer above its byte time) -- i.e. is the stage's HBM efficiency higher with two
microbatches in flight at once than with one at a time?

Two spans over the same layers (each its own weights copy, KV pool and workspaces: a span's
activation workspace is per handle), B sequences each prefilled with ctx tokens; one decode
graph per span.  Timed (HIP events, after warm-up): (a) sequential: both graphs on one stream,
one after the other, K steps; (b) concurrent: graph 1 on stream 1 and graph 2 on stream 2, K
steps each.  Prints ms per microbatch step and the ratio.
usage: python tools/concurrency_probe.py [--layers 9] [--steps 20]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from inferd_amd.runtime import MODELS, DecodeGraph, SpanRuntime  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", type=int, default=9)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--ctx", type=int, default=2048)
    a = ap.parse_args()
    d = MODELS["qwen3-8b"]
    dev = torch.device("cuda", 0)
    B, ctx, K = a.batch, a.ctx, a.steps
    n_steps = 3 * K + 8
    g = torch.Generator().manual_seed(5)
    spans, graphs = [], []
    for i in range(2):
        s = SpanRuntime(d, 9, a.layers, has_embed=False, has_lm_head=False, kv_pages=B * ((ctx + n_steps) // 64 + 2) + 4,
                        max_tokens=2 * ctx, max_seqs=B, max_positions=ctx + n_steps + 64, device=dev)
        s.init_synthetic(1234)
        sess = [("c", i, b) for b in range(B)]
        for c in range(0, B, 2):
            x = (torch.randn(2 * ctx, d.hidden, generator=g) * 0.5).to(torch.bfloat16)
            s.forward([(sid, ctx) for sid in sess[c:c + 2]], x=x, want_hidden=False)
        xin = (torch.randn(B, d.hidden, generator=g) * 0.5).to(torch.bfloat16).to(dev)
        hout = torch.empty(B, d.hidden, dtype=torch.bfloat16, device=dev)
        spans.append(s)
        graphs.append(DecodeGraph(s, sess, n_steps, x=xin, hidden_out=hout))
    torch.cuda.synchronize()
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    cur = torch.cuda.current_stream(dev)

    def ev():
        return torch.cuda.Event(enable_timing=True)

    for gr in graphs:        # warm-up
        for _ in range(4):
            gr.launch()
    torch.cuda.synchronize()
    # (a) sequential on one stream
    e0, e1 = ev(), ev()
    e0.record(cur)
    for _ in range(K):
        graphs[0].launch()
        graphs[1].launch()
    e1.record(cur)
    e1.synchronize()
    seq_ms = e0.elapsed_time(e1) / (2 * K)
    # (b) concurrent on two streams
    torch.cuda.synchronize()
    e0, e1 = ev(), ev()
    e0.record(cur)
    s1.wait_stream(cur)
    s2.wait_stream(cur)
    for _ in range(K):
        graphs[0].launch(s1)
        graphs[1].launch(s2)
    cur.wait_stream(s1)
    cur.wait_stream(s2)
    e1.record(cur)
    e1.synchronize()
    con_ms = e0.elapsed_time(e1) / (2 * K)
    # (a') sequential again (drift check)
    e0, e1 = ev(), ev()
    e0.record(cur)
    for _ in range(K):
        graphs[0].launch()
        graphs[1].launch()
    e1.record(cur)
    e1.synchronize()
    seq2_ms = e0.elapsed_time(e1) / (2 * K)
    for s in spans:
        s.check_errors()
    print(json.dumps({"layers": a.layers, "batch": B, "ctx": ctx, "steps": K,
                      "sequential_ms_per_microbatch_step": round(seq_ms, 4),
                      "sequential_again_ms": round(seq2_ms, 4),
                      "concurrent_ms_per_microbatch_step": round(con_ms, 4),
                      "concurrent_over_sequential": round(con_ms / min(seq_ms, seq2_ms), 4)}))


if __name__ == "__main__":
    main()
