"""What a receive posted ahead of its data costs the compute it overlaps (the asynchronous ring,
pipeline.PipelineStage): a decode stage of the Qwen3-8B pipeline (one of vhead_halves8's stages, or the
given range), stepped as the pipeline steps it (eager step + its lm_head shard) on the dedicated compute
stream, timed alone and with k waiting workgroups resident on a pool stream -- the stand-in for the RCCL
receive kernel of the next item (tools/queue_lab.hip: it polls a device flag with s_sleep, as a receive
polls its FIFO), released after the timed steps.  Interleaved rounds, medians.

usage: python tools/resident_probe.py [--range 4m..8] [--rows 18560] [--rounds 5] [out.json]"""
import argparse
import ctypes as C
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--range", default="4m..8")
    p.add_argument("--rows", type=int, default=18560)
    p.add_argument("--first-row", type=int, default=14336)
    p.add_argument("--rounds", type=int, default=5)
    p.add_argument("--reps", type=int, default=20)
    p.add_argument("out", nargs="?", default=os.path.join(ROOT, "gpurun_out", "resident_probe.json"))
    a = p.parse_args()
    import bench
    from inferd_amd.pipeline import StageRange
    from inferd_amd.runtime import MODELS, DecodeGraph, SpanRuntime
    from inferd_amd.ops import ops as T
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    d = MODELS["qwen3-8b"]
    r = StageRange.from_label(a.range)
    B, ctx = 16, 2048
    cs = torch.cuda.ExternalStream(T.dedicated_stream(dev), device=dev)
    side = torch.cuda.Stream(device=dev)
    lab = C.CDLL(os.path.join(ROOT, "tools", "labbin", "queue_lab.so"))
    lab.lab_wait.argtypes = [C.c_void_p, C.c_double, C.c_int, C.c_int, C.c_void_p]
    lab.lab_set.argtypes = [C.c_void_p, C.c_int, C.c_void_p]
    flag = torch.zeros(64, dtype=torch.int32, device=dev)
    steps = a.rounds * 6 * (a.reps + 2) + 8
    g = torch.Generator().manual_seed(5)
    with torch.cuda.stream(cs):
        span = SpanRuntime(d, r.first_layer, r.n_layers, has_embed=False, has_lm_head=False,
                           kv_pages=B * ((ctx + steps) // 64 + 2) + 4, max_tokens=2 * ctx, max_seqs=B,
                           max_positions=ctx + steps + 64, device=dev, head_first=a.first_row, head_rows=a.rows,
                           **r.span_kwargs())
        span.init_synthetic(1234)
        sess = [("p", b) for b in range(B)]
        for c in range(0, B, 2):
            n_in = bench.buffer_elems(d, 2 * ctx, 0, r.first_o, False, r.first_q)
            span.forward([(s, ctx) for s in sess[c:c + 2]], x=(torch.randn(n_in, generator=g) * 0.5).to(torch.bfloat16),
                         want_hidden=r.last_o or r.last_q)
        n_in = bench.buffer_elems(d, B, r.first_col, r.first_o, True, r.first_q)
        x = (torch.randn(n_in, generator=g) * 0.5).to(torch.bfloat16).to(dev)
        hout = torch.empty(bench.buffer_elems(d, B, r.last_col, r.last_o, True, r.last_q), dtype=torch.bfloat16,
                           device=dev)
        graph = DecodeGraph(span, sess, steps, x=x, hidden_out=hout)
        hd = bench._StageHead(span, False, False, B, dev)

        def go():
            graph.launch_eager()
            hd()
        for _ in range(4):
            go()
        torch.cuda.synchronize()
        res = {k: [] for k in (0, 1, 4, 16)}
        for _ in range(a.rounds):
            for k in res:
                flag.zero_()
                torch.cuda.synchronize()
                if k:
                    lab.lab_wait(flag.data_ptr(), 100000.0, k, 256, side.cuda_stream)
                go()
                go()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(cs)
                for _ in range(a.reps):
                    go()
                e1.record(cs)
                lab.lab_set(flag.data_ptr(), 1, cs.cuda_stream)
                e1.synchronize()
                torch.cuda.synchronize()
                res[k].append(e0.elapsed_time(e1) / a.reps * 1e3)
    med = {k: round(sorted(v)[len(v) // 2], 2) for k, v in res.items()}
    out = {"stage": r.label(), "head_rows": a.rows, "us_per_step_by_waiting_workgroups": med, "all": res,
           "note": "decode step + lm_head shard of one vhead_halves8 stage, eager, on the dedicated compute stream; "
                   "k workgroups of 256 lanes polling a flag (s_sleep 8) on a pool stream during the timed steps"}
    print(json.dumps(out), flush=True)
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
