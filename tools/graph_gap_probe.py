"""Lab: is the ~8.7 us GPU-idle gap between consecutive decode-graph replays (rocprofv3 kernel
trace of a 5-layer Qwen3-8B stage, B = 16, ctx 2048) a property of where the graph is launched?

Times `reps` back-to-back replays of one stage's decode graph (HIP events on the launching
stream) launched (a) on the current stream as the pipeline does by default (torch's default
stream), (b) on a dedicated torch.cuda.Stream (non-blocking), and (c) the same step launched
kernel by kernel (DecodeGraph.launch_eager -> inferd_span_step), interleaved, several rounds.

  python tools/graph_gap_probe.py > gpurun_out/graph_gap_probe.json
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from inferd_amd.pipeline import StageRange  # noqa: E402
from inferd_amd.runtime import MODELS, DecodeGraph, SpanRuntime  # noqa: E402


def main():
    d = MODELS["qwen3-8b"]
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    B, ctx, reps, rounds = 16, 2048, 40, 4
    r = StageRange(20, 10)
    n_launch = (rounds * 3 + 2) * (reps + 2)
    span = SpanRuntime(d, r.first_layer, r.n_layers, has_embed=False, has_lm_head=False,
                       kv_pages=B * ((ctx + n_launch) // 64 + 2) + 4, max_tokens=2 * ctx, max_seqs=B,
                       max_positions=ctx + n_launch + 64, device=dev)
    span.init_synthetic(1234)
    g = torch.Generator(device="cpu").manual_seed(7)
    sess = [("g", b) for b in range(B)]
    for c in range(0, B, 2):
        span.forward([(sid, ctx) for sid in sess[c:c + 2]],
                     x=(torch.randn(2 * ctx, d.hidden, generator=g) * 0.5).to(torch.bfloat16), want_hidden=False)
    x = (torch.randn(B, d.hidden, generator=g) * 0.5).to(torch.bfloat16).to(dev)
    hout = torch.empty(B, d.hidden, dtype=torch.bfloat16, device=dev)
    graph = DecodeGraph(span, sess, n_launch, x=x, hidden_out=hout)
    side = torch.cuda.Stream(device=dev)

    def timed(stream, eager=False):
        go = graph.launch_eager if eager else graph.launch
        with torch.cuda.stream(stream):
            for _ in range(2):
                go()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(reps):
                go()
            e1.record(stream)
        e1.synchronize()
        return e0.elapsed_time(e1) / reps * 1e3

    res = {"default_stream_us": [], "side_stream_us": [], "eager_us": []}
    for _ in range(rounds):
        res["default_stream_us"].append(round(timed(torch.cuda.current_stream(dev)), 2))
        res["side_stream_us"].append(round(timed(side), 2))
        res["eager_us"].append(round(timed(torch.cuda.current_stream(dev), eager=True), 2))
        torch.cuda.synchronize(dev)
    res["stage"] = r.label()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
