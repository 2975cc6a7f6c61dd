"""Headline benchmark: decode tokens/s of the Qwen3-8B layer-span pipeline (BASELINE.json).

Workload (BASELINE.json configs[2], the metric's config): Qwen3-8B, batch 16 decode at
2k context.  Synthetic token ids, synthetic weights from the counter-based generator
(no checkpoint is reachable offline).  One "step" = one decode step of every in-flight
microbatch of 16 sequences through all 36 layers + final norm + lm_head + greedy argmax.

  N = 1 : the whole model is one span on one GPU.
  N > 1 : the 36 layers are split into N even spans, one per GPU/rank -- BASELINE config 3:
          [18,18], [9,9,9,9], [5,5,5,5,4,4,4,4] at N = 2/4/8 (`--split balanced` prices each
          stage by its algorithmic decode bytes, the last stage also streaming the 1.24 GB
          lm_head: [19,17], [9,10,10,7], [4,5,5,5,5,5,5,2]); N microbatches of 16 sequences are in
          flight; hidden states move stage -> stage with RCCL send/recv over xGMI, greedy ids
          return last -> first.  Per-GPU work is fixed as N grows ("scaling": "weak").

Before timing: every sequence is prefilled with 2048 tokens through the real prefill
path (untimed; its rate is reported as `prefill`), so the KV cache holds real K/V.
Timed region: K decode steps bracketed by barrier + synchronize; each stage's step of a
microbatch is one replay of a captured HIP graph; value = tokens of all ranks /
max-over-ranks time.  Roofline: per-kernel-class HIP events (inferd_span_profile_*) on
the launch stream around every kernel of `--profile-steps` eager decode steps of the same
workload, run right after the timed region (HIP cannot time event nodes inside a replayed
graph); the dominant kernel class's algorithmic bytes per launch / its mean event time,
against 8 TB/s HBM.  `traffic` = PMC-measured HBM bytes per launch of that class
(tools/profile_round.sh -> the newest profiles/traffic_rNN.json).  cpu_baseline: the oracle
(oracle/qwen3_ref.py, `port`) on the host cores, rank 0 at N = 1 only.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
from inferd_amd.pipeline import balanced_split, buffer_elems, even_split  # noqa: E402  (host logic only)

HBM_PEAK_GBS = 8000.0        # MI355X HBM3E spec (MI355X_MICROARCH.md)
MFMA_BF16_PEAK_TFLOPS = 2500.0


def latest_traffic(kind: str, workload: str):
    """The newest committed PMC traffic summary (profiles/traffic[_prefill]_rNN.json) measured
    on `workload`: {kernel class: HBM bytes per launch}, or None."""
    import glob
    pat = os.path.join(ROOT, "profiles", f"traffic{'_prefill' if kind == 'prefill' else ''}_*r[0-9]*.json")
    for fn in sorted(glob.glob(pat), key=lambda f: f[-7:], reverse=True):
        with open(fn) as f:
            tr = json.load(f)
        if tr.get("workload") == workload:
            return tr.get("per_launch_bytes", {})
    return None


def measured_peaks(dev) -> dict:
    """The two peaks re-measured on this box by the library's probe kernels
    (inferd_amd/csrc/probe.hip), event-timed on the launch stream: a 1 GiB grid-stride read
    (beyond the 256 MiB Infinity Cache) and dense v_mfma_f32_16x16x32_bf16 chains from
    registers.  Median of 5 after 3 warm-ups.  Reported beside the spec peaks, which stay the
    roofline denominators."""
    import ctypes as C
    from inferd_amd import _lib
    L = _lib.load()
    s = torch.cuda.current_stream(dev)
    buf = torch.ones(1 << 28, dtype=torch.int32, device=dev)          # 1 GiB
    sink = torch.zeros(1024, dtype=torch.int32, device=dev)
    flops = C.c_double(0.0)

    def timed(launch):
        ts = []
        for i in range(8):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            launch()
            e1.record(s)
            e1.synchronize()
            if i >= 3:
                ts.append(e0.elapsed_time(e1) * 1e-3)
        return sorted(ts)[len(ts) // 2]

    nbytes = buf.numel() * 4
    t_rd = timed(lambda: _lib.check(L.inferd_probe_hbm_read(buf.data_ptr(), nbytes, sink.data_ptr(), 1024,
                                                            s.cuda_stream)))
    iters, n_wg = 8192, 2048
    t_mf = timed(lambda: _lib.check(L.inferd_probe_mfma(iters, n_wg, sink.data_ptr(), s.cuda_stream,
                                                        C.byref(flops))))
    del buf
    return {"hbm_read_GBps": round(nbytes / t_rd / 1e9, 1), "hbm_spec_GBps": HBM_PEAK_GBS,
            "mfma_bf16_TFLOPs": round(flops.value / t_mf / 1e12, 1), "mfma_spec_TFLOPs": MFMA_BF16_PEAK_TFLOPS,
            "how": "probe.hip: 1 GiB read (1024 workgroups x 8 waves, 1 MiB contiguous each, 16 B loads, 8 in "
                   "flight per lane); 2048 x 4 waves of 8 independent v_mfma_f32_16x16x32_bf16 chains on random "
                   "operands; HIP events, median of 5 after 3 warm-ups"}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=32)
    p.add_argument("--warmup", type=int, default=4)
    p.add_argument("--model", default="qwen3-8b")
    p.add_argument("--batch", type=int, default=16)
    p.add_argument("--ctx", type=int, default=2048)
    p.add_argument("--seed", type=int, default=1234)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-layers", type=int, default=2, help="layers timed by the CPU baseline sample")
    p.add_argument("--no-profile", action="store_true", help="skip the per-kernel HIP-event timing pass")
    p.add_argument("--no-prefill-line", action="store_true",
                   help="N=1 decode runs: skip the config-5 prefill measurement added to the JSON line")
    p.add_argument("--profile-steps", type=int, default=8, help="eager event-instrumented decode steps")
    p.add_argument("--prefill-chunk", type=int, default=2, help="sequences per prefill call")
    p.add_argument("--spans", default="", help="comma-separated layers per stage (BASELINE config 4: an uneven, "
                                                "balance.py-like split, e.g. 5,27,4; multiples of 0.5 cut between a "
                                                "layer's attention and MLP halves, e.g. 4.5,4.5,5,...); overrides "
                                                "--split")
    p.add_argument("--split", choices=("balanced", "even", "halves", "gateup", "sublayer"), default="even",
                   help="stage layer counts: even = counts differing by at most one (BASELINE config 3, the "
                        "default), balanced = min-max of per-stage decode bytes (lm_head priced on the last stage), "
                        "halves = min-max of per-stage decode time with cuts between a layer's attention and MLP "
                        "halves allowed (pipeline.halves_split), gateup = the same with boundaries inside a layer's "
                        "gate/up projection too (pipeline.gateup_split), sublayer = also between a layer's "
                        "attention and its o projection (pipeline.sublayer_split)")
    p.add_argument("--mode", choices=("decode", "prefill", "stages"), default="decode",
                   help="prefill: BASELINE config 5 (one 8-layer Qwen3-32B stage, 8k prompts, MFMA roofline); "
                        "stages: the per-stage decode projection of the 2/4/8-GPU splits on one GPU")
    p.add_argument("--no-sublayer-split", action="store_true",
                   help="N > 1 runs of the even split: skip the second measurement on the sub-layer split")
    p.add_argument("--no-stage-projection", action="store_true",
                   help="N=1 decode runs: skip the per-stage projection of the 2/4/8-GPU splits")
    p.add_argument("--head", choices=("vocab", "last"), default="vocab",
                   help="N > 1: vocab = the greedy head vocab-parallel over the stages (lm_head shards sized by "
                        "head_shards, the normed rows and running keys handed round the ring; the default), last = the "
                        "whole lm_head on the last stage (the reference's LastStage)")
    p.add_argument("--ring-slack", type=int, default=1,
                   help="microbatches in flight beyond the ring's minimum (S, or 2S with the vocab-parallel head)")
    p.add_argument("--no-calibrate", action="store_true",
                   help="N > 1, vocab head: size the lm_head shards from the cost table only (default: every rank "
                        "times its own stage first and the shards are re-balanced on the measured times)")
    p.add_argument("--prefill-layers", type=int, default=8)
    p.add_argument("--prefill-batch", type=int, default=1)
    p.add_argument("--prefill-len", type=int, default=8192)
    return p.parse_args()


def prefill_flops(d, n_layers: int, B: int, T: int) -> float:
    """Algorithmic flops of a span prefill: 2*params*tokens for the projections plus causal
    attention 2*2*H*d*T(T+1)/2 per sequence and layer."""
    h, I, H, KV, hd = d.hidden, d.intermediate, d.heads, d.kv_heads, d.head_dim
    lin = h * (H + 2 * KV) * hd + H * hd * h + 3 * h * I
    return n_layers * B * (2.0 * lin * T + 4.0 * H * hd * T * (T + 1) / 2)


def run_prefill(args):
    """`--mode prefill`: the config-5 line alone."""
    print(json.dumps(prefill_line(args, args.steps, args.warmup, torch.device("cuda", 0))), flush=True)


def run_stages(args):
    """`--mode stages`: the per-stage decode projection alone."""
    from inferd_amd.runtime import MODELS
    dev = torch.device("cuda", 0)
    d = MODELS[args.model]
    splits = projection_splits(d, args.batch, args.ctx)
    if args.spans:
        from inferd_amd.pipeline import ranges_from_sizes
        splits = {"spans": ranges_from_sizes(args.spans.split(","))}
    print(json.dumps({"stage_projection": stage_projection(d, splits, args.batch, args.ctx, dev, args.seed,
                                                           reps=args.steps)}), flush=True)


def prefill_line(args, steps: int, warmup: int, dev, peaks: bool = True) -> dict:
    """Config 5: one pipeline stage of Qwen3-32B (8 of 64 layers) prefilling B x 8k tokens.
    Per-GPU work of the 8-stage pipeline; the hand-off is one 8k x 5120 bf16 tensor."""
    from inferd_amd.runtime import MODELS, SpanRuntime
    d = MODELS["qwen3-32b" if args.model == "qwen3-8b" else args.model]
    B, T, L = args.prefill_batch, args.prefill_len, args.prefill_layers
    span = SpanRuntime(d, 8, L, has_embed=False, has_lm_head=False, kv_pages=B * (T // 64 + 2) + 4,
                       max_tokens=B * T, max_seqs=max(B, 1), max_positions=T + 64, device=dev)
    span.init_synthetic(args.seed)
    x = (torch.randn(B * T, d.hidden, device=dev) * 0.5).to(torch.bfloat16)
    for _ in range(warmup):
        span.forward([(None, T)] * B, x=x, want_hidden=True)
    # K prefill calls back to back between two synchronizes (same bracket as the decode
    # timing): each call's host work (page reservation, batch descriptor, H2D of its
    # metadata) is inside the timed region and overlaps the previous call's kernels
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        span.forward([(None, T)] * B, x=x, want_hidden=True)
    torch.cuda.synchronize()
    t = (time.perf_counter() - t0) / steps
    fl = prefill_flops(d, L, B, T)
    span.profile_start(1 << 12)
    span.forward([(None, T)] * B, x=x, want_hidden=True)
    torch.cuda.synchronize()
    prof = span.profile_stop()
    kernels = {k: {"launches": n, "avg_ms": round(ms / max(n, 1), 3)} for k, (ms, n) in prof.items() if n}
    tf = fl / t / 1e12
    # PMC-measured L2-to-fabric bytes per launch of the dominant kernel class
    # (tools/pmc_prefill.sh -> the newest profiles/traffic_prefill_rNN.json; MALL hits count)
    dom = max(kernels, key=lambda k: kernels[k]["avg_ms"] * kernels[k]["launches"])
    tr = latest_traffic("prefill", f"{d.name}-prefill-{L}layers-T{T}" + (f"-B{B}" if B > 1 else ""))
    traffic = None if tr is None else tr.get(dom)
    del span
    return {
        "metric": "prefill tokens/sec, Qwen3-32B 8-layer span (one of 8 pipeline stages)",
        "value": round(B * T / t, 1), "unit": "tokens/s", "n_gpus": 1, "steps": steps,
        "warmup": warmup, "ms_per_step": round(t * 1e3, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "bf16",
        "data": "synthetic hidden states + counter-generated synthetic weights",
        "config": {"workload": f"qwen3-32b layers 8-{8 + L - 1}, prefill {B} x {T} tokens",
                   "global_batch": B, "seq_len": T, "parallelism": "pp-stage"},
        "roofline": {"bound": "mfma", "achieved": round(tf, 1), "peak": MFMA_BF16_PEAK_TFLOPS,
                     "unit": "TFLOP/s", "frac": round(tf / MFMA_BF16_PEAK_TFLOPS, 4), "traffic": traffic,
                     "traffic_kernel": dom,
                     "alg_flops_per_step": fl},
        "kernels": kernels,
        "peaks_measured": measured_peaks(dev) if peaks else None}


def stage_split(d, n: int, B: int, ctx: int, how: str = "even"):
    """Layer ranges per stage.  "even" (default, BASELINE config 3): layer counts differing by
    at most one; "balanced": inferd_amd.pipeline.balanced_split with each stage priced by its
    algorithmic decode bytes (HBM-bound), so the last stage, which also streams the 1.24 GB
    lm_head, gets fewer layers."""
    if how == "even":
        return even_split(d.layers, n)
    kb = kernel_bytes(d, B, ctx)
    return balanced_split(d.layers, n, step_bytes(d, 1, B, ctx, False), kb["lm_head_argmax"])


# ------------------------------------------------------------------ algorithmic traffic
def kernel_bytes(d, B: int, ctx_mean: float) -> dict:
    """Algorithmic HBM bytes per launch of each kernel class for one decode step of B
    sequences at mean context ctx_mean (weights read once, activations read/written once,
    KV read once per layer)."""
    h, I, H, KV, hd = d.hidden, d.intermediate, d.heads, d.kv_heads, d.head_dim
    qkvN = (H + 2 * KV) * hd
    return {
        "rmsnorm": 2 * B * h * 2 + h * 2,
        "qkv_gemm": qkvN * h * 2 + B * h * 2 + B * qkvN * 2,
        "qk_norm_rope_kv": B * qkvN * 2 + B * H * hd * 2 + B * 2 * KV * hd * 2 + 2 * B * 64 * 2 * 2,
        "attention": B * ctx_mean * 2 * KV * hd * 2 + B * H * hd * 2 * 2,
        "o_gemm": h * H * hd * 2 + B * H * hd * 2 + 2 * B * h * 2,
        "gateup_gemm": 2 * I * h * 2 + B * h * 2 + B * I * 2,
        "down_gemm": h * I * 2 + B * I * 2 + 2 * B * h * 2,
        "lm_head_argmax": d.vocab * h * 2 + B * h * 2,
    }


def step_bytes(d, n_layers: int, B: int, ctx_mean: float, lm_head: bool) -> float:
    kb = kernel_bytes(d, B, ctx_mean)
    per_layer = sum(kb[k] for k in ("qkv_gemm", "qk_norm_rope_kv", "attention", "o_gemm", "gateup_gemm",
                                    "down_gemm")) + 2 * kb["rmsnorm"]
    return n_layers * per_layer + (kb["lm_head_argmax"] if lm_head else 0)


def range_bytes(d, r, B: int, ctx_mean: float, lm_head: bool) -> float:
    """Algorithmic decode bytes of a StageRange: per attention half its input norm, q/k/v,
    QK-norm/RoPE/cache write, attention and o; per MLP half its norm, gate/up and down."""
    kb = kernel_bytes(d, B, ctx_mean)
    attn = kb["rmsnorm"] + kb["qkv_gemm"] + kb["qk_norm_rope_kv"] + kb["attention"] + kb["o_gemm"]
    mlp = kb["rmsnorm"] + kb["gateup_gemm"] + kb["down_gemm"]
    n_attn = sum(1 for u in range(r.first_unit, r.first_unit + r.n_units) if u % 2 == 0)
    nb = n_attn * attn + (r.n_units - n_attn) * mlp + (kb["lm_head_argmax"] if lm_head else 0)
    # gate/up boundaries (StageRange.first_col / last_col): the gate/up columns move between
    # the two stages (weights in proportion; the act rows are counted once, by the receiver)
    gu_w = kb["gateup_gemm"] - B * d.intermediate * 2
    nb -= gu_w * r.first_col / d.intermediate
    nb += gu_w * r.last_col / d.intermediate
    # attention|o boundaries (StageRange.first_o / last_o): the shared attention unit's o GEMV
    # runs in the stage after the cut, the rest of it (norm, q/k/v, attention) in the one before
    if r.first_o:
        nb -= attn - kb["o_gemm"]
    if r.last_o:
        nb -= kb["o_gemm"]
    # q/k/v|attention boundaries (first_q / last_q): the norm and q/k/v GEMV before the cut, the
    # attention and o after it
    qkv = kb["rmsnorm"] + kb["qkv_gemm"]
    if r.first_q:
        nb -= qkv
    if r.last_q:
        nb -= attn - qkv
    return nb


# a vocab-parallel lm_head shard's fixed cost per decode step (its GEMV's ramp and tail, the key
# reduction, two launches), us; the per-row cost is the whole head's (cost table "head" less the
# final norm) / vocab.
HEAD_SHARD_FIXED_US = 7.0
FINAL_NORM_US = 5.5


def stage_base_us(d, ranges, B: int, ctx: int, head_last: bool = False):
    """Predicted decode time of each stage's layers (+ embedding on stage 0; the whole head on the last
    with head_last, else its final norm), us, and the whole head's GEMV cost: the measured cost table
    (pipeline.load_decode_costs) where one exists for the model, else bytes at 5 TB/s."""
    from inferd_amd import pipeline as P
    name = d.name.replace("-", "_")
    S = len(ranges)
    if os.path.exists(os.path.join(os.path.dirname(P.__file__), "data", f"decode_costs_{name}.json")):
        cal = P.load_decode_costs(name)
        base = [P.predicted_stage_us(r, cal, s == 0, head_last and s == S - 1) for s, r in enumerate(ranges)]
        head_us = cal["head"] - FINAL_NORM_US
    else:
        base = [range_bytes(d, r, B, ctx, head_last and s == S - 1) / 5e3 for s, r in enumerate(ranges)]
        head_us = d.vocab * d.hidden * 2 / 5e3
    if not head_last:
        base[-1] += FINAL_NORM_US
    return base, head_us


def head_shards(d, ranges, B: int, ctx: int, stage_us=None):
    """(first, rows) of the vocab-parallel lm_head per stage (pipeline.head_shard_split): the shards
    level the stages' decode times -- each stage's layer time (stage_us: measured, e.g. by the
    per-rank calibration; else stage_base_us's prediction) plus its shard's GEMV."""
    from inferd_amd.pipeline import head_shard_split
    base, head_us = stage_base_us(d, ranges, B, ctx)
    if stage_us is not None:
        base = list(stage_us)
    step = 128 if d.vocab % 128 == 0 else 16
    return head_shard_split(base, d.vocab, head_us, HEAD_SHARD_FIXED_US, step)


class _StageHead:
    """A stage's part of the vocab-parallel head, as PipelineStage._head runs it each ring
    iteration: stage 0 starts the running keys, a middle stage folds its shard in, the last stage
    finishes the argmax (a stage without rows only passes keys on / decodes them)."""

    def __init__(self, span, first: bool, last: bool, B: int, dev, normed=None, ids=None):
        self.span, self.first, self.last, self.B = span, first, last, B
        self.normed = normed if normed is not None else torch.zeros(span.normed_elems(B), dtype=torch.bfloat16,
                                                                    device=dev)
        self.keys = torch.zeros(B, dtype=torch.int64, device=dev)
        self.ids = ids if ids is not None else torch.zeros(B, dtype=torch.int32, device=dev)

    def __call__(self):
        first, rows = self.span.head_range
        if rows:
            self.span.head_shard(self.normed, self.B, keys_in=self.keys if first > 0 else None,
                                 keys_out=None if self.last else self.keys, ids=self.ids if self.last else None)
        elif self.last:
            torch.ops.inferd.argmax_combine(self.keys, 1, self.B, self.ids)


def stage_ms(d, r, first: bool, last: bool, B: int, ctx: int, dev, g, seed: int, warmup: int = 3,
             reps: int = 20, eager: bool = True, head=None, stats: dict | None = None) -> float:
    """One stage (StageRange r, with the embedding when first and final norm + lm_head + argmax
    when last) measured alone on this GPU: the span is built, B sequences are prefilled with
    ctx tokens through the real prefill path (stage 0 from random ids, later stages from random
    hidden states / records), one microbatch's decode step is captured as the stage's decode
    graph, and `reps` steps are timed with HIP events on the launch stream (after `warmup` steps),
    each stepped as the pipeline steps it: eagerly (DecodeGraph.launch_eager, the default) or as
    the graph's replay (eager=False).  head = (first row, rows): the greedy head runs
    vocab-parallel -- this stage owns those lm_head rows and runs its shard after every step
    (_StageHead), and the last stage ends with the final norm instead of the whole head.  Returns ms
    per step (stats, a dict: "head_ms" = the head part alone, timed the same way)."""
    from inferd_amd.runtime import DecodeGraph, SpanRuntime
    chunk = 2
    vh = head is not None
    hf, hr = head if vh else (0, 0)
    span = SpanRuntime(d, r.first_layer, r.n_layers, has_embed=first, has_lm_head=last and not vh,
                       kv_pages=B * ((ctx + warmup + reps) // 64 + 2) + 4, max_tokens=chunk * ctx,
                       max_seqs=B, max_positions=ctx + warmup + reps + 64, device=dev, head_first=hf, head_rows=hr,
                       final_norm_out=last and vh, **r.span_kwargs())
    span.init_synthetic(seed)
    sess = [("proj", b) for b in range(B)]
    for c in range(0, B, chunk):
        reqs = [(sid, ctx) for sid in sess[c:c + chunk]]
        if first:
            ids = torch.randint(0, d.vocab, (len(reqs) * ctx,), generator=g, dtype=torch.int32)
            span.forward(reqs, ids=ids, want_hidden=r.last_o or r.last_q, want_next_ids=last and not vh)
        else:     # (a record x | attention output at an attention|o boundary)
            n_in = buffer_elems(d, len(reqs) * ctx, 0, r.first_o, False, r.first_q)
            x = (torch.randn(n_in, generator=g) * 0.5).to(torch.bfloat16)
            span.forward(reqs, x=x, want_hidden=r.last_o or r.last_q, want_next_ids=last and not vh)
    ids = torch.zeros(B, dtype=torch.int32, device=dev) if first else None
    x = None if first else (torch.randn(B, d.hidden, generator=g) * 0.5).to(torch.bfloat16).to(dev)
    if r.first_col or r.first_o or r.first_q:
        # a record: h1 + the packed act, x + the attention output, or x + the q/k/v rows
        n_in = buffer_elems(d, B, r.first_col, r.first_o, True, r.first_q)
        x = torch.cat([x.reshape(-1), (torch.randn(n_in - B * d.hidden, generator=g) * 0.5 if (r.first_o or r.first_q)
                                       else torch.zeros(n_in - B * d.hidden)).to(torch.bfloat16).to(dev)])
    hout = None if last else torch.empty(buffer_elems(d, B, r.last_col, r.last_o, True, r.last_q),
                                         dtype=torch.bfloat16, device=dev)
    nid = torch.empty(B, dtype=torch.int32, device=dev) if last else None
    if vh and last:       # the final-normed rows; the ids come from the head shard
        hout, nid = torch.zeros(span.normed_elems(B), dtype=torch.bfloat16, device=dev), None
    graph = DecodeGraph(span, sess, warmup + reps, ids=ids, x=x, hidden_out=hout, next_ids=nid)
    step = graph.launch_eager if eager else graph.launch     # eager: the same step kernel by kernel
    go = step
    if vh:
        hd = _StageHead(span, first, last, B, dev, normed=hout if last else None)

        def go():
            step()
            hd()
    for _ in range(warmup):
        go()
    stream = torch.cuda.current_stream(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        go()
    e1.record(stream)
    e1.synchronize()
    ms = e0.elapsed_time(e1) / reps
    if vh and stats is not None:
        e0.record(stream)
        for _ in range(reps):
            hd()
        e1.record(stream)
        e1.synchronize()
        stats["head_ms"] = e0.elapsed_time(e1) / reps
    span.check_errors()
    del graph, span
    torch.cuda.synchronize(dev)
    return ms


# the per-hop hand-off latency the ring projection charges (us): the RCCL self-loop proxy of a
# record's send + receive on one GPU (tools/rccl_ring_probe.py -> the newest profiles/rccl_ring_probe_rNN.json)
# plus the record's bytes over one xGMI link (~153 GB/s per direction); without a probe file, this
HANDOFF_US_DEFAULT = 30.0
XGMI_LINK_GBS = 153.0


def handoff_us(nbytes: int) -> dict:
    """The per-hop hand-off charge for a record of nbytes: {"us", "proxy_us", "link_us", "source"}."""
    import glob
    link = nbytes / (XGMI_LINK_GBS * 1e3)
    for fn in sorted(glob.glob(os.path.join(ROOT, "profiles", "rccl_ring_probe_r*.json")), reverse=True):
        with open(fn) as f:
            pr = json.load(f)
        pts = sorted((int(k), v["gpu_us"]) for k, v in pr.get("self_loop", {}).items())
        if pts:
            b = min(pts, key=lambda p: abs(p[0] - nbytes))      # the nearest measured size
            return {"us": round(b[1] + link, 2), "proxy_us": b[1], "link_us": round(link, 2),
                    "source": os.path.basename(fn)}
    return {"us": HANDOFF_US_DEFAULT, "proxy_us": None, "link_us": round(link, 2), "source": "default"}


def ring_tick_us(c, h, vhead: bool, n_mb: int, x: float) -> float:
    """The asynchronous ring's period (pipeline.PipelineStage) for stage times c[s] (layers + head
    shard, us), head-shard parts h[s], per-hop hand-off latency x, n_mb microbatches in flight: no
    stage faster than its own work, and no microbatch faster than its lap round the ring.  Whole head
    (S hops per lap): n_mb P >= sum c + S x.  Vocab-parallel head: the ids of item i leave the last
    stage one lap behind its layers, S P after its normed rows, so (n_mb - S) P >= sum (c - h) + h[S-1]
    + S x (the layer path plus the last shard), and the normed rows reach stage 0's shard in time,
    S P >= sum (c - h) - (c[0] - h[0]) + S x."""
    S = len(c)
    P = max(c)
    if S == 1:
        return P
    L = [ci - hi for ci, hi in zip(c, h)]
    if not vhead:
        return max(P, (sum(c) + S * x) / n_mb)
    return max(P, (sum(L) + h[-1] + S * x) / (n_mb - S), (sum(L) - L[0] + S * x) / S)


def stage_projection(d, splits: dict, B: int, ctx: int, dev, seed: int, warmup: int = 10, reps: int = 60,
                     slack: int = 1) -> dict:
    """Every stage of every split measured alone on this GPU with its real role (stage_ms:
    embedding on stage 0, final norm + lm_head + argmax on the last, or -- a split whose value is
    {"ranges", "vhead": True} -- the greedy head vocab-parallel: every stage also runs its lm_head shard
    (head_shards) and the last one the final norm).  Per split: tick = the slowest stage (compute
    only); ring_tick = the asynchronous ring's period with the hand-off in it (ring_tick_us: n_mb =
    ring_microbatches(S, vhead, slack), x = handoff_us of the 128 KB-and-up records); each stage's
    fraction of the HBM roofline at the ring tick = its algorithmic bytes (+ its shard's rows x hidden x
    2) / (ring tick x 8 TB/s), bubble = 1 - sum / (S x ring tick), and the projected rate
    B / ring tick (one microbatch of B sequences completes a decode step per period)."""
    from inferd_amd.pipeline import ring_microbatches
    out = {}
    g = torch.Generator(device="cpu").manual_seed(seed + 5)
    for name, sp in splits.items():
        vhead = isinstance(sp, dict) and sp.get("vhead", False)
        ranges = sp["ranges"] if isinstance(sp, dict) else sp
        S = len(ranges)
        shards = head_shards(d, ranges, B, ctx) if vhead else None
        first_tick = None
        for attempt in range(2 if vhead else 1):
            stages, hms = [], []
            for s, r in enumerate(ranges):
                last = s == S - 1
                st = {}
                ms = stage_ms(d, r, s == 0, last, B, ctx, dev, g, seed, warmup, reps,
                              head=shards[s] if vhead else None, stats=st)
                nb = range_bytes(d, r, B, ctx + warmup + (reps + 1) / 2.0, last and not vhead)
                if vhead:
                    nb += shards[s][1] * d.hidden * 2
                hms.append(st.get("head_ms", 0.0))
                row = {"range": r.label(), "units": r.n_units, "ms": round(ms, 4), "alg_bytes": int(nb),
                       "frac_own": round(nb / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}
                if vhead:
                    row.update(head_rows=shards[s][1], head_ms=round(hms[-1], 4))
                stages.append(row)
            if vhead and attempt == 0:
                # the shards re-sized on these stages' measured layer times, as bench.py --gpus N's
                # per-rank calibration does (calibrate_shards), then every stage measured again
                first_tick = max(st["ms"] for st in stages)
                shards = head_shards(d, ranges, B, ctx, stage_us=[(st["ms"] - h) * 1e3 for st, h in zip(stages, hms)])
        tick = max(st["ms"] for st in stages)
        n_mb = ring_microbatches(S, vhead, slack)
        x = handoff_us(B * d.hidden * 2)
        rt = ring_tick_us([st["ms"] * 1e3 for st in stages], [v * 1e3 for v in hms], vhead, n_mb, x["us"]) * 1e-3
        for st in stages:
            st["frac_at_tick"] = round(st["alg_bytes"] / (rt * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
        out[name] = {"stages": stages, "tick_ms": tick, "ring_tick_ms": round(rt, 4), "microbatches": n_mb,
                     "tick_ms_model_shards": first_tick,
                     "handoff_us": x, "vocab_parallel_head": vhead,
                     "min_frac_at_tick": min(st["frac_at_tick"] for st in stages),
                     "bubble_frac": round(1 - sum(st["ms"] for st in stages) / (S * rt), 4),
                     "projected_tokens_per_s": round(B / (rt * 1e-3), 1)}
    return out


def projection_summary(proj: dict) -> dict:
    """The compact per-split view of stage_projection: {split: [ring tick ms, lowest stage's HBM
    fraction at it, bubble]} (the per-stage detail stays under stage_projection)."""
    return {k: [v["ring_tick_ms"], v["min_frac_at_tick"], v["bubble_frac"]] for k, v in proj.items()}


def projected_scaling(proj: dict, one_gpu: float) -> dict:
    """The 1/2/4/8-GPU curve the stage projection implies (compute only, no hand-off): per stage
    count the even split's (BASELINE config 3), the fastest split's and the best-balanced split's
    (highest lowest-stage HBM fraction) projected tokens/s, with efficiency against N x this
    run's one-GPU value."""
    out = {"1": {"tokens_per_s": round(one_gpu, 1)}}
    for n in (2, 4, 8):
        cand = {k: v for k, v in proj.items() if k.endswith(str(n)) and not k.startswith("config4")}
        if f"even{n}" not in cand:
            continue
        fast = max(cand, key=lambda k: cand[k]["projected_tokens_per_s"])
        bal = max(cand, key=lambda k: cand[k]["min_frac_at_tick"])
        ev = cand[f"even{n}"]["projected_tokens_per_s"]
        row = {"even": ev, "even_efficiency": round(ev / (n * one_gpu), 3)}
        if f"vhead_even{n}" in cand:      # config 3's even split with the vocab-parallel head (the bench's N > 1 default)
            v = cand[f"vhead_even{n}"]
            row["even_vocab_head"] = {"tokens_per_s": v["projected_tokens_per_s"],
                                      "efficiency": round(v["projected_tokens_per_s"] / (n * one_gpu), 3),
                                      "min_stage_frac": v["min_frac_at_tick"]}
        for tag, k in (("fastest", fast), ("balanced", bal)):
            row[tag] = {"split": k, "tokens_per_s": cand[k]["projected_tokens_per_s"],
                        "efficiency": round(cand[k]["projected_tokens_per_s"] / (n * one_gpu), 3),
                        "min_stage_frac": cand[k]["min_frac_at_tick"]}
        out[str(n)] = row
    return out


def model_costs(d, B: int = 16, ctx: int = 2048, gbs: float = 5000.0) -> dict:
    """The split search's time / byte model of a model WITHOUT a measured cost table, from its own
    dimensions (kernel_bytes at gbs GB/s, the rate the 8B decode kernels average): keyword arguments
    of pipeline.gateup_split / halves_split (the DECODE_US_8B defaults there are Qwen3-8B's)."""
    kb = kernel_bytes(d, B, ctx)
    qkv = kb["rmsnorm"] + kb["qkv_gemm"]
    attn = qkv + kb["qk_norm_rope_kv"] + kb["attention"] + kb["o_gemm"]
    mlp = kb["rmsnorm"] + kb["gateup_gemm"] + kb["down_gemm"]

    def us(b):
        return b / gbs / 1e3
    return {"costs": {"attn_half": us(attn), "mlp_half": us(mlp), "stage_norm": 5.0,
                      "head": us(kb["lm_head_argmax"]) + 10.0},
            "mb": {"attn_half": attn / 1e6, "gateup": kb["gateup_gemm"] / 1e6, "down": kb["down_gemm"] / 1e6,
                   "head": kb["lm_head_argmax"] / 1e6, "o": kb["o_gemm"] / 1e6, "qkv": qkv / 1e6},
            "gateup_us": us(kb["gateup_gemm"]), "o_us": us(kb["o_gemm"]), "q_us": us(qkv)}


def vhead_params(d, B: int = 16, ctx: int = 2048) -> dict:
    """gateup_split's vhead argument: the vocab-parallel head's per-row and fixed costs as
    head_shards prices them"""
    from inferd_amd import pipeline as P
    name = d.name.replace("-", "_")
    if os.path.exists(os.path.join(os.path.dirname(P.__file__), "data", f"decode_costs_{name}.json")):
        head_us = P.load_decode_costs(name)["head"] - FINAL_NORM_US
    else:
        head_us = d.vocab * d.hidden * 2 / 5e3
    return {"vocab": d.vocab, "row_mb": d.hidden * 2 / 1e6, "head_us": head_us, "fixed_us": HEAD_SHARD_FIXED_US,
            "norm_us": FINAL_NORM_US, "step": 128 if d.vocab % 128 == 0 else 16}


def sub_split(d, n: int, o_cuts: bool, vhead: bool = False):
    """The sub-layer splits (pipeline.gateup_split: gate/up boundaries; o_cuts: attention|o
    boundaries too) on the measured boundary-cost table where one exists for the model
    (pipeline.measured_split, inferd_amd/data/decode_costs_*.json), else on the model's own
    byte-derived time model (model_costs; ADVICE r05: not Qwen3-8B's kernel means)."""
    import os
    from inferd_amd import pipeline as P
    name = d.name.replace("-", "_")
    vh = vhead_params(d) if vhead else None
    if os.path.exists(os.path.join(os.path.dirname(P.__file__), "data", f"decode_costs_{name}.json")):
        return P.measured_split(d.layers, n, d.intermediate, o_cuts=o_cuts, name=name, vhead=vh)
    return P.gateup_split(d.layers, n, d.intermediate, o_cuts=o_cuts, vhead=vh, **model_costs(d))


# BASELINE config 4: uneven, balance.py-like splits, 36-layer models
CONFIG4_SPLITS = {3: [5, 27, 4], 4: [6, 12, 12, 6], 8: [2, 3, 5, 6, 6, 6, 5, 3]}


def projection_splits(d, B: int, ctx: int, sizes=(2, 4, 8)) -> dict:
    """The splits stage_projection measures: BASELINE config 3's even splits, the layer-granular
    byte-balanced split, the half-layer and sub-layer time-balanced splits at each stage count,
    and BASELINE config 4's uneven splits (their stage imbalance and bubble)."""
    from inferd_amd.pipeline import StageRange, halves_split, ranges_from_sizes
    out = {}
    for n in sizes:       # the greedy head vocab-parallel: config 3's even split and equal half-layer stages
        if n > d.layers or n == 1:
            continue
        out[f"vhead_even{n}"] = {"ranges": [StageRange.layers(f, k) for f, k in stage_split(d, n, B, ctx, "even")],
                                 "vhead": True}
        if (2 * d.layers) % n == 0 and (2 * d.layers // n) % 2:
            out[f"vhead_halves{n}"] = {"ranges": ranges_from_sizes([d.layers / n] * n), "vhead": True}
        # sub-layer cuts chosen for the vocab-parallel head (gateup_split(vhead=...)): stages whose
        # layer bytes run slow give them up for lm_head rows
        out[f"vhead_sublayer{n}"] = {"ranges": sub_split(d, n, True, vhead=True), "vhead": True}
    if d.layers == 36:
        for n, sp in CONFIG4_SPLITS.items():
            out[f"config4_uneven{n}"] = ranges_from_sizes(sp)
    for n in sizes:
        if n > d.layers:
            continue
        out[f"even{n}"] = [StageRange.layers(f, k) for f, k in stage_split(d, n, B, ctx, "even")]
        bal = [StageRange.layers(f, k) for f, k in stage_split(d, n, B, ctx, "balanced")]
        if bal != out[f"even{n}"]:
            out[f"balanced{n}"] = bal
        hs = halves_split(d.layers, n) if d.name == "qwen3-8b" else \
            halves_split(d.layers, n, model_costs(d, B, ctx)["costs"])
        for name, sp in (("halves", hs), ("gateup", sub_split(d, n, False)),
                         ("sublayer", sub_split(d, n, True))):
            if all(isinstance(v, dict) or sp != v for v in out.values()):
                out[f"{name}{n}"] = sp
    return out


# ------------------------------------------------------------------ CPU baseline
def _cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


def _cpu_threads() -> int:
    threads = len(os.sched_getaffinity(0))
    return min(threads, int(os.environ.get("OMP_NUM_THREADS", threads)))


def _median_time(fn, warmup: int = 2, reps: int = 5) -> float:
    """BASELINE.md's CPU measurement plan: 2 warm-up runs, then the median of 5."""
    for _ in range(warmup):
        fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    return ts[len(ts) // 2]


def cpu_baseline(d_name: str, B: int, ctx: int, seed: int, n_layers_sample: int) -> dict:
    """Oracle (`port`) decode on the host cores: a bounded sample of `n_layers_sample`
    Qwen3-8B layers, one decode step of B sequences at context ctx (KV cache pre-filled with
    random bf16 K/V: the step's cost does not depend on the cached values; the cache is
    reset to ctx tokens before every run), 2 warm-ups + median of 5, plus the final norm +
    lm_head the same way; tokens/s extrapolated to the full 36-layer model."""
    from oracle import qwen3_ref as R
    threads = _cpu_threads()
    torch.set_num_threads(threads)
    d = R.CONFIGS[d_name]
    sp = R.RefSpan(d, seed, 0, n_layers_sample - 1, False, False, torch.bfloat16, "sdpa")
    g = torch.Generator().manual_seed(0)
    kv = [((torch.randn((B, d.kv_heads, ctx, d.head_dim), generator=g)).to(torch.bfloat16),
           (torch.randn((B, d.kv_heads, ctx, d.head_dim), generator=g)).to(torch.bfloat16))
          for _ in range(n_layers_sample)]
    x = torch.randn((B, 1, d.hidden), generator=g).to(torch.bfloat16)

    def step():
        caches = []
        for k, v in kv:
            c = R.LayerCache()
            c.k, c.v = k, v
            caches.append(c)
        sp.sessions["bench"] = caches
        sp.lengths["bench"] = ctx
        sp.forward_cached("bench", x)
    t_layers = _median_time(step) / n_layers_sample
    gw = R.gen_global_weights(d, seed)
    t_head = _median_time(lambda: torch.argmax(torch.nn.functional.linear(
        R.rms_norm(x[:, -1], gw["norm"], d.eps), gw["lm_head"]), -1))
    t_step = t_layers * d.layers + t_head
    return {"value": round(B / t_step, 3), "unit": "tokens/s", "cores": threads, "kind": "port",
            "cpu": _cpu_model(),
            "sample": f"oracle/qwen3_ref.py bf16 on {threads} host threads ({_cpu_model()}): {n_layers_sample} "
                      f"Qwen3-8B layers, one decode step of B={B} at ctx={ctx} (random KV), 2 warm-ups + median of 5 "
                      f"= {t_layers * 1e3:.1f} ms/layer; lm_head {t_head * 1e3:.1f} ms; extrapolated to {d.layers} "
                      f"layers = {t_step:.2f} s/step"}


def cpu_config1(seed: int, steps: int = 16) -> dict:
    """BASELINE config 1 end to end on the host: Qwen3-0.6B as two 14-layer spans (the
    oracle's restatement of the reference's FirstStage / LastStage), greedy decode of a
    32-token prompt with the petals protocol's full recompute every step
    (send_message.py:46-60), bf16; 2 warm-up steps, then `steps` timed steps."""
    from oracle import qwen3_ref as R
    threads = _cpu_threads()
    torch.set_num_threads(threads)
    d = R.CONFIGS["qwen3-0.6b"]
    b0 = R.RefSpan(d, seed, 0, 13, True, False, torch.bfloat16, "sdpa")
    b1 = R.RefSpan(d, seed, 14, 27, False, True, torch.bfloat16, "sdpa")
    ids = torch.randint(0, d.vocab, (32,), generator=torch.Generator().manual_seed(11)).tolist()

    def one(ids):
        return int(torch.argmax(b1.forward(b0.forward(torch.tensor([ids])))[0, -1]))
    for _ in range(2):
        one(ids)
    t0 = time.perf_counter()
    for _ in range(steps):
        ids = ids + [one(ids)]
    dt = time.perf_counter() - t0
    return {"value": round(steps / dt, 3), "unit": "tokens/s", "cores": threads, "kind": "port",
            "cpu": _cpu_model(),
            "sample": f"config 1: Qwen3-0.6B, 2 spans (14+14 layers), greedy, 32-token prompt, {steps} steps of "
                      f"full recompute (T = 32..{31 + steps}), bf16, 2 warm-up steps"}


# ------------------------------------------------------------------ main
CAL_CLIP = 0.05    # calibrate_shards: measured / predicted stage time clipped to 1 -+ this


def clip_calibration(measured, predicted, clip: float = CAL_CLIP):
    """The per-rank stage times the shards are sized on: each measurement trusted within `clip` of
    the cost model (device spread 1-3 % plus the 2 % re-measurement noise fit well inside), so one
    outlier -- a rank whose timing overlapped something else -- cannot hand it the whole
    vocabulary.  Returns (times used, ranks clipped)."""
    used, clipped = [], []
    for r, (m, p) in enumerate(zip(measured, predicted)):
        ratio = m / p if (m > 0 and p > 0 and m == m) else 1.0
        c = min(max(ratio, 1.0 - clip), 1.0 + clip)
        if c != ratio:
            clipped.append(r)
        used.append(p * c)
    return used, clipped


def calibrate_shards(d, ranges, rank: int, world: int, dev, dist, args) -> dict:
    """Per-rank calibration before the pipeline is built (vocab-parallel head): every rank times
    its own stage's layers alone (stage_ms with its real role, the whole head excluded) on its own
    GPU, the times are all-gathered and the lm_head shards are sized on them (head_shards) -- so the
    split follows the GPUs it runs on, not one box's cost table (MI355X_MICROARCH.md: 1-3 % spread
    between devices on memory-bound kernels)."""
    rg = ranges[rank]
    g = torch.Generator(device="cpu").manual_seed(args.seed + 29 + rank)
    first, last = rank == 0, rank == world - 1
    zero = (0, 16) if first else (16, 16)          # a one-tile shard: the stage's layers + final norm, ~no head
    st = {}
    ms = stage_ms(d, rg, first, last, args.batch, args.ctx, dev, g, args.seed, 3, 20, head=zero, stats=st)
    t = torch.zeros(world, dtype=torch.float64, device=dev)
    t[rank] = (ms - st.get("head_ms", 0.0)) * 1e3
    if dist:
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
    us = [float(v) for v in t.cpu()]
    pred, _ = stage_base_us(d, ranges, args.batch, args.ctx)
    used, clipped = clip_calibration(us, pred)
    return {"stage_us": [round(v, 1) for v in us], "predicted_us": [round(v, 1) for v in pred],
            "used_us": [round(v, 1) for v in used], "clipped_ranks": clipped,
            "shards": head_shards(d, ranges, args.batch, args.ctx, stage_us=used)}


def pipeline_run(d, ranges, rank: int, world: int, dev, dist, args, profile: bool = True, vhead: bool = False,
                 shards=None) -> dict:
    """One pipeline measurement on this rank: build the stage of `ranges` (vhead: the greedy head
    vocab-parallel, this rank owning lm_head rows shards[rank]), prefill every microbatch (untimed),
    W warm-up and K timed decode steps (one decode step per stage per microbatch step, the
    asynchronous ring of pipeline.PipelineStage) between barriers, then the eager event-timed kernel
    profile.  Times are the max over ranks."""
    from inferd_amd import pipeline as P
    B, ctx, K, W = args.batch, args.ctx, args.steps, args.warmup
    rg = ranges[rank]
    vhead = vhead and world > 1
    if vhead and shards is None:
        shards = head_shards(d, ranges, B, ctx)
    if world > 1:
        head = (f" + lm_head rows {shards[rank][0]}..{shards[rank][0] + shards[rank][1] - 1}" if shards[rank][1]
                else "") + (" + final norm" if rank == world - 1 else "") if vhead else \
            (" + norm/lm_head" if rank == world - 1 else "")
        print(f"bench.py: rank {rank} on {dev}: layers {rg.label()} of {d.layers}"
              f"{' + embed' if rank == 0 else ''}{head}", file=sys.stderr, flush=True)
    n_mb = P.ring_microbatches(world, vhead, args.ring_slack)     # microbatches in flight
    st = P.PipelineStage(d, rank, world, rg.first_layer, rg.n_layers, device=dev, seed=args.seed,
                         n_microbatches=n_mb, batch=B, max_ctx=ctx + K + W + args.profile_steps + 64,
                         prefill_chunk=args.prefill_chunk, sharded_head=vhead,
                         head_shard=shards[rank] if vhead else (0, 0), **rg.span_kwargs())
    # ---- prefill (untimed): every microbatch's sequences get `ctx` real tokens
    g = torch.Generator().manual_seed(args.seed + 17)
    prompts = [torch.randint(0, d.vocab, (B, ctx), generator=g) for _ in range(n_mb)]
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    st.prefill(prompts)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    t_prefill = time.perf_counter() - t0
    # ---- decode: warmup + timed (one decode-graph step per stage per microbatch step, launched eagerly)
    st.prepare_decode(W + K)
    st.decode(W)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    st.decode(K)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    tick = st.tick_stats
    # ---- per-kernel HIP-event timings: the same decode kernels launched eagerly (events
    # cannot be timed inside a replayed graph); right after the timed region, same cache state
    prof = st.profile_decode(args.profile_steps) if profile else None
    t = torch.tensor([elapsed, t_prefill], dtype=torch.float64, device=dev)
    if dist:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed, t_prefill = float(t[0]), float(t[1])
    # per-stage compute per microbatch step (event-timed kernels) -> imbalance / hand-off
    stage_ms = torch.zeros(world, dtype=torch.float64, device=dev)
    if prof:
        stage_ms[rank] = sum(ms for ms, n in prof.values()) / (args.profile_steps * n_mb)
    if dist:
        dist.all_reduce(stage_ms, op=dist.ReduceOp.SUM)
    stage_ms = [float(v) for v in stage_ms.cpu()]
    return {"st": st, "elapsed": elapsed, "t_prefill": t_prefill, "tick": tick, "prof": prof, "stage_ms": stage_ms,
            "n_mb": n_mb, "shards": shards}


def main():
    args = parse()
    if args.mode == "prefill":
        return run_prefill(args)
    if args.mode == "stages":
        return run_stages(args)
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world} ranks were launched")
    # INFERD_DIST_BACKEND=gloo (rehearsal on a box with fewer GPUs than ranks: ranks share
    # devices round-robin and the stage hand-offs go through host memory); default RCCL
    backend = os.environ.get("INFERD_DIST_BACKEND", "nccl")
    dev_index = local_rank % torch.cuda.device_count() if backend == "gloo" else local_rank
    torch.cuda.set_device(dev_index)
    dev = torch.device("cuda", dev_index)
    dist = None
    if world > 1:
        import torch.distributed as dist
        # a wedged hand-off fails within 2 minutes with the process group's error instead of
        # sitting until the driver's limit
        from datetime import timedelta
        if backend == "gloo":
            dist.init_process_group("gloo", timeout=timedelta(seconds=120))
        else:
            dist.init_process_group("nccl", device_id=dev, timeout=timedelta(seconds=120))

    ranks = [{"rank": rank, "local_rank": local_rank, "device": f"cuda:{dev_index}",
              "name": torch.cuda.get_device_name(dev_index)}]
    if dist:
        gathered = [None] * world
        dist.all_gather_object(gathered, ranks[0])
        ranks = gathered
        if rank == 0:
            print(f"bench.py: {world} ranks over {dist.get_backend()} ("
                  f"{'RCCL' if dist.get_backend() == 'nccl' else dist.get_backend()}): "
                  + ", ".join(f"rank {r['rank']} -> {r['device']}" for r in ranks), file=sys.stderr, flush=True)

    from inferd_amd import pipeline as P
    from inferd_amd.runtime import MODELS

    d = MODELS[args.model]
    B, ctx, K, W = args.batch, args.ctx, args.steps, args.warmup
    if args.spans:
        ranges = P.ranges_from_sizes(args.spans.split(","))
        assert len(ranges) == world and sum(r.n_units for r in ranges) == 2 * d.layers, \
            f"--spans {args.spans}: need {world} stages, {d.layers} layers"
    elif args.split == "halves":
        ranges = P.halves_split(d.layers, world)
    elif args.split in ("gateup", "sublayer"):
        ranges = sub_split(d, world, args.split == "sublayer")
    else:
        ranges = [P.StageRange.layers(f, k) for f, k in stage_split(d, world, B, ctx, args.split)]
    vhead = world > 1 and args.head == "vocab"
    cal = None
    if vhead and not args.no_calibrate:
        cal = calibrate_shards(d, ranges, rank, world, dev, dist, args)
    run = pipeline_run(d, ranges, rank, world, dev, dist, args, profile=not args.no_profile, vhead=vhead,
                       shards=cal["shards"] if cal else None)
    st, elapsed, t_prefill, tick, prof, stage_ms = (run[k] for k in ("st", "elapsed", "t_prefill", "tick", "prof",
                                                                     "stage_ms"))
    n_mb = run["n_mb"]
    tokens = K * n_mb * B
    value = tokens / elapsed
    ms_per_step = elapsed / K * 1e3
    ctx_mean = ctx + W + K + (args.profile_steps + 1) / 2.0   # context during the profiled steps
    kb = kernel_bytes(d, B, ctx_mean)
    if run["shards"]:        # this rank's lm_head shard (vocab-parallel head) streams only its rows
        kb["lm_head_argmax"] = run["shards"][rank][1] * d.hidden * 2 + B * d.hidden * 2

    # dominant kernel class of this rank (by total event time) -> roofline
    roof, kernels = None, None
    if prof:
        kernels = {}
        for name, (ms, n) in prof.items():
            if n == 0:
                continue
            avg_us = ms / n * 1e3
            gbs = kb[name] / (avg_us * 1e-6) / 1e9
            kernels[name] = {"launches": n, "avg_us": round(avg_us, 2), "total_ms": round(ms, 3),
                             "alg_bytes": int(kb[name]), "GB/s": round(gbs, 1),
                             "frac": round(gbs / HBM_PEAK_GBS, 4)}
        dom = max(kernels, key=lambda k: kernels[k]["total_ms"])
        tr = latest_traffic("decode", f"{args.model}-decode-B{B}-ctx{ctx}")
        traffic = None if tr is None else tr.get(dom)
        roof = {"bound": "hbm", "kernel": dom, "achieved": kernels[dom]["GB/s"], "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": kernels[dom]["frac"], "traffic": traffic,
                "alg_bytes_per_launch": kernels[dom]["alg_bytes"]}

    if rank == 0:
        sb = step_bytes(d, d.layers, B, ctx_mean, True) * n_mb
        out = {
            "metric": "decode tokens/sec, Qwen3-8B layer-span pipeline",
            "value": round(value, 2),
            "unit": "tokens/s",
            "n_gpus": world,
            "steps": K,
            "warmup": W,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic token ids + counter-generated synthetic weights (no checkpoint offline)",
            "config": {"workload": f"{args.model} greedy decode, batch {B} per microbatch at {ctx} context "
                                   f"(prefilled), {n_mb} microbatch(es) in flight",
                       "global_batch": B * n_mb, "seq_len": ctx, "parallelism": f"pp{world}",
                       # layers per stage (a shared attention unit counts a quarter layer on each side)
                       "spans": [r.n_units / 2 + (r.last_col - r.first_col) / d.intermediate / 2 -
                                 0.25 * (r.first_o + r.last_o + r.first_q + r.last_q) for r in ranges],
                       "stage_ranges": [r.label() for r in ranges],
                       "head": ("vocab-parallel: lm_head rows per stage " + str([n for _, n in run["shards"]]))
                       if run["shards"] else "whole lm_head on the last stage",
                       "ring": f"asynchronous, {n_mb} microbatches" if world > 1 else None},
            "calibration": cal,
            "roofline": roof,
            "roofline_step": {"bound": "hbm", "alg_bytes_per_step": int(sb),
                              "achieved": round(sb / (ms_per_step * 1e-3) / 1e9 / world, 1),
                              "peak": HBM_PEAK_GBS, "unit": "GB/s per GPU",
                              "frac": round(sb / (ms_per_step * 1e-3) / 1e9 / world / HBM_PEAK_GBS, 4)},
            "kernels": kernels,
            "stages": None if not prof else {
                "spans": [r.label() for r in ranges],
                "compute_ms_per_microbatch": [round(v, 4) for v in stage_ms],
                "tick_ms": round(ms_per_step / n_mb, 4),
                "bubble_frac": round(1 - sum(stage_ms) / (world * max(stage_ms)), 4) if max(stage_ms) > 0 else None,
                "handoff_ms_per_tick": round(ms_per_step / n_mb - max(stage_ms), 4),
                "host_us_per_tick_rank0": tick["host_us_per_tick"],
                "exchange_us_per_tick_rank0": tick["exchange_us_per_tick"],
                "note": "compute from event-timed eager kernels (slightly above in-graph time), with the "
                        "rank's lm_head shard under a vocab-parallel head; tick = ms_per_step / microbatches; "
                        "handoff = tick - slowest stage; host_us = rank 0's host time per ring iteration "
                        "outside the hand-offs (launches, page-table advance, schedule), exchange_us = its "
                        "receive / send posts and stream waits"},
            "prefill": {"tokens": n_mb * B * ctx, "seconds": round(t_prefill, 3),
                        "tokens_per_s": round(n_mb * B * ctx / t_prefill, 1)},
            "cpu_baseline": None,
            "ranks": ranks if world > 1 else None,
            "backend": None if not dist else dist.get_backend(),
        }
        out["peaks_measured"] = measured_peaks(dev)
        out["sublayer_split"] = None
        if world == 1 and not args.no_prefill_line:
            # BASELINE config 5 in the same run (the driver's default bench call times it too)
            st.release()
            pf = prefill_line(args, 8, 2, dev)
            keep = ("metric", "value", "unit", "ms_per_step", "steps", "warmup", "config", "roofline", "kernels")
            out["prefill_config5"] = {k: pf[k] for k in keep}
            # config 5 batched (B in {1, 4}): four 8k prompts per call
            args.prefill_batch = 4
            pf = prefill_line(args, 4, 1, dev, peaks=False)
            args.prefill_batch = 1
            out["prefill_config5_b4"] = {k: pf[k] for k in keep}
        if world == 1 and not args.no_stage_projection:
            # the 2/4/8-GPU splits, every stage's decode graph timed alone on this GPU
            st.release()
            out["stage_projection"] = stage_projection(d, projection_splits(d, B, ctx), B, ctx, dev, args.seed,
                                                       slack=args.ring_slack)
            out["projected_scaling"] = projected_scaling(out["stage_projection"], value)
            out["stage_projection_summary"] = projection_summary(out["stage_projection"])
        if world == 1 and not args.no_cpu_baseline:
            st.release()
            out["cpu_baseline"] = cpu_baseline(args.model, B, ctx, args.seed, args.cpu_layers)
            out["cpu_baseline_config1"] = cpu_config1(args.seed)
    if world > 1 and not args.no_sublayer_split and args.split == "even" and not args.spans:
        # beside config 3's even split, same run: the sub-layer split chosen for the vocab-parallel
        # head (the projection's best-balanced split at 2, 4 and 8 stages) and north_star's
        # sub-layer split with the whole head on the last stage
        alts = []
        if vhead:
            alts.append(("sublayer_vocab_head", sub_split(d, world, True, vhead=True), True,
                         "sub-layer cuts chosen for the vocab-parallel head (gateup_split(vhead=...)), "
                         "shards calibrated per rank"))
        alts.append(("sublayer_split", sub_split(d, world, True), False,
                     "pipeline.sublayer_split's stages (measured cost table), the whole lm_head on the last stage"))
        for key, alt, vh, note in alts:
            st.release()
            cal2 = calibrate_shards(d, alt, rank, world, dev, dist, args) if vh and not args.no_calibrate else None
            r2 = pipeline_run(d, alt, rank, world, dev, dist, args, profile=False, vhead=vh,
                              shards=cal2["shards"] if cal2 else None)
            r2["st"].release()
            st = r2["st"]
            if rank == 0:
                out[key] = {
                    "value": round(K * r2["n_mb"] * B / r2["elapsed"], 2), "unit": "tokens/s",
                    "ms_per_step": round(r2["elapsed"] / K * 1e3, 4), "stage_ranges": [r.label() for r in alt],
                    "head_rows": [n for _, n in r2["shards"]] if r2["shards"] else None,
                    "microbatches": r2["n_mb"], "tick_ms": round(r2["elapsed"] / K * 1e3 / r2["n_mb"], 4),
                    "exchange_us_per_tick_rank0": r2["tick"]["exchange_us_per_tick"],
                    "note": note + "; `value` above is BASELINE config 3's even split"}
    if rank == 0:
        # the driver keeps the tail of stdout: the compact results go last
        for k in ("stage_projection_summary", "projected_scaling", "sublayer_split", "sublayer_vocab_head",
                  "prefill_config5", "prefill_config5_b4"):
            if k in out:
                v = out.pop(k)
                if k.startswith("prefill_config5") and v is not None:
                    out.setdefault("prefill_kernels", {})[k] = v.pop("kernels", None)
                out[k] = v
        print(json.dumps(out), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
