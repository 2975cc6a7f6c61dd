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


def stage_ms(d, r, first: bool, last: bool, B: int, ctx: int, dev, g, seed: int, warmup: int = 3,
             reps: int = 20, eager: bool = True) -> float:
    """One stage (StageRange r, with the embedding when first and final norm + lm_head + argmax
    when last) measured alone on this GPU: the span is built, B sequences are prefilled with
    ctx tokens through the real prefill path (stage 0 from random ids, later stages from random
    hidden states / records), one microbatch's decode step is captured as the stage's decode
    graph, and `reps` steps are timed with HIP events on the launch stream (after `warmup` steps),
    each stepped as the pipeline steps it: eagerly (DecodeGraph.launch_eager, the default) or as
    the graph's replay (eager=False).  Returns ms per step."""
    from inferd_amd.runtime import DecodeGraph, SpanRuntime
    chunk = 2
    span = SpanRuntime(d, r.first_layer, r.n_layers, has_embed=first, has_lm_head=last,
                       kv_pages=B * ((ctx + warmup + reps) // 64 + 2) + 4, max_tokens=chunk * ctx,
                       max_seqs=B, max_positions=ctx + warmup + reps + 64, device=dev, **r.span_kwargs())
    span.init_synthetic(seed)
    sess = [("proj", b) for b in range(B)]
    for c in range(0, B, chunk):
        reqs = [(sid, ctx) for sid in sess[c:c + chunk]]
        if first:
            ids = torch.randint(0, d.vocab, (len(reqs) * ctx,), generator=g, dtype=torch.int32)
            span.forward(reqs, ids=ids, want_hidden=False, want_next_ids=last)
        else:     # (a record x | attention output at an attention|o boundary)
            n_in = buffer_elems(d, len(reqs) * ctx, 0, r.first_o, False, r.first_q)
            x = (torch.randn(n_in, generator=g) * 0.5).to(torch.bfloat16)
            span.forward(reqs, x=x, want_hidden=r.last_o or r.last_q, want_next_ids=last)
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
    graph = DecodeGraph(span, sess, warmup + reps, ids=ids, x=x, hidden_out=hout, next_ids=nid)
    go = graph.launch_eager if eager else graph.launch     # eager: the same step kernel by kernel
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
    span.check_errors()
    del graph, span
    torch.cuda.synchronize(dev)
    return ms


def stage_projection(d, splits: dict, B: int, ctx: int, dev, seed: int, warmup: int = 3, reps: int = 20) -> dict:
    """Every stage of every split measured alone on this GPU with its real role (stage_ms:
    embedding on stage 0, final norm + lm_head + argmax on the last).  The lockstep pipeline
    (pipeline.py) ticks at its slowest stage, so per split: tick = max stage ms, each stage's
    fraction of the HBM roofline at that tick = its algorithmic bytes / (tick x 8 TB/s) (SURVEY
    §8(d)), bubble = 1 - sum / (S x tick), and the compute-only projected rate B / tick (one
    microbatch of B sequences completes a decode step per tick: S microbatches in flight, each a
    token every S ticks; the
    xGMI hand-off excluded)."""
    out = {}
    g = torch.Generator(device="cpu").manual_seed(seed + 5)
    for name, ranges in splits.items():
        S = len(ranges)
        stages = []
        for s, r in enumerate(ranges):
            last = s == S - 1
            ms = stage_ms(d, r, s == 0, last, B, ctx, dev, g, seed, warmup, reps)
            nb = range_bytes(d, r, B, ctx + warmup + (reps + 1) / 2.0, last)
            stages.append({"range": r.label(), "units": r.n_units, "ms": round(ms, 4), "alg_bytes": int(nb),
                           "frac_own": round(nb / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)})
        tick = max(st["ms"] for st in stages)
        for st in stages:
            st["frac_at_tick"] = round(st["alg_bytes"] / (tick * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
        out[name] = {"stages": stages, "tick_ms": tick,
                     "min_frac_at_tick": min(st["frac_at_tick"] for st in stages),
                     "bubble_frac": round(1 - sum(st["ms"] for st in stages) / (S * tick), 4),
                     "projected_tokens_per_s": round(B / (tick * 1e-3), 1)}
    return out


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
        for tag, k in (("fastest", fast), ("balanced", bal)):
            row[tag] = {"split": k, "tokens_per_s": cand[k]["projected_tokens_per_s"],
                        "efficiency": round(cand[k]["projected_tokens_per_s"] / (n * one_gpu), 3),
                        "min_stage_frac": cand[k]["min_frac_at_tick"]}
        out[str(n)] = row
    return out


def sub_split(d, n: int, o_cuts: bool):
    """The sub-layer splits (pipeline.gateup_split: gate/up boundaries; o_cuts: attention|o
    boundaries too) on the measured boundary-cost table where one exists for the model
    (pipeline.measured_split, inferd_amd/data/decode_costs_*.json), else on the kernel-mean model."""
    import os
    from inferd_amd import pipeline as P
    name = d.name.replace("-", "_")
    if os.path.exists(os.path.join(os.path.dirname(P.__file__), "data", f"decode_costs_{name}.json")):
        return P.measured_split(d.layers, n, d.intermediate, o_cuts=o_cuts, name=name)
    return P.gateup_split(d.layers, n, d.intermediate, o_cuts=o_cuts)


# BASELINE config 4: uneven, balance.py-like splits, 36-layer models
CONFIG4_SPLITS = {3: [5, 27, 4], 4: [6, 12, 12, 6], 8: [2, 3, 5, 6, 6, 6, 5, 3]}


def projection_splits(d, B: int, ctx: int, sizes=(2, 4, 8)) -> dict:
    """The splits stage_projection measures: BASELINE config 3's even splits, the layer-granular
    byte-balanced split, the half-layer and sub-layer time-balanced splits at each stage count,
    and BASELINE config 4's uneven splits (their stage imbalance and bubble)."""
    from inferd_amd.pipeline import StageRange, halves_split, ranges_from_sizes
    out = {}
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
        for name, sp in (("halves", halves_split(d.layers, n)), ("gateup", sub_split(d, n, False)),
                         ("sublayer", sub_split(d, n, True))):
            if all(sp != v for v in out.values()):
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
def pipeline_run(d, ranges, rank: int, world: int, dev, dist, args, profile: bool = True) -> dict:
    """One pipeline measurement on this rank: build the stage of `ranges`, prefill every
    microbatch (untimed), W warm-up and K timed decode steps (one decode-graph step per stage
    per microbatch step) between barriers, then the eager event-timed kernel profile.  Times are
    the max over ranks."""
    from inferd_amd import pipeline as P
    B, ctx, K, W = args.batch, args.ctx, args.steps, args.warmup
    rg = ranges[rank]
    if world > 1:
        print(f"bench.py: rank {rank} on {dev}: layers {rg.label()} of {d.layers}"
              f"{' + embed' if rank == 0 else ''}{' + norm/lm_head' if rank == world - 1 else ''}",
              file=sys.stderr, flush=True)
    n_mb = world                                   # microbatches in flight
    st = P.PipelineStage(d, rank, world, rg.first_layer, rg.n_layers, device=dev, seed=args.seed,
                         n_microbatches=n_mb, batch=B, max_ctx=ctx + K + W + args.profile_steps + 64,
                         prefill_chunk=args.prefill_chunk, **rg.span_kwargs())
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
    return {"st": st, "elapsed": elapsed, "t_prefill": t_prefill, "tick": tick, "prof": prof, "stage_ms": stage_ms}


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
    run = pipeline_run(d, ranges, rank, world, dev, dist, args, profile=not args.no_profile)
    st, elapsed, t_prefill, tick, prof, stage_ms = (run[k] for k in ("st", "elapsed", "t_prefill", "tick", "prof",
                                                                     "stage_ms"))
    n_mb = world
    tokens = K * n_mb * B
    value = tokens / elapsed
    ms_per_step = elapsed / K * 1e3
    ctx_mean = ctx + W + K + (args.profile_steps + 1) / 2.0   # context during the profiled steps
    kb = kernel_bytes(d, B, ctx_mean)

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
                       "stage_ranges": [r.label() for r in ranges]},
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
                "note": "compute from event-timed eager kernels (slightly above in-graph time); tick = "
                        "ms_per_step / microbatches; handoff = tick - slowest stage; host_us = rank 0's host "
                        "time per tick outside the stage exchange (graph launch, page-table advance, "
                        "schedule), exchange_us = its batch_isend_irecv + wait"},
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
            out["stage_projection"] = stage_projection(d, projection_splits(d, B, ctx), B, ctx, dev, args.seed)
            out["projected_scaling"] = projected_scaling(out["stage_projection"], value)
        if world == 1 and not args.no_cpu_baseline:
            st.release()
            out["cpu_baseline"] = cpu_baseline(args.model, B, ctx, args.seed, args.cpu_layers)
            out["cpu_baseline_config1"] = cpu_config1(args.seed)
    if world > 1 and not args.no_sublayer_split and args.split == "even" and not args.spans:
        # north_star's balanced pipeline beside config 3's even split, same run: the sub-layer split
        # (every stage >= 60 % of the HBM roofline at the tick by the stage projection)
        st.release()
        alt = sub_split(d, world, True)
        r2 = pipeline_run(d, alt, rank, world, dev, dist, args, profile=False)
        r2["st"].release()
        if rank == 0:
            out["sublayer_split"] = {
                "value": round(K * world * B / r2["elapsed"], 2), "unit": "tokens/s",
                "ms_per_step": round(r2["elapsed"] / K * 1e3, 4), "stage_ranges": [r.label() for r in alt],
                "tick_ms": round(r2["elapsed"] / K * 1e3 / world, 4),
                "exchange_us_per_tick_rank0": r2["tick"]["exchange_us_per_tick"],
                "note": "the same workload on pipeline.sublayer_split's stages (measured cost table); "
                        "`value` above is BASELINE config 3's even split"}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
