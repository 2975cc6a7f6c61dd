"""A/B of lab builds of the span library on the config-5 prefill (Qwen3-32B layers, B x 8k
tokens): every library (tools/build_probes.sh -> tools/probe_libs/) is loaded in ONE process
through its C-ABI, each creates its own span with the same synthetic weights, and the
variants run interleaved round by round (cdna_hip_programming.md §5.4 rule 24).  Per round
and library: one profiled forward (per-kernel-class times from inferd_span_profile_*) and the
output's difference from the first library's.

usage: python tools/span_ab.py name=path.so [name=path.so ...] [--layers 2] [--T 8192] [--rounds 5]
("span" = the product library inferd_amd/libinferd_span.so.)"""
import argparse
import ctypes as C
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from inferd_amd import _lib  # noqa: E402
from inferd_amd.runtime import MODELS, KvTable  # noqa: E402

CLASSES = ("norm", "qkv", "rope", "attn", "o", "gateup", "down", "lmhead")


def load(path):
    lib = C.CDLL(path)
    for name in ("inferd_span_create", "inferd_span_destroy", "inferd_span_init_synthetic", "inferd_span_forward",
                 "inferd_span_profile_start", "inferd_span_profile_stop", "inferd_last_error"):
        res, a = _lib.SIGNATURES[name]
        getattr(lib, name).restype = res
        getattr(lib, name).argtypes = a
    return lib


def check(lib, rc):
    if rc != 0:
        raise RuntimeError(lib.inferd_last_error().decode())


def main():
    p = argparse.ArgumentParser()
    p.add_argument("libs", nargs="+")
    p.add_argument("--layers", type=int, default=2)
    p.add_argument("--T", type=int, default=8192)
    p.add_argument("--B", type=int, default=1)
    p.add_argument("--rounds", type=int, default=5)
    p.add_argument("--seed", type=int, default=1234)
    args = p.parse_args()
    d = MODELS["qwen3-32b"]
    dev = torch.device("cuda", 0)
    B, T, L = args.B, args.T, args.layers
    pages = B * (T // 64 + 2) + 4
    st = _lib.stream_ptr()
    table = KvTable(pages)
    for b in range(B):
        table.reserve(b, T)
    bd = table.build_batch([(b, T) for b in range(B)], dev)
    batch = _lib.batch_struct(bd.words, bd.shape)
    cfg = _lib.SpanConfig(hidden=d.hidden, intermediate=d.intermediate, heads=d.heads, kv_heads=d.kv_heads,
                          head_dim=d.head_dim, vocab=d.vocab, first_layer=8, n_layers=L, has_embed=0, has_lm_head=0,
                          rms_eps=d.eps, rope_theta=d.rope_theta, max_positions=T + 64, kv_pages=pages,
                          max_tokens=B * T, max_seqs=max(B, 1))
    spans = []
    for spec in args.libs:
        name, path = spec.split("=", 1)
        if path == "span":
            path = os.path.join(ROOT, "inferd_amd", "libinferd_span.so")
        lib = load(path)
        h = C.c_void_p()
        check(lib, lib.inferd_span_create(C.byref(cfg), C.byref(h)))
        check(lib, lib.inferd_span_init_synthetic(h, args.seed, st))
        spans.append((name, lib, h))
    x = (torch.randn(B * T, d.hidden, device=dev) * 0.5).to(torch.bfloat16)
    outs = {n: torch.empty_like(x) for n, _, _ in spans}
    times = {n: {c: [] for c in CLASSES + ("total",)} for n, _, _ in spans}
    tot = (C.c_double * 8)()
    cnt = (C.c_int32 * 8)()
    for rnd in range(args.rounds + 1):
        for name, lib, h in spans:
            check(lib, lib.inferd_span_profile_start(h, 1 << 12))
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            check(lib, lib.inferd_span_forward(h, C.byref(batch), None, x.data_ptr(), outs[name].data_ptr(), None,
                                               None, None, st))
            e1.record()
            torch.cuda.synchronize()
            check(lib, lib.inferd_span_profile_stop(h, tot, cnt, 8))
            if rnd == 0:
                continue  # warm-up round
            times[name]["total"].append(e0.elapsed_time(e1))
            for i, c in enumerate(CLASSES):
                if cnt[i]:
                    times[name][c].append(tot[i] / cnt[i])
        print(f"round {rnd} done", flush=True)
    base = spans[0][0]
    for name, _, _ in spans:
        parts = []
        for c in CLASSES + ("total",):
            t = sorted(times[name][c])
            if t:
                parts.append(f"{c} {t[len(t) // 2] * 1e3:8.1f}")
        diff = (outs[name].float() - outs[base].float()).abs().max().item()
        print(f"{name:8s} us per launch (median): " + " | ".join(parts) + f" | maxdiff vs {base} {diff:.3g}",
              flush=True)
    for name, lib, h in spans:
        lib.inferd_span_destroy(h)


if __name__ == "__main__":
    main()
