"""A/B of lab builds of the span library (tools/build_probes.sh -> tools/probe_libs/) on the
prefill attention (inferd_attention through each library's C-ABI, all loaded in ONE process,
variants interleaved round by round), with each variant's error against an fp32 causal
attention of the same bf16 inputs on a few heads.

Qwen3-32B dims (H=64, KV=8), B x T causal prompt (BASELINE config 5).
usage: python tools/attn_ab.py name=path.so [name=path.so ...] [--T 8192] [--rounds 7]
"""
import argparse
import ctypes as C
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from inferd_amd import _lib  # noqa: E402
from inferd_amd.runtime import KvTable  # noqa: E402
from kv_layout import read_kv  # noqa: E402


def load(path):
    lib = C.CDLL(path)
    for name in ("inferd_attention", "inferd_attention_workspace_bytes", "inferd_last_error"):
        res, args = _lib.SIGNATURES[name]
        getattr(lib, name).restype = res
        getattr(lib, name).argtypes = args
    return lib


def main():
    p = argparse.ArgumentParser()
    p.add_argument("libs", nargs="+")
    p.add_argument("--T", type=int, default=8192)
    p.add_argument("--B", type=int, default=1)
    p.add_argument("--rounds", type=int, default=7)
    p.add_argument("--reps", type=int, default=3)
    p.add_argument("--heads", default="0,21,42,63")
    p.add_argument("--qscale", type=float, default=1.2, help="q ~ N(0, qscale^2): larger scores, more rescales")
    args = p.parse_args()
    libs = [(s.split("=", 1)[0], load(s.split("=", 1)[1])) for s in args.libs]
    dev = torch.device("cuda", 0)
    H, KV, B, T = 64, 8, args.B, args.T
    pages_per = (T + 63) // 64
    table = KvTable(B * pages_per)
    for b in range(B):
        table.reserve(b, T)
    bd = table.build_batch([(b, T) for b in range(B)], dev)
    batch = _lib.batch_struct(bd.words, bd.shape)
    pool_pages = (B * pages_per + 15) // 16 * 16
    g = torch.Generator(device=dev).manual_seed(5)
    kv = (torch.randn(pool_pages * 2 * KV * 64 * 128, device=dev, generator=g)).to(torch.bfloat16)
    q = (torch.randn(B * T, H, 128, device=dev, generator=g) * args.qscale).to(torch.bfloat16)
    out = torch.empty(B * T, H * 128, dtype=torch.bfloat16, device=dev)
    st = _lib.stream_ptr()
    flops = B * 4.0 * H * 128 * T * (T + 1) / 2
    # fp32 reference of sequence 0 on a few heads
    K, V = read_kv(kv, KV, table.pages(0), T)
    K, V = K.to(dev).float(), V.to(dev).float()
    heads = [int(h) for h in args.heads.split(",")]
    mask = torch.ones(T, T, dtype=torch.bool, device=dev).tril()
    refs = {}
    for h in heads:
        s = (q[:T, h].float() @ K[h // (H // KV)].t()) * 128 ** -0.5
        refs[h] = torch.softmax(s.masked_fill(~mask, float("-inf")), -1) @ V[h // (H // KV)]
    del mask
    times = {n: [] for n, _ in libs}
    errs = {}
    first = None
    for rnd in range(args.rounds):
        for n, L in libs:
            def call():
                rc = L.inferd_attention(q.data_ptr(), kv.data_ptr(), batch, H, KV, out.data_ptr(), None, 0, st)
                assert rc == 0, L.inferd_last_error()
            call()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.reps):
                call()
            e1.record()
            torch.cuda.synchronize()
            times[n].append(e0.elapsed_time(e1) / args.reps)
            if rnd == 0:
                o = out.view(B * T, H, 128)
                e = [((o[:T, h].float() - refs[h]).pow(2).mean() / refs[h].pow(2).mean()).sqrt().item() for h in heads]
                mx = [(o[:T, h].float() - refs[h]).abs().max().item() for h in heads]
                errs[n] = (sum(e) / len(e), max(mx))
                if first is None:
                    first = out.clone()
                else:
                    print(f"{n}: output bit-identical to {libs[0][0]}: {torch.equal(out, first)}", flush=True)
    for n, _ in libs:
        t = sorted(times[n])
        med = t[len(t) // 2]
        print(f"{n:>10}: {med * 1e3:8.1f} us (min {t[0] * 1e3:8.1f})  {flops / med / 1e9:7.1f} TF/s  "
              f"vs fp32: rms rel {errs[n][0]:.3e}  max abs {errs[n][1]:.3e}", flush=True)


if __name__ == "__main__":
    main()
