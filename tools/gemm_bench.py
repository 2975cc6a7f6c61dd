"""Prefill GEMM timing on the GPU box: the span library's GEMM (inferd_gemm; a lab build is
selected with INFERD_LIB, see tools/build_probes.sh) on the Qwen3-32B projection shapes
(BASELINE config 5, M = 8192 prompt rows), interleaved rounds in ONE process
(cdna_hip_programming.md §5.4 rule 24), uniform random operands (rule 25).

usage: python tools/gemm_bench.py [--m 8192] [--rounds 5] [--variants span,torch,name=lib.so,...]
("torch" times torch.matmul = hipBLASLt on the same operands, no epilogue: the library ceiling;
name=lib.so loads another build of the span library -- e.g. a tools/probe_libs/ build -- so
A/B variants run interleaved in one process on one box.)
"""
import argparse
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from inferd_amd import _lib  # noqa: E402

SHAPES = {  # name: (N_out, K, epilogue)
    "qkv": (10240, 5120, 0),
    "o": (5120, 8192, 1),
    "gateup": (25600, 5120, 2),
    "down": (5120, 25600, 1),
    # K sweep on the qkv shape: time(K) = per-tile overhead + K-proportional main loop
    "qkv_k1": (10240, 1024, 0),
    "qkv_k2": (10240, 2048, 0),
    # the 2.5-round o/down grids against whole-round neighbours (512 tiles = 2 rounds, 768 = 3)
    "o_n4096": (4096, 8192, 1),
    "o_n6144": (6144, 8192, 1),
    "down_n4096": (4096, 25600, 1),
    "down_n6144": (6144, 25600, 1),
}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--m", type=int, default=8192)
    p.add_argument("--rounds", type=int, default=5)
    p.add_argument("--reps", type=int, default=3)
    p.add_argument("--variants", default="span")
    p.add_argument("--shapes", default=",".join(SHAPES))
    args = p.parse_args()
    L = _lib.load()
    libs = {"span": L}
    for v in args.variants.split(","):
        if "=" in v:
            lab = ctypes.CDLL(v.split("=", 1)[1])
            for name in ("inferd_gemm", "inferd_last_error"):
                res, a = _lib.SIGNATURES[name]
                getattr(lab, name).restype = res
                getattr(lab, name).argtypes = a
            libs[v.split("=", 1)[0]] = lab
    dev = torch.device("cuda", 0)
    M = args.m
    st = _lib.stream_ptr()
    bufs = {}
    for name in args.shapes.split(","):
        n, k, epi = SHAPES[name]
        rows = 2 * n if epi == 2 else n
        a = (torch.rand(M, k, device=dev) * 2 - 1).to(torch.bfloat16)
        w = ((torch.rand(rows, k, device=dev) * 2 - 1) * 0.05).to(torch.bfloat16)
        wp = torch.empty_like(w)
        _lib.check(L.inferd_pack_weight(w.data_ptr(), rows, k, wp.data_ptr(), st))
        if "torch" not in args.variants.split(","):
            w = None
        c = torch.empty(M, n, dtype=torch.bfloat16, device=dev)
        r = (torch.rand(M, n, device=dev) * 2 - 1).to(torch.bfloat16) if epi == 1 else None
        bufs[name] = (a, wp, c, r, n, k, epi, w)
    torch.cuda.synchronize()
    variants = [v.split("=", 1)[0] for v in args.variants.split(",")]
    times = {(s, v): [] for s in bufs for v in variants}
    outs = {}
    for rnd in range(args.rounds):
        for name, (a, wp, c, r, n, k, epi, w) in bufs.items():
            for v in variants:
                if v == "torch":  # hipBLASLt through torch.matmul: plain GEMM, no epilogue (ceiling probe)
                    call = lambda: torch.matmul(a, w.t())  # noqa: E731
                else:
                    LL = libs[v]
                    call = lambda: _lib.check(LL.inferd_gemm(a.data_ptr(), wp.data_ptr(), c.data_ptr(),  # noqa: E731
                                                             None if r is None else r.data_ptr(), M, n, k, epi, st))
                call()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(args.reps):
                    call()
                e1.record()
                torch.cuda.synchronize()
                times[(name, v)].append(e0.elapsed_time(e1) / args.reps)
                if rnd == 0 and v != "torch":
                    outs[(name, v)] = c.clone()
        print(f"round {rnd} done", flush=True)
    for name, (a, wp, c, r, n, k, epi, w) in bufs.items():
        fl = 2.0 * M * n * k * (2 if epi == 2 else 1)
        line = [f"{name:7s} M={M} N={n} K={k}"]
        for v in variants:
            t = sorted(times[(name, v)])
            med = t[len(t) // 2]
            line.append(f"{v}: {med * 1e3:8.1f} us {fl / med / 1e9:7.1f} TF/s (min {fl / t[0] / 1e9:7.1f})")
        base = outs[(name, variants[0])]
        for v in variants[1:]:
            if v == "torch":
                continue
            d = (outs[(name, v)].float() - base.float()).abs().max().item()
            line.append(f"maxdiff[{v}]={d:.3g}")
        print(" | ".join(line), flush=True)


if __name__ == "__main__":
    main()
