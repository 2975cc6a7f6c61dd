"""Lab: where the time of a tail-split prefill GEMM goes (Qwen3-32B o / down: 640 tiles = 2.5
rounds of 256 CUs).  Needs a library built with the workgroup stamps:
    tools/build_probes.sh gemm.hip st='-DW4_STAMP=1' with tools/archive/gemm_stamps_r04.hip (the
    round-4 kernels with the W4_STAMP hooks) copied over inferd_amd/csrc/gemm.hip in a scratch
    checkout: the product gemm.hip carries no lab hooks
    python tools/w4_stamps.py tools/probe_libs/libinferd_span_st.so [--shape o|down]
Runs inferd_gemm (EPI_RESID, the op API's tail split) a few times, then reads the last call's
per-workgroup stamps (100 MHz real-time clock): start, end of the K-loop, after the tail-split
publish / combine, end; prints per-phase timelines relative to the first workgroup's start."""
import argparse
import ctypes as C
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from inferd_amd import _lib  # noqa: E402

SHAPES = {"o": (5120, 8192), "down": (5120, 25600)}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("lib")
    p.add_argument("--shape", default="o")
    p.add_argument("--m", type=int, default=8192)
    args = p.parse_args()
    L = C.CDLL(args.lib)
    for name in ("inferd_gemm", "inferd_pack_weight", "inferd_last_error"):
        res, a = _lib.SIGNATURES[name]
        getattr(L, name).restype = res
        getattr(L, name).argtypes = a
    L.inferd_lab_w4_stamps.restype = C.c_int
    L.inferd_lab_w4_stamps.argtypes = [C.c_void_p, C.c_int]
    dev = torch.device("cuda", 0)
    N, K = SHAPES[args.shape]
    M = args.m
    st = _lib.stream_ptr()
    a = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
    w = ((torch.rand(N, K, device=dev) * 2 - 1) * 0.05).to(torch.bfloat16)
    wp = torch.empty_like(w)
    assert L.inferd_pack_weight(w.data_ptr(), N, K, wp.data_ptr(), st) == 0
    c = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    r = (torch.rand(M, N, device=dev) * 2 - 1).to(torch.bfloat16)
    for _ in range(4):
        assert L.inferd_gemm(a.data_ptr(), wp.data_ptr(), c.data_ptr(), r.data_ptr(), M, N, K, 1, st) == 0
    torch.cuda.synchronize()
    n = 4096
    buf = np.zeros(n * 6, dtype=np.uint64)
    assert L.inferd_lab_w4_stamps(buf.ctypes.data, n) == 0
    s = buf.reshape(n, 6).astype(np.int64)
    used = s[:, 0] > 0
    s = s[used]
    t0 = s[:, 0].min()
    us = (s[:, :4] - t0) / 100.0  # 100 MHz -> µs
    g = len(s)
    xcc = s[:, 4] & 0xF
    hw = s[:, 5]
    cu = ((hw >> 8) & 0xF) | (((hw >> 13) & 0x7) << 4) | (((hw >> 12) & 1) << 7)
    print(f"{args.shape}: M={M} N={N} K={K}, {g} workgroups, kernel span {us[:, 3].max():.1f} us")
    order = np.argsort(us[:, 0], kind="stable")
    # workgroups in dispatch order, in chunks of 256 (one per CU per round)
    for r0 in range(0, g, 256):
        idx = np.arange(r0, min(r0 + 256, g))
        st_, kl, sp, en = us[idx, 0], us[idx, 1], us[idx, 2], us[idx, 3]
        print(f" wg {r0:4d}-{idx[-1]:4d}: start {st_.min():7.1f}..{st_.max():7.1f}  k-loop end {kl.min():7.1f}.."
              f"{kl.max():7.1f} (dur med {np.median(kl - st_):6.1f})  split {np.median(sp - kl):5.1f}  "
              f"end {en.min():7.1f}..{en.max():7.1f}")
    # per CU: number of workgroups and busy time
    key = xcc * 256 + cu
    ks, cnt = np.unique(key, return_counts=True)
    print(f" distinct (xcc, cu): {len(ks)}; workgroups per CU min/med/max {cnt.min()}/{int(np.median(cnt))}/{cnt.max()}")
    gaps = []
    for k in ks:
        m = np.where(key == k)[0]
        m = m[np.argsort(us[m, 0])]
        for i in range(1, len(m)):
            gaps.append(us[m[i], 0] - us[m[i - 1], 3])
    if gaps:
        gaps = np.array(gaps)
        print(f" gap between a CU's consecutive workgroups: med {np.median(gaps):.2f} us, max {gaps.max():.2f} us")
    late = order[-8:]
    for i in late:
        print(f"  late wg {i}: xcc {xcc[i]} cu {cu[i]} start {us[i, 0]:.1f} kloop {us[i, 1]:.1f} split {us[i, 2]:.1f} end {us[i, 3]:.1f}")


if __name__ == "__main__":
    main()
