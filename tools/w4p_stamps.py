"""Lab: per-tile timeline of the persistent q/k/v GEMM with its fused epilogue (Qwen3-32B, 8k
prompt: 1280 tiles of 256 x 256 = 5 per CU).  Needs a stamp build:
    tools/build_probes.sh gemm.hip st='-DW4_STAMP=1' with tools/archive/gemm_stamps_r04.hip (the
    round-4 kernels with the W4_STAMP hooks) copied over inferd_amd/csrc/gemm.hip in a scratch
    checkout: the product gemm.hip carries no lab hooks
    python tools/w4p_stamps.py tools/probe_libs/libinferd_span_st.so
Runs one 1-layer span prefill through that library's C-ABI, then reads the q/k/v GEMM's stamps
(100 MHz clock; per unit and wave: start with step 0 landed, end of K-loop, end of epilogue)
and prints K-loop and epilogue durations by head kind (q, k, v) and the gaps between units."""
import ctypes as C
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
from inferd_amd import _lib  # noqa: E402
from inferd_amd.runtime import MODELS, KvTable  # noqa: E402
from span_ab import check, load  # noqa: E402


def main():
    lib = load(sys.argv[1])
    lib.inferd_lab_w4p_stamps.restype = C.c_int
    lib.inferd_lab_w4p_stamps.argtypes = [C.c_void_p, C.c_int]
    d = MODELS["qwen3-32b"]
    dev = torch.device("cuda", 0)
    T = 8192
    pages = T // 64 + 6
    st = _lib.stream_ptr()
    table = KvTable(pages)
    table.reserve(0, T)
    bd = table.build_batch([(0, T)], dev)
    batch = _lib.batch_struct(bd.words, bd.shape)
    cfg = _lib.SpanConfig(hidden=d.hidden, intermediate=d.intermediate, heads=d.heads, kv_heads=d.kv_heads,
                          head_dim=d.head_dim, vocab=d.vocab, first_layer=8, n_layers=1, has_embed=0, has_lm_head=0,
                          rms_eps=d.eps, rope_theta=d.rope_theta, max_positions=T + 64, kv_pages=pages,
                          max_tokens=T, max_seqs=1)
    h = C.c_void_p()
    check(lib, lib.inferd_span_create(C.byref(cfg), C.byref(h)))
    check(lib, lib.inferd_span_init_synthetic(h, 1234, st))
    x = (torch.randn(T, d.hidden, device=dev) * 0.5).to(torch.bfloat16)
    out = torch.empty_like(x)
    for _ in range(3):
        check(lib, lib.inferd_span_forward(h, C.byref(batch), None, x.data_ptr(), out.data_ptr(), None, None, None, st))
    torch.cuda.synchronize()
    n_units = (T // 256) * ((d.heads + 2 * d.kv_heads) * 128 // 256)
    buf = np.zeros(2048 * 16, dtype=np.uint64)
    check(lib, lib.inferd_lab_w4p_stamps(buf.ctypes.data, 2048))
    s = buf.reshape(2048, 4, 4)[:n_units].astype(np.int64)
    t0 = s[:, :, 0][s[:, :, 0] > 0].min()
    us = (s - t0) / 100.0
    grid_n = (d.heads + 2 * d.kv_heads) * 128 // 256
    print(f"q/k/v GEMM: {n_units} units, span {us[:, :, 2].max():.1f} us")
    # unit -> tile: XCD-contiguous order with GM = 8 groups (gemm.hip tile_order_v); the head of
    # wave w is 2 * bn + (w & 1), recovered here from the unit's own tile mapping
    nwg = n_units
    kinds = {"q": [], "k": [], "v": []}
    for v in range(n_units):
        xcd, q_, r_ = v & 7, nwg >> 3, nwg & 7
        wg = (xcd * (q_ + 1) if xcd < r_ else r_ * (q_ + 1) + (xcd - r_) * q_) + (v >> 3)
        group = wg // (8 * grid_n)
        gsz = min(T // 256 - group * 8, 8)
        inn = wg - group * 8 * grid_n
        bn = inn // gsz
        for w in range(4):
            hd = 2 * bn + (w & 1)
            kind = "q" if hd < d.heads else ("k" if hd < d.heads + d.kv_heads else "v")
            kl = us[v, w, 1] - us[v, w, 0]
            ep = us[v, w, 2] - us[v, w, 1]
            kinds[kind].append((kl, ep))
    for k, l in kinds.items():
        a = np.array(l)
        print(f" {k}: {len(a)} wave-units  K-loop med {np.median(a[:, 0]):6.1f} us  epilogue med {np.median(a[:, 1]):6.2f} "
              f"p90 {np.percentile(a[:, 1], 90):6.2f} max {a[:, 1].max():6.2f} us")
    # per CU (units v, v + 256, ...): gap between a unit's epilogue end (max over waves) and the
    # next unit's start (min over waves)
    g = []
    for v in range(n_units - 256):
        g.append(us[v + 256, :, 0].min() - us[v, :, 2].max())
    g = np.array(g)
    print(f" unit-to-unit gap (step 0 of the next unit landed after this unit's last epilogue): med {np.median(g):.2f} "
          f"p90 {np.percentile(g, 90):.2f} max {g.max():.2f} us")
    ends = us[:, :, 2].max(1)
    print(f" last unit ends: {np.sort(ends)[-8:].round(1)}; per-CU finish spread "
          f"{np.percentile(ends[-256:], 10):.1f} .. {ends[-256:].max():.1f} us")
    lib.inferd_span_destroy(h)


if __name__ == "__main__":
    main()
