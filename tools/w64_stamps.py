"""Per-phase cycle anatomy of the one-wave-per-SIMD prefill attention lab (tools/labsrc/attn_w64.hip
built with -DAP_STAMP=1: s_memtime laps of workgroup 0 / wave 0 per page -- the heaviest query block
of head 0, one 8192-token prompt at Qwen3-32B dims).  Laps per page: 0->1 barrier + page DMA issue,
1->2 rescale, 2->3 phase A (S of the next page || softmax), 3->4 mask, 4->5 phase B (P.V || rest).
usage: python tools/w64_stamps.py lib.so [out.json]"""
import ctypes as C
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from inferd_amd import _lib  # noqa: E402
from inferd_amd.runtime import KvTable  # noqa: E402


def main():
    lib = C.CDLL(sys.argv[1])
    for name in ("inferd_attention", "inferd_last_error"):
        res, args = _lib.SIGNATURES[name]
        getattr(lib, name).restype = res
        getattr(lib, name).argtypes = args
    lib.inferd_lab_stamps.argtypes = [C.c_void_p]
    dev = torch.device("cuda", 0)
    H, KV, T = 64, 8, 8192
    table = KvTable((T + 63) // 64)
    table.reserve(0, T)
    bd = table.build_batch([(0, T)], dev)
    batch = _lib.batch_struct(bd.words, bd.shape)
    g = torch.Generator(device=dev).manual_seed(5)
    pool = ((T + 63) // 64 + 15) // 16 * 16
    kv = torch.randn(pool * 2 * KV * 64 * 128, device=dev, generator=g).to(torch.bfloat16)
    q = (torch.randn(T, H, 128, device=dev, generator=g) * 1.2).to(torch.bfloat16)
    out = torch.empty(T, H * 128, dtype=torch.bfloat16, device=dev)
    runs = []
    for _ in range(4):
        rc = lib.inferd_attention(q.data_ptr(), kv.data_ptr(), batch, H, KV, out.data_ptr(), None, 0, _lib.stream_ptr())
        assert rc == 0, lib.inferd_last_error()
        torch.cuda.synchronize()
        buf = (C.c_ulonglong * (8 * 160))()
        assert lib.inferd_lab_stamps(buf) == 0
        runs.append(list(buf))
    names = ["barrier+dma", "rescale", "phase_a", "mask", "phase_b", "to_next_top"]
    res = []
    for st in runs[1:]:
        n = 0
        acc = [0] * 6
        for i in range(1, 127):
            s = st[i * 8:i * 8 + 6]
            nxt = st[(i + 1) * 8]
            if not all(s) or not nxt:
                break
            lap = [s[1] - s[0], s[2] - s[1], s[3] - s[2], s[4] - s[3], s[5] - s[4], nxt - s[5]]
            acc = [a + b for a, b in zip(acc, lap)]
            n += 1
        res.append({"pages": n, **{k: round(a / max(n, 1)) for k, a in zip(names, acc)},
                    "total": round(sum(acc) / max(n, 1))})
    out_d = {"per_page_cycles_runs": res,
             "note": "s_memtime cycles per page (pages 1..126), workgroup 0 wave 0, heaviest query block; "
                     "phase_a/phase_b hold 32 MFMAs each (32 cycles each at the pipe floor)"}
    print(json.dumps(out_d, indent=1))
    if len(sys.argv) > 2:
        with open(sys.argv[2], "w") as f:
            json.dump(out_d, f, indent=1)


if __name__ == "__main__":
    main()
