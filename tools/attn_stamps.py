"""Per-phase account of the shipped prefill attention on BASELINE config 5's
shape: Qwen3-32B heads (H = 64, KV = 8), one 8192-token causal prompt.

Builds (if needed) and loads tools/labbin/libattn_stamps.so (tools/attn_prefill_stamps.hip: the
product kernel's page functions, included unchanged, under a copy of its top level with s_memtime
stamps per phase), checks its output is bit-identical to the product library's, times the
product kernel alone (HIP events), and prints per-wave phase cycles and their shares as JSON.

  python tools/attn_stamps.py > gpurun_out/attn_stamps.json
"""
import ctypes as C
import json
import os
import subprocess
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from inferd_amd import _lib  # noqa: E402
from inferd_amd.runtime import KvTable  # noqa: E402

PHASES = ("prologue", "wait_page0", "s_softmax", "pv", "barrier", "issue_next", "epilogue")
MFMA_CYCLES = 16      # matrix-pipe cycles per v_mfma_f32_16x16x32_bf16 (SQ_VALU_MFMA_BUSY_CYCLES / MFMA,
                      # profiles/mfma_prefill_r04.json: the GEMMs' 16.0)
NB = 3


def main():
    so = os.path.join(ROOT, "tools", "labbin", "libattn_stamps.so")
    src = os.path.join(ROOT, "tools", "attn_prefill_stamps.hip")
    if not os.path.exists(so) or os.path.getmtime(so) < os.path.getmtime(src):
        os.makedirs(os.path.dirname(so), exist_ok=True)
        subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++20", "-fPIC",
                               "-fno-honor-nans", "-fno-slp-vectorize", "-shared", src, "-o", so])
    lab = C.CDLL(so)
    lab.lab_attn_prefill_stamps.restype = C.c_int
    lab.lab_attn_prefill_stamps.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_void_p,
                                            C.c_void_p, C.c_void_p]
    lab.lab_attn_prefill_grid.restype = C.c_int
    lab.lab_attn_prefill_grid.argtypes = [C.c_void_p, C.c_int]
    lib = _lib.load()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    H, KV, B, T = 64, 8, 1, 8192
    pages_per = (T + 63) // 64
    table = KvTable(B * pages_per)
    table.reserve(0, T)
    bd = table.build_batch([(0, T)], dev)
    batch = _lib.batch_struct(bd.words, bd.shape)
    pool_pages = (B * pages_per + 15) // 16 * 16
    g = torch.Generator(device=dev).manual_seed(5)
    kv = torch.randn(pool_pages * 2 * KV * 64 * 128, device=dev, generator=g).to(torch.bfloat16)
    q = (torch.randn(B * T, H, 128, device=dev, generator=g) * 1.2).to(torch.bfloat16)
    out_p = torch.empty(B * T, H * 128, dtype=torch.bfloat16, device=dev)
    out_l = torch.empty_like(out_p)
    st = _lib.stream_ptr()
    n = lab.lab_attn_prefill_grid(C.byref(batch), H)
    stamps = torch.zeros(n * B * 4 * 12, dtype=torch.int64, device=dev)

    def prod():
        assert lib.inferd_attention(q.data_ptr(), kv.data_ptr(), C.byref(batch), H, KV, out_p.data_ptr(), None, 0,
                                    st) == 0, lib.inferd_last_error()

    def labrun():
        assert lab.lab_attn_prefill_stamps(q.data_ptr(), kv.data_ptr(), C.byref(batch), H, KV, out_l.data_ptr(),
                                           stamps.data_ptr(), st) == 0

    times = {"product": [], "stamped": []}
    for _ in range(5):
        for name, fn in (("product", prod), ("stamped", labrun)):
            fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(3):
                fn()
            e1.record()
            torch.cuda.synchronize()
            times[name].append(e0.elapsed_time(e1) / 3)
    identical = bool(torch.equal(out_p, out_l))
    s = stamps.view(-1, 12).cpu()
    work = s[s[:, 7] > 0]
    wave_cyc = work[:, :7].sum(1).double()
    tot = work[:, :7].double().sum(0)
    pages = work[:, 7].double().sum().item()
    masked = work[:, 8].double().sum().item()
    per_page = {p: round(tot[i].item() / pages, 1) for i, p in enumerate(PHASES) if p in ("s_softmax", "pv", "barrier",
                                                                                          "issue_next")}
    mfma_per_page = (16 * NB) + (16 * NB + 2 * NB)      # S: 16 K fragments x NB; P.V: 16 V fragments x NB + row sums
    wall = (work[:, 11] - work[:, 10]).double() * 10.0  # ns (100 MHz realtime)
    clock = (wave_cyc / wall).median().item()           # shader cycles per ns of the same waves
    med = lambda xs: sorted(xs)[len(xs) // 2]  # noqa: E731
    flops = B * 4.0 * H * 128 * T * (T + 1) / 2
    page_cyc = sum(per_page.values())
    res = {
        "workload": "qwen3-32b prefill attention, H 64 / KV 8, T 8192, B 1 (config 5)",
        "method": "tools/attn_prefill_stamps.hip: s_memtime laps per wave around each phase of the shipped kernel's "
                  "page loop (page functions included from the product source); s_memrealtime for wall time",
        "output_bit_identical_to_product": identical,
        "product_us_median": round(med(times["product"]) * 1e3, 1),
        "stamped_us_median": round(med(times["stamped"]) * 1e3, 1),
        "product_tflops": round(flops / (med(times["product"]) * 1e-3) * 1e-12, 1),
        "waves_with_work": int(work.shape[0]),
        "pages_computed_per_wave": round(pages / work.shape[0], 2),
        "masked_page_frac": round(masked / pages, 4),
        "cycle_share": {p: round(tot[i].item() / tot.sum().item(), 4) for i, p in enumerate(PHASES)},
        "cycles_per_computed_page": per_page,
        "mfma_per_page_per_wave": mfma_per_page,
        "mfma_pipe_cycles_per_page_per_wave": mfma_per_page * MFMA_CYCLES,
        "implied_mfma_busy_in_page_loop": round(2 * mfma_per_page * MFMA_CYCLES / page_cyc, 4),
        "shader_clock_ghz_median": round(clock, 3),
        "wg_wall_us": {"median": round(wall.median().item() / 1e3, 1), "max": round(wall.max().item() / 1e3, 1)},
        "note": "two waves share each SIMD (two workgroups of four waves per CU), so a wave's page time holds its "
                "partner's MFMAs too: implied busy = 2 x MFMA cycles / page cycles.  s_memtime laps add ~+11 % "
                "of wave cycles (MI355X_MICROARCH.md)",
    }
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
