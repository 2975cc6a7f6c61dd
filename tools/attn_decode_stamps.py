"""Per-phase anatomy of the shipped decode attention (attn_decode_kernel<8, FUSED>) on BASELINE
config 3's shape: Qwen3-8B heads (H = 32, KV = 8), B = 16 sequences at 2048 cached tokens, one
decode token each, inside a 1-layer span's decode forward (split-K q/k/v partials in, packed
output for the o GEMV -- the product path).

Loads the lab build tools/probe_libs/libinferd_span_decstamps.so (attention.hip compiled with
-DATTN_DEC_STAMPS: s_memrealtime stamps per workgroup into a buffer of its own; the product
binary is unchanged) beside the product library, runs both spans on the same weights and
inputs (outputs must be bit-identical), times the product's decode forward per kernel class
(HIP events) and prints the lab launch's phase timeline as JSON: when workgroups start, how long
their K/V stream runs, the spread between a workgroup's waves, the LDS merge, the chunk
hand-off (publish, ticket) and the last arriver's merge, all in microseconds of the 100 MHz
real-time clock.

  tools/build_probes.sh attention.hip decstamps='-DATTN_DEC_STAMPS=1'
  python tools/attn_decode_stamps.py [--layers=36] [name=lib.so ...] > gpurun_out/attn_decode_stamps.json
"""
import ctypes as C
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from inferd_amd import _lib  # noqa: E402
from inferd_amd.runtime import MODELS, KvTable  # noqa: E402

SLOTS = 16
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


def pct(v, q):
    v = sorted(v)
    return v[min(len(v) - 1, int(q * (len(v) - 1) + 0.5))]


def summary(v):
    return {"min": round(min(v), 2), "p10": round(pct(v, 0.1), 2), "median": round(statistics.median(v), 2),
            "p90": round(pct(v, 0.9), 2), "max": round(max(v), 2)}


def stamp_summary(launches):
    per = {k: [] for k in ("start_offset", "q_landed", "q_ready", "q_ready_chunk0", "q_ready_chunk1", "stream_wave_max",
                           "stream_end_chunk0", "stream_end_chunk1", "wave_spread", "lds_merge", "publish",
                           "ticket", "last_merge", "stream_end_abs", "exit_abs")}
    spans_us, out = [], []
    for s in launches:
        s = s[s[:, 0] != 0].double()
        t0 = s[:, 0].min()
        us = (s - t0) / 100.0
        end = us[:, 13].max().item()
        spans_us.append(end)
        last = (s[:, 14].long() & 1) == 1
        wave_end = us[:, 2:10].max(dim=1).values
        per["start_offset"] += us[:, 0].tolist()
        per["q_landed"] += (us[:, 15] - us[:, 0]).tolist()
        per["q_ready"] += (us[:, 1] - us[:, 0]).tolist()
        chunk = (s[:, 14].long() >> 16) & 0xFF
        per["q_ready_chunk0"] += (us[chunk == 0, 1] - us[chunk == 0, 0]).tolist()
        per["q_ready_chunk1"] += (us[chunk == 1, 1] - us[chunk == 1, 0]).tolist()
        per["stream_wave_max"] += (wave_end - us[:, 1]).tolist()
        per["wave_spread"] += (wave_end - us[:, 2:10].min(dim=1).values).tolist()
        per["lds_merge"] += (us[:, 10] - wave_end).tolist()
        per["publish"] += (us[:, 11] - us[:, 10]).tolist()
        per["ticket"] += (us[:, 12] - us[:, 11]).tolist()
        per["last_merge"] += (us[last, 13] - us[last, 12]).tolist()
        per["stream_end_abs"] += wave_end.tolist()
        per["stream_end_chunk0"] += wave_end[chunk == 0].tolist()
        per["stream_end_chunk1"] += wave_end[chunk == 1].tolist()
        per["exit_abs"] += us[:, 13].tolist()
        out.append({"workgroups": int(s.shape[0]), "first_to_last_exit_us": round(end, 2),
                    "last_start_us": round(us[:, 0].max().item(), 2),
                    "stream_end_p50_us": round(statistics.median(wave_end.tolist()), 2),
                    "stream_end_max_us": round(wave_end.max().item(), 2), "last_arrivers": int(last.sum().item())})
    return {"first_to_last_exit_us_median": round(statistics.median(spans_us), 2),
            "phase_us": {k: summary(v) for k, v in per.items() if v}, "launches": out}


def main():
    libs = {"product": os.path.join(ROOT, "inferd_amd", "libinferd_span.so")}
    argv = sys.argv[1:]
    n_layers = 1
    if argv and argv[0].startswith("--layers="):
        n_layers = int(argv.pop(0).split("=")[1])
    for spec in argv or ["stamps=tools/probe_libs/libinferd_span_decstamps.so"]:
        name, path = spec.split("=", 1)
        libs[name] = path if os.path.isabs(path) else os.path.join(ROOT, path)
    d = MODELS["qwen3-8b"]
    dev = torch.device("cuda", 0)
    B, ctx, rounds = 16, 2048, 9
    st = _lib.stream_ptr()
    pages = B * (ctx // 64 + 2) + 16
    table = KvTable(pages)
    for b in range(B):
        table.reserve(b, ctx)
    pre = table.build_batch([(b, ctx) for b in range(B)], dev)
    cfg = _lib.SpanConfig(hidden=d.hidden, intermediate=d.intermediate, heads=d.heads, kv_heads=d.kv_heads,
                          head_dim=d.head_dim, vocab=d.vocab, first_layer=0, n_layers=n_layers, has_embed=0, has_lm_head=0,
                          rms_eps=d.eps, rope_theta=d.rope_theta, max_positions=ctx + 64, kv_pages=pages,
                          max_tokens=B * ctx, max_seqs=B)
    spans = {}
    g = torch.Generator(device="cpu").manual_seed(7)
    x = (torch.randn(B * ctx, d.hidden, generator=g) * 0.5).to(torch.bfloat16).to(dev)
    xo = torch.empty_like(x)
    pre_batch = _lib.batch_struct(pre.words, pre.shape)
    for name, path in libs.items():
        lib = load(path)
        h = C.c_void_p()
        check(lib, lib.inferd_span_create(C.byref(cfg), C.byref(h)))
        check(lib, lib.inferd_span_init_synthetic(h, 1234, st))
        check(lib, lib.inferd_span_forward(h, C.byref(pre_batch), None, x.data_ptr(), xo.data_ptr(), None, None,
                                           None, st))
        stamped = hasattr(lib, "inferd_lab_dec_stamps")
        if stamped:
            lib.inferd_lab_dec_stamps.restype = C.c_int
            lib.inferd_lab_dec_stamps.argtypes = [C.c_void_p]
        spans[name] = (lib, h, stamped)
    torch.cuda.synchronize()
    for b in range(B):
        table.advance(b, ctx)
        table.reserve(b, 1)
    dec = table.build_batch([(b, 1) for b in range(B)], dev)
    dec_batch = _lib.batch_struct(dec.words, dec.shape)
    xd = (torch.randn(B, d.hidden, generator=g) * 0.5).to(torch.bfloat16).to(dev)
    outs = {n: torch.empty_like(xd) for n in spans}
    n_wg = 2 * d.kv_heads * B * 4          # >= the launch's grid (chunks x kv heads x sequences)
    stamps = torch.zeros(n_wg * SLOTS, dtype=torch.int64, device=dev)
    tot = (C.c_double * 8)()
    cnt = (C.c_int32 * 8)()
    prof = {n: {c: [] for c in CLASSES} for n in spans}
    launches = {n: [] for n in spans}
    for rnd in range(rounds + 1):
        for name, (lib, h, stamped) in spans.items():
            # an event-timed forward (per kernel class), then a stamped one (lab builds with stamps)
            check(lib, lib.inferd_span_profile_start(h, 16 * n_layers + 16))
            check(lib, lib.inferd_span_forward(h, C.byref(dec_batch), None, xd.data_ptr(), outs[name].data_ptr(),
                                               None, None, None, st))
            torch.cuda.synchronize()
            check(lib, lib.inferd_span_profile_stop(h, tot, cnt, 8))
            if rnd:
                for i, c in enumerate(CLASSES):
                    if cnt[i]:
                        prof[name][c].append(tot[i] / cnt[i] * 1e3)
            if stamped:
                stamps.zero_()
                check(lib, lib.inferd_lab_dec_stamps(C.c_void_p(stamps.data_ptr())))
                check(lib, lib.inferd_span_forward(h, C.byref(dec_batch), None, xd.data_ptr(), outs[name].data_ptr(),
                                                   None, None, None, st))
                torch.cuda.synchronize()
                check(lib, lib.inferd_lab_dec_stamps(None))
                if rnd:
                    launches[name].append(stamps.view(-1, SLOTS).cpu())
    res = {"workload": "qwen3-8b %d-layer span decode, B=16 at ctx 2048 (config 3 shape; stamps: the last layer's "
                       "attention launch); libraries interleaved round by round, medians over %d rounds"
                       % (n_layers, rounds), "libs": {}}
    for name in spans:
        r = {"path": os.path.relpath(libs[name], ROOT),
             "bit_identical_to_product": bool(torch.equal(outs[name], outs["product"])),
             "kernel_us_median": {c: round(statistics.median(v), 2) for c, v in prof[name].items() if v}}
        if launches[name]:
            r["stamps"] = stamp_summary(launches[name])
        res["libs"][name] = r
    res["note"] = ("stamps.phase_us per workgroup over all stamped launches: start_offset = its entry after the "
                   "launch's first workgroup; q_landed = entry -> the q image in LDS (wave 0); q_ready = entry -> q arithmetic "
                   "(and, chunk 1, the new token's K/V write) done (wave 0); stream_wave_max = q "
                   "ready -> its slowest wave's last K/V item; wave_spread = slowest - fastest wave; lds_merge = "
                   "slowest wave -> after the LDS merge barrier; publish = partial stores drained; ticket = the "
                   "arrival add + barrier; last_merge = the last arriver's chunk merge and output stores; *_abs = "
                   "times after the launch's first entry (100 MHz s_memrealtime)")
    print(json.dumps(res, indent=1))
    for lib, h, _ in spans.values():
        lib.inferd_span_destroy(h)


if __name__ == "__main__":
    main()
