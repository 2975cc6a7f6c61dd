"""Per-launch HBM traffic of the decode kernels from rocprofv3 PMC counters.

Run on the GPU box (two separate counter passes, as MI355X_MICROARCH.md §HBM prescribes:
FETCH_SIZE and WRITE_SIZE do not fit one TCC pass):

  rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- \
      python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-profile
  rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- \
      python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-profile
  python3 tools/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write > profiles/traffic_rNN.json

Corrections (MI355X_MICROARCH.md §HBM): both counters are in KiB; on gfx950 FETCH_SIZE reports
half the bytes of a wide (16 B/lane) coalesced streaming read, so fetched bytes =
2 * FETCH_SIZE * 1024 for the 16-B-per-lane streams the decode kernels issue; WRITE_SIZE is
exact for 16-B stores.  Infinity-Cache hits are counted as fetches.

Kernel classes: decode-phase dispatches (after the last prefill kernel) are mapped to the
bench's classes; o_proj and down_proj use the same template instance (EPI_RESID), so they
are told apart by order within a layer (o first, down second).
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def rows(d):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    out = []
    for fn in files:
        with open(fn) as f:
            out.extend(csv.DictReader(f))
    return out


PREFILL_KEYS = ("gemm_tiled", "gemm_w4", "attn_prefill", "row_inv_rms", "qk_norm_rope_kv")


def classify(name):
    """Bench kernel class of a decode-phase dispatch name (None: not a decode kernel)."""
    if "gemm_decode_kernel" in name:
        m = re.search(r"gemm_decode_kernel<([^>]+)>", name)
        if not m:
            return "gemm_decode"
        epi = int(m.group(1).split(",")[5])  # <MT, S, NW, TW, D, EPI, NORM>
        return {0: "qkv_gemm", 1: "resid_gemm", 2: "gateup_gemm", 3: "lm_head_gemv", 4: "qkv_gemm"}[epi]
    for key, cls in (("attn_decode_kernel", "attention"), ("qk_norm_rope_kv", "qk_norm_rope_kv"),
                     ("rmsnorm", "rmsnorm"), ("argmax_reduce", "argmax_reduce")):
        if key in name:
            return cls
    return None


def decode_phase(seq):
    """Dispatches after the last prefill kernel (the bench prefills before it decodes)."""
    last = -1
    for i, (name, _) in enumerate(seq):
        if any(k in name for k in PREFILL_KEYS):
            last = i
    return seq[last + 1:]


def per_dispatch(d, counter):
    """{dispatch id: (kernel name, value)} in dispatch order."""
    vals = {}
    for r in rows(d):
        if r.get("Counter_Name") != counter:
            continue
        did = int(r.get("Dispatch_Id", r.get("Correlation_Id", 0)))
        name = r.get("Kernel_Name", "")
        vals[did] = (name, vals.get(did, (name, 0.0))[1] + float(r["Counter_Value"]))
    return [vals[k] for k in sorted(vals)]


def summarize(seq, scale):
    acc = defaultdict(list)
    resid_toggle = 0
    for name, v in decode_phase(seq):
        c = classify(name)
        if c is None:
            continue
        if c == "resid_gemm":
            c = "o_gemm" if resid_toggle == 0 else "down_gemm"
            resid_toggle ^= 1
        acc[c].append(v * scale)
    return {k: sum(v) / len(v) for k, v in acc.items()}


def main():
    fetch_dir, write_dir = sys.argv[1], sys.argv[2]
    fetch = summarize(per_dispatch(fetch_dir, "FETCH_SIZE"), 2 * 1024.0)
    write = summarize(per_dispatch(write_dir, "WRITE_SIZE"), 1024.0)
    per = {k: int(fetch.get(k, 0) + write.get(k, 0)) for k in sorted(set(fetch) | set(write))}
    # the bench's lm_head_argmax class times the lm_head GEMV and the argmax reduce together
    # (one launch of each per step): its per-launch traffic is their sum, not their mean
    if "lm_head_gemv" in per:
        per["lm_head_argmax"] = per["lm_head_gemv"] + per.get("argmax_reduce", 0)
    print(json.dumps({
        "workload": "qwen3-8b-decode-B16-ctx2048",
        "method": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes); bytes = 2*FETCH_SIZE*1024 "
                  "(gfx950 half-count of 16-B streaming reads) + WRITE_SIZE*1024; mean over launches",
        "per_launch_bytes": per,
        "fetch_bytes": {k: int(v) for k, v in fetch.items()},
        "write_bytes": {k: int(v) for k, v in write.items()},
    }, indent=1))


if __name__ == "__main__":
    main()
