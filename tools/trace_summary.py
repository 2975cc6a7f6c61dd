"""Per-class kernel durations of the decode phase from a rocprofv3 --kernel-trace CSV.

  python3 tools/trace_summary.py gpurun_out/prof_r01/trace > profiles/r01/decode_kernel_trace.json

Dispatches after the last prefill kernel are classified like tools/pmc_traffic.py (o / down
told apart by order).  Reports mean kernel duration (End - Start) per class and the mean
gap between consecutive decode kernels (launch boundaries inside the replayed graphs).
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_traffic import PREFILL_KEYS, classify  # noqa: E402


def main():
    d = sys.argv[1]
    files = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no kernel_trace.csv under {d}")
    rows = []
    for fn in files:
        with open(fn) as f:
            rows.extend(csv.DictReader(f))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    last = -1
    for i, r in enumerate(rows):
        if any(k in r["Kernel_Name"] for k in PREFILL_KEYS):
            last = i
    rows = rows[last + 1:]
    acc = defaultdict(list)
    toggle = 0
    gaps = []
    prev_end = None
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        c = classify(r["Kernel_Name"])
        if c is None:
            prev_end = None
            continue
        if c == "resid_gemm":
            c = "o_gemm" if toggle == 0 else "down_gemm"
            toggle ^= 1
        acc[c].append((e - s) / 1e3)
        if prev_end is not None and 0 <= s - prev_end < 50_000:
            gaps.append((s - prev_end) / 1e3)
        prev_end = e
    out = {"source": "rocprofv3 --kernel-trace (decode phase: dispatches after the last prefill kernel)",
           "classes": {k: {"launches": len(v), "avg_us": round(sum(v) / len(v), 2),
                           "min_us": round(min(v), 2), "max_us": round(max(v), 2)} for k, v in sorted(acc.items())},
           "mean_gap_us": round(sum(gaps) / len(gaps), 2) if gaps else None}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
