"""Per decode-kernel class of a first vs an inner pipeline stage (tools/first_stage_pmc.sh): mean
duration, fetched bytes (2 x FETCH_SIZE KiB, the gfx950 correction) and the clock the chip held
(GRBM_GUI_ACTIVE / 8 XCDs / duration).  python tools/first_stage_pmc.py gpurun_out/first_pmc"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def rows(pattern):
    out = []
    for fn in glob.glob(pattern, recursive=True):
        with open(fn) as f:
            out.extend(csv.DictReader(f))
    return out


def cls(name):
    if "gemm_decode_kernel" in name:
        return "gemv<" + name.split("<", 1)[1].split(">", 1)[0] + ">"
    if "attn_decode" in name:
        return "attention"
    return None


def main():
    d = sys.argv[1]
    res = {}
    for m in ("first", "inner"):
        dur, fetch, grbm = defaultdict(list), defaultdict(list), defaultdict(list)
        for r in rows(os.path.join(d, f"trace_{m}", "**", "*kernel_trace.csv")):
            c = cls(r["Kernel_Name"])
            if c:
                dur[c].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
        per = defaultdict(dict)
        for r in rows(os.path.join(d, f"pmc_{m}", "**", "*counter_collection.csv")):
            c = cls(r.get("Kernel_Name", ""))
            if c:
                did = r.get("Dispatch_Id", r.get("Correlation_Id"))
                per[(c, did)][r["Counter_Name"]] = per[(c, did)].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        for (c, _), v in per.items():
            fetch[c].append(2 * v.get("FETCH_SIZE", 0.0) * 1024)
            grbm[c].append(v.get("GRBM_GUI_ACTIVE", 0.0))
        out = {}
        for c in sorted(dur):
            t = sum(dur[c]) / len(dur[c])
            g = sum(grbm[c]) / max(len(grbm[c]), 1)
            out[c] = {"us": round(t * 1e6, 2), "fetch_MB": round(sum(fetch[c]) / max(len(fetch[c]), 1) / 1e6, 2),
                      "clock_ghz_pmc_pass": round(g / 8 / t * 1e-9, 3) if t else None}
        res[m] = out
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
