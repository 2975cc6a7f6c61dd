"""Summarise rocprofv3 counter_collection CSVs: per kernel (name filter), counters summed over
dispatches and normalised by SQ_WAVE_CYCLES when present.  usage: pmc_summary.py <dir>... [--filter s]"""
import collections
import csv
import glob
import sys

args = [a for a in sys.argv[1:] if not a.startswith("--")]
flt = sys.argv[sys.argv.index("--filter") + 1] if "--filter" in sys.argv else ""
for d in args:
    if d == flt:
        continue
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        agg = collections.defaultdict(lambda: collections.defaultdict(float))
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if flt and flt not in k:
                continue
            agg[k[:70]][r["Counter_Name"]] += float(r["Counter_Value"])
        for k, v in agg.items():
            print(d, "|", k)
            wc = v.get("SQ_WAVE_CYCLES")
            for c, x in sorted(v.items()):
                print(f"   {c:28s} {x:14.4g}" + (f"  {x / wc:7.3f}" if wc else ""))
