"""Lab: per-page phase timings (s_memtime) of block 0 / wave 0 of the one-wave-per-SIMD prefill
attention, from a library built with -DAP_STAMP=1 (tools/build_attn_probes.sh st='-DAP_STAMP=1'),
on the attn_bench prefill workload.  usage: INFERD_LIB=<stamp lib> python tools/attn_stamps.py"""
import ctypes
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["INFERD_ATTN_PREFILL"] = "1"
sys.argv = [sys.argv[0], "--rounds", "1", "--reps", "1"]
sys.path.insert(0, os.path.join(ROOT, "tools"))
import attn_bench  # noqa: E402
from inferd_amd import _lib  # noqa: E402

attn_bench.main()
L = _lib.load()
buf = (ctypes.c_ulonglong * (8 * 160))()
assert L.inferd_lab_stamps(buf) == 0
st = np.frombuffer(buf, dtype=np.uint64).reshape(160, 8).astype(np.int64)
names = ["wait+barrier+dma", "rescale", "phaseA", "mask", "phaseB", "-> next"]
rows = []
for i in range(159):
    if st[i, 5] == 0 or st[i + 1, 0] == 0:
        continue
    d = [st[i, 1] - st[i, 0], st[i, 2] - st[i, 1], st[i, 3] - st[i, 2], st[i, 4] - st[i, 3], st[i, 5] - st[i, 4],
         st[i + 1, 0] - st[i, 5]]
    rows.append(d)
rows = np.array(rows)
print(f"pages stamped: {len(rows)}")
for j, n in enumerate(names):
    print(f"{n:20s} median {np.median(rows[:, j]):8.0f}  mean {rows[:, j].mean():8.0f}  max {rows[:, j].max():8.0f}")
print("first pages:", rows[:4].tolist())
