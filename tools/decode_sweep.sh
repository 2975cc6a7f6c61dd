#!/bin/bash
# Decode-GEMM tuning sweep on the GPU box: one short bench per (waves/WG, K slices) setting.
# Usage: tools/decode_sweep.sh "4:0:1 8:1:0"   (NW:KS:FUSE_NORM, KS 0 = auto)
set -o pipefail
mkdir -p gpurun_out/sweep
for cfg in ${1:-"4:0:1 8:0:1 4:1:1 8:1:1"}; do
  IFS=: read nw ks fuse <<< "$cfg"
  echo "== NW=$nw KS=$ks FUSE_NORM=$fuse"
  INFERD_DECODE_NW=$nw INFERD_DECODE_KS=$ks INFERD_FUSE_NORM=$fuse timeout -k 10 300 python3 bench.py --steps 16 --warmup 2 \
      --no-cpu-baseline > gpurun_out/sweep/nw${nw}_ks${ks}_f${fuse}.log 2>&1 || { echo "bench failed ($?)"; exit 1; }
  tail -1 gpurun_out/sweep/nw${nw}_ks${ks}_f${fuse}.log | python3 -c '
import json,sys
d=json.loads(sys.stdin.read())
k=d.get("kernels") or d.get("profile") or {}
print(d["value"], d["ms_per_step"])
for n,v in k.items(): print("  %-16s %7.2f us %6.0f GB/s"%(n,v["avg_us"],v["GB/s"]))'
done
