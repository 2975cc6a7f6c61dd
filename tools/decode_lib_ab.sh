#!/bin/bash
# Decode A/B of whole-library builds on the GPU box: one short decode bench per library, the
# product library first and last (drift check).  A lab build lives in tools/probe_libs/<name>/
# as libinferd_span.so and is picked up through LD_LIBRARY_PATH (the torch-ops library finds
# libinferd_span.so by RUNPATH, which LD_LIBRARY_PATH precedes).
# usage: tools/decode_lib_ab.sh <name> [<name> ...]   -> gpurun_out/decode_ab/<i>_<name>.log
set -o pipefail
mkdir -p gpurun_out/decode_ab
args="--steps 32 --warmup 4 --no-cpu-baseline --no-prefill-line"
i=0
for n in base "$@" base; do
  i=$((i+1))
  if [ "$n" = base ]; then
    timeout -k 10 240 python3 bench.py $args > gpurun_out/decode_ab/${i}_$n.log 2>&1 || { echo "bench $n failed ($?)"; exit 1; }
  else
    LD_LIBRARY_PATH="$GRAFT_REPO_ROOT/tools/probe_libs/$n${LD_LIBRARY_PATH:+:$LD_LIBRARY_PATH}" \
      timeout -k 10 240 python3 bench.py $args > gpurun_out/decode_ab/${i}_$n.log 2>&1 || { echo "bench $n failed ($?)"; exit 1; }
  fi
  tail -1 gpurun_out/decode_ab/${i}_$n.log | python3 -c '
import json,sys
d=json.loads(sys.stdin.read()); k=d.get("kernels") or {}
print("'"$n"'", d["value"], d["ms_per_step"], " ".join("%s=%.2f"%(a[:6],b["avg_us"]) for a,b in k.items()), flush=True)'
done
