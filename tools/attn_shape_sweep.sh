#!/bin/bash
# Decode attention (waves, chunks) A/B on the GPU box via short decode benches.
set -o pipefail
mkdir -p gpurun_out/ashape
for cfg in ${1:-8:2 4:4 8:4 4:2 4:8 8:3}; do
  IFS=: read nw nc <<< "$cfg"
  INFERD_ATTN_NW=$nw INFERD_ATTN_NC=$nc timeout -k 10 200 python3 bench.py --steps 16 --warmup 2 --no-cpu-baseline \
      > gpurun_out/ashape/a${nw}_${nc}.log 2>&1 || { echo "bench failed ($?)"; exit 1; }
  tail -1 gpurun_out/ashape/a${nw}_${nc}.log | python3 -c '
import json,sys
d=json.loads(sys.stdin.read()); k=d["kernels"]
print("nw:nc '$cfg'", d["value"], d["ms_per_step"], "attention=%.2f" % k["attention"]["avg_us"])'
done
