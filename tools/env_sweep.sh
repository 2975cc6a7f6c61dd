#!/bin/bash
# Decode-bench A/B over environment settings on the GPU box.
# usage: tools/env_sweep.sh "VAR=a,VAR2=b" "VAR=c" ...   (one short bench per argument; "-" = no vars)
set -o pipefail
mkdir -p gpurun_out/envsweep
i=0
for cfg in "$@"; do
  i=$((i+1))
  envs=""; [ "$cfg" != "-" ] && envs=$(echo "$cfg" | tr ',' ' ')
  env $envs timeout -k 10 200 python3 bench.py --steps 16 --warmup 2 --no-cpu-baseline \
      > gpurun_out/envsweep/run$i.log 2>&1 || { echo "bench failed ($?) for $cfg"; exit 1; }
  tail -1 gpurun_out/envsweep/run$i.log | python3 -c '
import json,sys
d=json.loads(sys.stdin.read()); k=d["kernels"]
print("'"$cfg"'", d["value"], d["ms_per_step"], " ".join("%s=%.1f"%(n[:6],v["avg_us"]) for n,v in k.items()))'
done
