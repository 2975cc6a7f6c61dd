#!/bin/bash
# Prefill PMC traffic (two separate counter passes) on the GPU box:
#   tools/pmc_prefill.sh [B] -> gpurun_out/pmc_prefill[_bB]/traffic_prefill.json (B 8k prompts per call)
set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B=${1:-1}
export PMC_BATCH=$B
out=gpurun_out/pmc_prefill$([ "$B" = 1 ] || echo _b$B)
mkdir -p $out
args="--mode prefill --steps 1 --warmup 1 --prefill-batch $B"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $out/fetch -o run --output-format csv -- python3 bench.py $args > $out/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $out/write -o run --output-format csv -- python3 bench.py $args > $out/write.log 2>&1
python3 tools/pmc_prefill.py $out/fetch $out/write > $out/traffic_prefill.json
echo pmc prefill done
