#!/bin/bash
# Prefill PMC traffic (two separate counter passes) on the GPU box:
#   tools/pmc_prefill.sh -> gpurun_out/pmc_prefill/traffic_prefill.json
set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/pmc_prefill
mkdir -p $out
args="--mode prefill --steps 1 --warmup 1"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $out/fetch -o run --output-format csv -- python3 bench.py $args > $out/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $out/write -o run --output-format csv -- python3 bench.py $args > $out/write.log 2>&1
python3 tools/pmc_prefill.py $out/fetch $out/write > $out/traffic_prefill.json
echo pmc prefill done
