#!/bin/bash
# Round profile of the decode bench on the GPU box: kernel trace + stats, then the two PMC
# passes (FETCH_SIZE, WRITE_SIZE separately, MI355X_MICROARCH.md §HBM) -> traffic JSON.
# Usage: tools/profile_decode.sh <round tag, e.g. r01>
set -eo pipefail
tag=${1:-r01}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/prof_$tag
mkdir -p $out
args="--steps 8 --warmup 2 --no-cpu-baseline --no-profile"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/trace -o run --output-format csv -- python3 bench.py $args > $out/trace.log 2>&1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d $out/pmc_fetch -o run --output-format csv -- python3 bench.py $args > $out/fetch.log 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d $out/pmc_write -o run --output-format csv -- python3 bench.py $args > $out/write.log 2>&1
python3 tools/pmc_traffic.py $out/pmc_fetch $out/pmc_write > $out/traffic.json
find $out -name "*kernel_stats.csv" -exec cp {} $out/kernel_stats.csv \;
echo done
