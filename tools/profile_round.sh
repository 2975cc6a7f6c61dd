#!/bin/bash
# Round profile on the GPU box (summaries go to profiles/<tag>/ after the merge-back):
#   decode : rocprofv3 --kernel-trace --stats of the decode bench, then the two PMC passes
#            (FETCH_SIZE, WRITE_SIZE separately: MI355X_MICROARCH.md §HBM) -> traffic JSON
#   prefill: --kernel-trace --stats of the config-5 prefill bench
# usage: tools/profile_round.sh <tag>
set -eo pipefail
tag=${1:-r01}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/prof_$tag
mkdir -p $out
args="--steps 8 --warmup 2 --no-cpu-baseline --no-profile --no-prefill-line --no-stage-projection"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace -o run --output-format csv -- python3 bench.py $args > $out/trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $out/pmc_fetch -o run --output-format csv -- python3 bench.py $args > $out/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $out/pmc_write -o run --output-format csv -- python3 bench.py $args > $out/write.log 2>&1
python3 tools/pmc_traffic.py $out/pmc_fetch $out/pmc_write > $out/traffic.json
python3 tools/trace_summary.py $out/trace > $out/decode_kernel_trace.json
find $out/trace -name "*kernel_stats.csv" -exec cp {} $out/decode_kernel_stats.csv \;
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/ptrace -o run --output-format csv -- python3 bench.py --mode prefill --steps 4 --warmup 1 --no-cpu-baseline > $out/ptrace.log 2>&1
find $out/ptrace -name "*kernel_stats.csv" -exec cp {} $out/prefill_kernel_stats.csv \;
echo profile done
