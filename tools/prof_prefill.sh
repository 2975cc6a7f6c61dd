set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/prof_r01b
mkdir -p $out
timeout -k 10 400 python3 -u bench.py > $out/bench_n1.log 2>&1
timeout -k 10 300 python3 -u bench.py --mode prefill --steps 16 --warmup 3 > $out/bench_prefill.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/ptrace -o run --output-format csv -- python3 bench.py --mode prefill --steps 4 --warmup 1 --no-cpu-baseline > $out/ptrace.log 2>&1
find $out/ptrace -name "*kernel_stats.csv" -exec cp {} $out/prefill_kernel_stats.csv \;
echo done
