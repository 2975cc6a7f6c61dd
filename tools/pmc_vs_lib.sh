#!/bin/bash
# Prefill GEMM variants vs hipBLASLt (torch.matmul) on one shape: kernel names/durations and
# SQ counters (clock = GRBM_GUI_ACTIVE / 8 / duration; MFMA busy; LDS waits and bank conflicts).
# usage: tools/pmc_vs_lib.sh <outdir> <shape> [variants]
set -eo pipefail
out=${1:-gpurun_out/vslib}
shape=${2:-qkv}
variants=${3:-w4,torch}
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $out/trace -o run --output-format csv -- python3 tools/gemm_bench.py --rounds 2 --reps 2 --variants $variants --shapes $shape > $out/trace.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_ACTIVE_INST_ANY -d $out/pmc -o run --output-format csv -- python3 tools/gemm_bench.py --rounds 1 --reps 1 --variants $variants --shapes $shape > $out/pmc.log 2>&1
echo done
