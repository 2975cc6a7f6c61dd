#!/bin/bash
# Ring GEMM vs hipBLASLt (torch.matmul) on one prefill shape: kernel names/durations and
# clock (GRBM_GUI_ACTIVE over the kernel's duration) + MFMA busy.  usage: tools/pmc_vs_lib.sh <outdir> <shape>
set -eo pipefail
out=${1:-gpurun_out/vslib}
shape=${2:-qkv}
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $out/trace -o run --output-format csv -- python3 tools/gemm_bench.py --rounds 2 --reps 2 --variants ring,torch --shapes $shape > $out/trace.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU -d $out/pmc -o run --output-format csv -- python3 tools/gemm_bench.py --rounds 1 --reps 1 --variants ring,torch --shapes $shape > $out/pmc.log 2>&1
echo done
