#!/bin/bash
# SQ-level PMC pass over the prefill attention and GEMM microbenches (GPU box).
# usage: tools/pmc_kernels.sh <outdir>
set -eo pipefail
out=${1:-gpurun_out/pmc}
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rocprofv3 -L > $out/counters.txt 2>&1 || true
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_BUSY_CYCLES"
timeout -s KILL 90 rocprofv3 --pmc $C -d $out/attn -o run --output-format csv -- python3 tools/attn_bench.py --rounds 1 --reps 1 > $out/attn.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc $C -d $out/gemm -o run --output-format csv -- python3 tools/gemm_bench.py --rounds 1 --reps 1 --variants ring --shapes gateup,down > $out/gemm.log 2>&1
echo pmc done
