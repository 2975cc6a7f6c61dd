#!/bin/bash
# SQ-level PMC passes over the prefill attention variants (GPU box).  usage: tools/pmc_attn.sh <outdir> <variants...>
set -eo pipefail
out=${1:-gpurun_out/pmc_attn}; shift
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
C1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_BUSY_CYCLES"
C2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_ACTIVE_INST_MISC SQ_INSTS_SALU"
for v in "$@"; do
  INFERD_ATTN_PREFILL=$v timeout -s KILL 90 rocprofv3 --pmc $C1 -d $out/v${v}_a -o run --output-format csv -- python3 tools/attn_bench.py --rounds 1 --reps 1 > $out/v${v}_a.log 2>&1
  INFERD_ATTN_PREFILL=$v timeout -s KILL 90 rocprofv3 --pmc $C2 -d $out/v${v}_b -o run --output-format csv -- python3 tools/attn_bench.py --rounds 1 --reps 1 > $out/v${v}_b.log 2>&1
done
echo pmc done
