#!/bin/bash
# SQ-level PMC passes over the prefill attention (tools/attn_bench.py) on the GPU box, one pair of
# passes per library: the product library by default, or lab builds given as name=path.
# usage: tools/pmc_attn.sh <outdir> [name=lib.so ...]
set -eo pipefail
out=${1:-gpurun_out/pmc_attn}; shift || true
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
C1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_BUSY_CYCLES"
C2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_ACTIVE_INST_MISC SQ_INSTS_SALU"
libs=("$@"); [ ${#libs[@]} -eq 0 ] && libs=("span=inferd_amd/libinferd_span.so")
for nl in "${libs[@]}"; do
  n=${nl%%=*}; lib=${nl#*=}
  export INFERD_LIB=$lib
  timeout -s KILL 90 rocprofv3 --pmc $C1 -d $out/${n}_a -o run --output-format csv -- python3 tools/attn_bench.py --rounds 1 --reps 1 > $out/${n}_a.log 2>&1
  timeout -s KILL 90 rocprofv3 --pmc $C2 -d $out/${n}_b -o run --output-format csv -- python3 tools/attn_bench.py --rounds 1 --reps 1 > $out/${n}_b.log 2>&1
done
echo pmc done
