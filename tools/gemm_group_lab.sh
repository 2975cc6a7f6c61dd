#!/bin/bash
# Prefill GEMM tile grouping lab (GPU box): time the 32B projection shapes with lab builds of
# tile_order_v's row-block group GM (tools/build_probes.sh gemm.hip gmN='-DW4_GM=N'), then one
# FETCH_SIZE pass per selected build.  usage: tools/gemm_group_lab.sh "base gm1 ..." "base gm1"
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
lib_of() { [ "$1" = base ] && echo "$GRAFT_REPO_ROOT/inferd_amd/libinferd_span.so" || echo "$GRAFT_REPO_ROOT/tools/probe_libs/libinferd_span_$1.so"; }
for g in $1; do
  echo "== time $g"
  INFERD_LIB=$(lib_of $g) timeout -k 10 150 python tools/gemm_bench.py --variants 256 --shapes gateup,down,qkv,o --rounds 5 \
    > gpurun_out/grp_$g.log 2>&1 || { echo "rc=$? at $g"; exit 1; }
  grep "M=" gpurun_out/grp_$g.log
done
for g in $2; do
  echo "== fetch $g"
  (cd /tmp && INFERD_LIB=$(lib_of $g) timeout -s KILL 100 rocprofv3 --pmc FETCH_SIZE -d "$GRAFT_REPO_ROOT/gpurun_out/pmc_grp_$g" \
    -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/tools/gemm_bench.py" --variants 256 --shapes gateup,down \
    --rounds 1 --reps 1 > "$GRAFT_REPO_ROOT/gpurun_out/pmc_grp_$g.log" 2>&1) || { echo "rc=$? at fetch $g"; exit 1; }
done
echo lab done
