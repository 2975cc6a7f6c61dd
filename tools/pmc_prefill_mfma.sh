#!/bin/bash
# Prefill MFMA utilisation on the GPU box: two SQ/GRBM counter passes (7 SQ + 1 GRBM counters each,
# within one pass's limits: MFMA busy / VALU, then the wave-cycle split parked / issue-stalled /
# issuing) and one un-counted kernel-trace pass for the durations.
#   tools/pmc_prefill_mfma.sh -> gpurun_out/pmc_mfma/mfma_prefill.json
set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B=${1:-1}
export PMC_BATCH=$B
out=gpurun_out/pmc_mfma$([ "$B" = 1 ] || echo _b$B)
mkdir -p $out
args="--mode prefill --steps 1 --warmup 1 --no-cpu-baseline --prefill-batch $B"
C="SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
timeout -s KILL 240 rocprofv3 --pmc $C -d $out/pmc -o run --output-format csv -- python3 bench.py $args > $out/pmc.log 2>&1
C2="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_COEXEC_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
timeout -s KILL 240 rocprofv3 --pmc $C2 -d $out/pmc2 -o run --output-format csv -- python3 bench.py $args > $out/pmc2.log 2>&1
timeout -k 10 240 rocprofv3 --kernel-trace -d $out/trace -o run --output-format csv -- python3 bench.py $args > $out/trace.log 2>&1
python3 tools/pmc_prefill_mfma.py $out/pmc $out/trace $out/pmc2 > $out/mfma_prefill.json
echo pmc mfma done
