#!/bin/bash
# First vs inner stage decode kernels: FETCH_SIZE and GRBM_GUI_ACTIVE per dispatch (one pass each
# mode) plus kernel traces, for tools/first_stage_pmc.py.  usage (GPU box): bash tools/first_stage_pmc.sh
set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/first_pmc
mkdir -p $out
for m in first inner; do
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE -d $out/pmc_$m -o run --output-format csv -- python3 tools/first_stage_probe.py $m > $out/pmc_$m.log 2>&1
  timeout -k 10 120 rocprofv3 --kernel-trace -d $out/trace_$m -o run --output-format csv -- python3 tools/first_stage_probe.py $m > $out/trace_$m.log 2>&1
done
echo first stage pmc done
