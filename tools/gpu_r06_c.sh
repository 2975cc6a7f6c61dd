#!/bin/bash
# round 6, GPU call C: the whole GPU suite (durations) and the default N = 1 bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -q -m gpu --timeout 600 --timeout-method thread tests --durations=45 \
  > gpurun_out/gpu_suite.log 2>&1 && \
timeout -k 10 600 python -u bench.py > gpurun_out/bench_n1_c.json 2> gpurun_out/bench_n1_c.err
rc=$?
tail -60 gpurun_out/gpu_suite.log; tail -c 1500 gpurun_out/bench_n1_c.json
exit $rc
