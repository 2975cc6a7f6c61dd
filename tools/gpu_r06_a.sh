#!/bin/bash
# round 6, GPU call A: the ring hand-off probe, then the new head / ring GPU tests
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/rccl_ring_probe.py gpurun_out/rccl_ring_probe.json > gpurun_out/probe.log 2>&1 && \
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_head.py \
  tests/test_pipeline_gpu.py tests/test_gpu_rccl.py "tests/test_gpu_parity.py::test_q8b_pipeline_vocab_parallel_head" \
  --durations=20 > gpurun_out/t1.log 2>&1
rc=$?
tail -40 gpurun_out/t1.log
exit $rc
