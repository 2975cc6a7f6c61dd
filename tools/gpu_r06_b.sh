#!/bin/bash
# round 6, GPU call B: ring / head GPU tests on the compute-stream build, the N = 2 / 4 bench rehearsal
# over gloo (ranks sharing this GPU), then the default N = 1 bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_pipeline_gpu.py \
  tests/test_gpu_rccl.py "tests/test_gpu_parity.py::test_q8b_pipeline_vocab_parallel_head" > gpurun_out/t2.log 2>&1 && \
INFERD_DIST_BACKEND=gloo timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 4 --warmup 1 --no-cpu-baseline \
  > gpurun_out/rehearse_n2.log 2>&1 && \
INFERD_DIST_BACKEND=gloo timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
  --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 4 --steps 4 --warmup 1 --no-cpu-baseline \
  --no-sublayer-split > gpurun_out/rehearse_n4.log 2>&1 && \
timeout -k 10 600 python -u bench.py > gpurun_out/bench_n1.json 2> gpurun_out/bench_n1.err
rc=$?
tail -5 gpurun_out/t2.log; tail -c 1500 gpurun_out/rehearse_n4.log; tail -c 3000 gpurun_out/bench_n1.json
exit $rc
