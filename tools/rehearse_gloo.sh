set -eo pipefail
mkdir -p gpurun_out
export INFERD_DIST_BACKEND=gloo
for n in 2 4; do
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus $n --steps 4 --warmup 1 --no-cpu-baseline --no-profile > gpurun_out/rehearse_n$n.log 2>&1
done
timeout -k 10 300 python bench.py > gpurun_out/bench_n1_b.log 2>&1
