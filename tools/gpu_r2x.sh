#!/bin/bash
# 2-rank rehearsal of the default bench (graph replay) on one GPU with gloo
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
ZKMI_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 2 \
  --steps 10 --warmup 3 --batch 262144 > gpurun_out/r2x_gloo2.log 2>&1 \
  || { tail -30 gpurun_out/r2x_gloo2.log; exit 1; }
grep '^{' gpurun_out/r2x_gloo2.log | cut -c1-300
