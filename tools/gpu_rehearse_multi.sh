#!/bin/bash
# Multi-rank rehearsal of bench.py on a 1-GPU box: torchrun ranks share the
# GPU over gloo host collectives (ZKMI_BENCH_BACKEND=gloo).  The 8-GPU RCCL
# run itself is the driver's; this checks the launch / collective / report
# path at world 2 and 4 for the default and the sharded GET workloads.
set -o pipefail
OUT=gpurun_out/multi
mkdir -p $OUT
export ZKMI_BENCH_BACKEND=gloo
run() {
  local n=$1 tag=$2; shift 2
  timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
    --master-addr 127.0.0.1 --master-port $((29500 + n)) bench.py --gpus $n \
    --steps 10 --warmup 2 "$@" > $OUT/$tag.log 2>&1
  local rc=$?
  echo "$tag rc=$rc $(grep -h '^{' $OUT/$tag.log | tail -1 | cut -c1-300)"
  return $rc
}
run 2 get2 --no-rtt && run 4 get4 --no-rtt && run 2 sharded2 --no-rtt --sharded && \
  run 4 ens4 --workload ensemble
