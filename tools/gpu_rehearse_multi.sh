#!/bin/bash
# Multi-rank rehearsal of bench.py on a 1-GPU box: ranks share the GPU over
# gloo host collectives (ZKMI_BENCH_BACKEND=gloo).  The 8-GPU RCCL run
# itself is the driver's; this checks bench.py's own launcher (--gpus N
# outside torchrun), the torchrun launch, the sharded GET (R2 slots +
# all_to_all) and the replica comparison at world 2 and 8, and the ensemble.
# BATCH (default 262144) sizes the GET batch per rank.
set -o pipefail
OUT=gpurun_out/multi
mkdir -p $OUT
export ZKMI_BENCH_BACKEND=gloo
B=${BATCH:-262144}
own() {       # bench.py starts the ranks itself
  local n=$1 tag=$2; shift 2
  timeout -k 10 300 python bench.py --gpus $n --steps 5 --warmup 2 "$@" \
    > $OUT/$tag.log 2>&1
  local rc=$?
  echo "$tag rc=$rc $(grep -h '^{' $OUT/$tag.log | tail -1 | cut -c1-400)"
  return $rc
}
trun() {      # torchrun starts them (the driver's form)
  local n=$1 tag=$2; shift 2
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
    --master-addr 127.0.0.1 --master-port $((29500 + n)) bench.py --gpus $n \
    --steps 5 --warmup 2 "$@" > $OUT/$tag.log 2>&1
  local rc=$?
  echo "$tag rc=$rc $(grep -h '^{' $OUT/$tag.log | tail -1 | cut -c1-400)"
  return $rc
}
own 2 get2_own --no-rtt --batch $B && trun 2 get2_torchrun --no-rtt --batch $B && \
  own 2 get2_sharded --no-rtt --batch $B --sharded && \
  own 8 get8_own --no-rtt --batch $B && \
  own 2 storm2 --no-rtt --workload storm --batch 65536 && \
  own 4 ens4 --workload ensemble
