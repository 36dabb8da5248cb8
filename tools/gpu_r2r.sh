#!/bin/bash
# variable vs fixed-size GET at the same mean payload, with kernel profiles
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in "--data-bytes 512" "--data-dist uniform:0-1024" "--data-bytes 1024"; do
timeout -k 10 240 python bench.py --steps 20 --warmup 3 --no-rtt $v \
  > gpurun_out/r2r_get.json 2> gpurun_out/r2r_get.err \
  || { tail -20 gpurun_out/r2r_get.err; exit 1; }
echo "[$v]"; cut -c90-220 gpurun_out/r2r_get.json
done
PROF=r2v28f BENCH_ARGS="--data-bytes 512" WORKLOADS="get" bash tools/prof_stats.sh && \
PROF=r2v28v BENCH_ARGS="--data-dist uniform:0-1024" WORKLOADS="get" bash tools/prof_stats.sh
