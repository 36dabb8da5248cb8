#!/bin/bash
# streams 1 vs 2 (graph replay), kernel profile of the default get
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in "--streams 1" "--streams 2" "--streams 1 --batch 2097152" "--streams 2 --batch 2097152"; do
timeout -k 10 240 python bench.py --steps 30 --warmup 5 --no-rtt $v \
  > gpurun_out/r2q_get.json 2> gpurun_out/r2q_get.err \
  || { tail -20 gpurun_out/r2q_get.err; exit 1; }
echo "[$v]"; cut -c90-220 gpurun_out/r2q_get.json
done
PROF=r2v27 WORKLOADS="get" bash tools/prof_stats.sh
