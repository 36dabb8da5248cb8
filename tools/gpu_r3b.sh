#!/bin/bash
# connections per GPU with graph replay
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in "--streams 2" "--streams 3" "--streams 4" "--streams 2"; do
timeout -k 10 240 python bench.py --steps 30 --warmup 5 --no-rtt $v \
  > gpurun_out/r3b_get.json 2> gpurun_out/r3b_get.err \
  || { tail -20 gpurun_out/r3b_get.err; exit 1; }
echo "[$v]"; cut -c90-200 gpurun_out/r3b_get.json
done
