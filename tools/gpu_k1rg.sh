#!/bin/bash
# Request-stream groups on the mix workload's requests (creates / sets with
# 100-byte data, deletes); each run under its own time limit.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
for g in 1 2 4 8; do
  timeout -k 10 120 python tools/microbench/k1_bench.py --workload mix --req-group $g --reps 5 \
    > $OUT/k1rg_$g.log 2>&1 || exit $?
  echo "req-group $g: $(grep request $OUT/k1rg_$g.log)"
done
