#!/bin/bash
# K1 reply scan with groups of 8 vs 4 tiles, then the payload / write
# workload profiles; each step under its own time limit.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
for g in 8 4; do
  timeout -k 10 120 python tools/microbench/k1_bench.py --group $g > $OUT/k1g${g}.log 2>&1 || exit $?
  echo "group $g: $(grep reply $OUT/k1g${g}.log)"
done
bash tools/gpu_varprof.sh
