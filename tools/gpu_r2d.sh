#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
for d in "uniform:0-200" "uniform:0-1024"; do
  timeout -k 10 200 python bench.py --no-rtt --data-dist $d --name-pad 0-16 \
    > $OUT/r2d_var_${d#uniform:}.log 2>&1
  rc=$?; tail -1 $OUT/r2d_var_${d#uniform:}.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 200 python bench.py --no-rtt --data-bytes 512 > $OUT/r2d_fixed512.log 2>&1
rc=$?; tail -1 $OUT/r2d_fixed512.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc
