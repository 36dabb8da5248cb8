#!/bin/bash
# full GPU suite, then the default bench and the variable-size GET runs
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -x -v -m gpu --timeout 120 \
  --timeout-method thread > $OUT/r2e_tests.log 2>&1
rc=$?; tail -4 $OUT/r2e_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > $OUT/r2e_bench.log 2>&1
rc=$?; tail -1 $OUT/r2e_bench.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_r2d.sh
