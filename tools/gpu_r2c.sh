#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_bulk.py tests/test_kernels.py -k "bulk or storm or handshake" \
  -m gpu > $OUT/r2c_tests.log 2>&1
rc=$?; tail -5 $OUT/r2c_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > $OUT/r2c_bench.log 2>&1
rc=$?; tail -1 $OUT/r2c_bench.log; [ $rc -eq 0 ] || exit $rc
