#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_kernels.py -k "storm or handshake" -m gpu > $OUT/r2b_tests.log 2>&1
rc=$?; tail -5 $OUT/r2b_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --no-rtt --workload storm > $OUT/r2b_storm.log 2>&1
rc=$?; tail -1 $OUT/r2b_storm.log; [ $rc -eq 0 ] || exit $rc
