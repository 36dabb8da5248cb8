#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_kernels.py -k "frame_scan or pipeline" -m gpu > $OUT/r2f_tests.log 2>&1
rc=$?; tail -4 $OUT/r2f_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_r2d.sh
