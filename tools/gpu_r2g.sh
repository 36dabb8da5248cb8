#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_kernels.py -k "frame_scan or pipeline" -m gpu > $OUT/r2g_tests.log 2>&1
rc=$?; tail -3 $OUT/r2g_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/diag/k1_var.py > $OUT/r2g_k1var.log 2>&1
rc=$?; cut -c1-200 $OUT/r2g_k1var.log | grep -v amdgpu.ids; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --no-rtt > $OUT/r2g_get.log 2>&1
rc=$?; tail -1 $OUT/r2g_get.log | cut -c1-250; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_r2d.sh
