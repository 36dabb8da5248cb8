#!/bin/bash
# K1 unmapped-tile walk: the K1 GPU tests (dense length words, length-like
# zxids, repair), GET and mix microbenchmarks; each step under its own limit.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
TAG=${TAG:-k1w}
timeout -k 10 300 python -u -m pytest tests/test_frame_repair.py tests/test_kernels.py \
  -x -v -s -m gpu --timeout 120 --timeout-method thread > $OUT/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "FAIL|Error|assert|group .:" $OUT/${TAG}_tests.log | tail -12; tail -2 $OUT/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/microbench/k1_bench.py > $OUT/${TAG}_get.log 2>&1
rc=$?; echo "get rc=$rc"; tail -3 $OUT/${TAG}_get.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/microbench/k1_bench.py --workload mix --reps 5 --zxid 0x8000005 > $OUT/${TAG}_mix.log 2>&1
rc=$?; echo "mix rc=$rc"; tail -3 $OUT/${TAG}_mix.log; exit $rc
