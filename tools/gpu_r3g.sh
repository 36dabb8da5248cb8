#!/bin/bash
# encoder writers at 5 waves/SIMD (launch bounds): K13/K10 tests + benches
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_kernels.py -m gpu > gpurun_out/r3g_tests.log 2>&1 \
  || { tail -40 gpurun_out/r3g_tests.log; exit 1; }
tail -2 gpurun_out/r3g_tests.log
for v in "" "" "--workload mix" "--data-bytes 512"; do
timeout -k 10 240 python bench.py --steps 30 --warmup 5 --no-rtt $v \
  > gpurun_out/r3g_get.json 2> gpurun_out/r3g_get.err \
  || { tail -20 gpurun_out/r3g_get.err; exit 1; }
echo "[$v]"; cut -c90-200 gpurun_out/r3g_get.json
done
