#!/bin/bash
# staggered streams: tests + get bench A/B
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_kernels.py -m gpu -k "pipeline or serve or tree" > gpurun_out/r2k_tests.log 2>&1 \
  || { tail -40 gpurun_out/r2k_tests.log; exit 1; }
tail -3 gpurun_out/r2k_tests.log
for v in "" "--no-stagger" "" "--no-stagger" "--streams 3" "--streams 4"; do
timeout -k 10 240 python bench.py --steps 30 --warmup 5 --no-rtt $v \
  > gpurun_out/r2k_get.json 2> gpurun_out/r2k_get.err \
  || { tail -20 gpurun_out/r2k_get.err; exit 1; }
echo "[$v]"; cut -c90-220 gpurun_out/r2k_get.json
done
