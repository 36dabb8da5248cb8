#!/bin/bash
# late-exit candidates first: K1 tests, fixed/variable GET
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_kernels.py tests/test_torch_ops.py -m gpu \
  > gpurun_out/r3q_tests.log 2>&1 || { tail -40 gpurun_out/r3q_tests.log; exit 1; }
tail -2 gpurun_out/r3q_tests.log
for v in "" "--data-bytes 512" "--data-dist uniform:0-1024" "--data-dist uniform:0-200"; do
timeout -k 10 240 python bench.py --steps 20 --warmup 3 --no-rtt $v \
  > gpurun_out/r3q_get.json 2> gpurun_out/r3q_get.err \
  || { tail -20 gpurun_out/r3q_get.err; exit 1; }
echo "[$v]"; cut -c90-200 gpurun_out/r3q_get.json
done
