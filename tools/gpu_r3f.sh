#!/bin/bash
# block-sum scan folded into the writers: full GPU tests + bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests -m gpu > gpurun_out/r3f_tests.log 2>&1 || { tail -40 gpurun_out/r3f_tests.log; exit 1; }
tail -2 gpurun_out/r3f_tests.log
for v in "" "" "--workload mix" "--workload storm"; do
timeout -k 10 240 python bench.py --steps 30 --warmup 5 --no-rtt $v \
  > gpurun_out/r3f_get.json 2> gpurun_out/r3f_get.err \
  || { tail -20 gpurun_out/r3f_get.err; exit 1; }
echo "[$v]"; cut -c90-200 gpurun_out/r3f_get.json
done
