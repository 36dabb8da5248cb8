#!/bin/bash
# batched payload loads in the reply writer: tests, fixed/variable GET
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_kernels.py tests/test_torch_ops.py tests/test_ordering.py tests/test_bulk.py -m gpu \
  > gpurun_out/r2t_tests.log 2>&1 \
  || { tail -40 gpurun_out/r2t_tests.log; exit 1; }
tail -2 gpurun_out/r2t_tests.log
for v in "" "--data-bytes 512" "--data-dist uniform:0-1024" "--data-dist uniform:0-200"; do
timeout -k 10 240 python bench.py --steps 20 --warmup 3 --no-rtt $v \
  > gpurun_out/r2t_get.json 2> gpurun_out/r2t_get.err \
  || { tail -20 gpurun_out/r2t_get.err; exit 1; }
echo "[$v]"; cut -c90-220 gpurun_out/r2t_get.json
done
PROF=r2v30v BENCH_ARGS="--data-dist uniform:0-1024" WORKLOADS="get" bash tools/prof_stats.sh
