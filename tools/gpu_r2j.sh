#!/bin/bash
# K1 fs_check: kernel tests, get bench (fixed + variable), profile
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_kernels.py tests/test_torch_ops.py tests/test_ordering.py -m gpu \
  > gpurun_out/r2j_tests.log 2>&1 \
  || { tail -40 gpurun_out/r2j_tests.log; exit 1; }
tail -3 gpurun_out/r2j_tests.log
timeout -k 10 240 python bench.py --steps 20 --warmup 5 --no-rtt \
  > gpurun_out/r2j_get.json 2> gpurun_out/r2j_get.err \
  || { tail -20 gpurun_out/r2j_get.err; exit 1; }
cut -c1-330 gpurun_out/r2j_get.json
timeout -k 10 240 python bench.py --steps 10 --warmup 3 --no-rtt --data-dist uniform:0-1024 \
  > gpurun_out/r2j_var.json 2> gpurun_out/r2j_var.err \
  || { tail -20 gpurun_out/r2j_var.err; exit 1; }
cut -c1-330 gpurun_out/r2j_var.json
PROF=r2v24 WORKLOADS="get" bash tools/prof_stats.sh
