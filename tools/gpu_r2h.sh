#!/bin/bash
# ordering tests, then chain / mix / get bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_ordering.py tests/test_kernels.py -m gpu > gpurun_out/r2h_tests.log 2>&1 \
  || { tail -40 gpurun_out/r2h_tests.log; exit 1; }
tail -3 gpurun_out/r2h_tests.log
timeout -k 10 240 python bench.py --workload chain --steps 10 --warmup 3 --no-rtt \
  > gpurun_out/r2h_chain.json 2> gpurun_out/r2h_chain.err \
  || { tail -20 gpurun_out/r2h_chain.err; exit 1; }
cat gpurun_out/r2h_chain.json
timeout -k 10 240 python bench.py --workload mix --steps 10 --warmup 3 --no-rtt \
  > gpurun_out/r2h_mix.json 2> gpurun_out/r2h_mix.err \
  || { tail -20 gpurun_out/r2h_mix.err; exit 1; }
cat gpurun_out/r2h_mix.json
timeout -k 10 240 python bench.py --steps 20 --warmup 5 --no-rtt \
  > gpurun_out/r2h_get.json 2> gpurun_out/r2h_get.err \
  || { tail -20 gpurun_out/r2h_get.err; exit 1; }
cat gpurun_out/r2h_get.json
