#!/bin/bash
# ordering tests + chain profile
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_ordering.py -m gpu > gpurun_out/r2i_tests.log 2>&1 \
  || { tail -40 gpurun_out/r2i_tests.log; exit 1; }
tail -3 gpurun_out/r2i_tests.log
timeout -k 10 240 python bench.py --workload chain --steps 10 --warmup 3 --no-rtt \
  > gpurun_out/r2i_chain.json 2> gpurun_out/r2i_chain.err \
  || { tail -20 gpurun_out/r2i_chain.err; exit 1; }
cat gpurun_out/r2i_chain.json
PROF=r2v23 WORKLOADS="chain" bash tools/prof_stats.sh
