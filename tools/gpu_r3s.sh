#!/bin/bash
# candidate alive walk reads issued together: K1 tests, phase timing, get bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_kernels.py -m gpu > gpurun_out/r3s_tests.log 2>&1 \
  || { tail -40 gpurun_out/r3s_tests.log; exit 1; }
tail -2 gpurun_out/r3s_tests.log
timeout -k 10 200 python tools/diag/k1_dbg.py > gpurun_out/r3s_k1dbg.log 2>&1 \
  || { tail -20 gpurun_out/r3s_k1dbg.log; exit 1; }
grep -E "tiles|survivor|wait|walk|end " gpurun_out/r3s_k1dbg.log
for v in "" ""; do
timeout -k 10 240 python bench.py --steps 30 --warmup 5 --no-rtt $v \
  > gpurun_out/r3s_get.json 2> gpurun_out/r3s_get.err \
  || { tail -20 gpurun_out/r3s_get.err; exit 1; }
cut -c90-200 gpurun_out/r3s_get.json
done
