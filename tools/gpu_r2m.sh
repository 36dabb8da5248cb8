#!/bin/bash
# survivor loop streamlining: K1 tests, per-phase timing, get bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_kernels.py tests/test_torch_ops.py -m gpu > gpurun_out/r2m_tests.log 2>&1 \
  || { tail -40 gpurun_out/r2m_tests.log; exit 1; }
tail -2 gpurun_out/r2m_tests.log
timeout -k 10 200 python tools/diag/k1_dbg.py > gpurun_out/r2m_k1dbg.log 2>&1 \
  || { tail -20 gpurun_out/r2m_k1dbg.log; exit 1; }
grep -E "tiles|survivor|frontier|end " gpurun_out/r2m_k1dbg.log
for v in get get; do
timeout -k 10 240 python bench.py --steps 30 --warmup 5 --no-rtt \
  > gpurun_out/r2m_get.json 2> gpurun_out/r2m_get.err \
  || { tail -20 gpurun_out/r2m_get.err; exit 1; }
cut -c90-220 gpurun_out/r2m_get.json
done
timeout -k 10 240 python bench.py --steps 10 --warmup 3 --no-rtt --data-dist uniform:0-1024 \
  > gpurun_out/r2m_var.json 2> gpurun_out/r2m_var.err \
  || { tail -20 gpurun_out/r2m_var.err; exit 1; }
cut -c90-220 gpurun_out/r2m_var.json
