#!/bin/bash
# frontier minimum body length: K1 tests, A/B on fixed/variable GET
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_kernels.py tests/test_torch_ops.py -m gpu > gpurun_out/r2u_tests.log 2>&1 \
  || { tail -40 gpurun_out/r2u_tests.log; exit 1; }
tail -2 gpurun_out/r2u_tests.log
for m in 8 0; do
for v in "" "--data-bytes 512" "--data-dist uniform:0-1024"; do
ZKMI_FS_MINB=$m timeout -k 10 240 python bench.py --steps 20 --warmup 3 --no-rtt $v \
  > gpurun_out/r2u_get.json 2> gpurun_out/r2u_get.err \
  || { tail -20 gpurun_out/r2u_get.err; exit 1; }
echo "[minb=$m $v]"; cut -c90-200 gpurun_out/r2u_get.json
done
done
