#!/bin/bash
# frontier floor 16 and 32 (reply-only streams)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_kernels.py tests/test_torch_ops.py -m gpu > gpurun_out/r2v_tests.log 2>&1 \
  || { tail -40 gpurun_out/r2v_tests.log; exit 1; }
tail -2 gpurun_out/r2v_tests.log
for m in 16 32; do
for v in "" "--data-bytes 512" "--data-dist uniform:0-1024"; do
ZKMI_FS_MINB=$m timeout -k 10 240 python bench.py --steps 20 --warmup 3 --no-rtt $v \
  > gpurun_out/r2v_get.json 2> gpurun_out/r2v_get.err \
  || { tail -20 gpurun_out/r2v_get.err; exit 1; }
echo "[minb=$m $v]"; cut -c90-200 gpurun_out/r2v_get.json
done
done
