#!/bin/bash
# fs_tile tiles per workgroup A/B (ZKMI_FS_TPB)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for t in 4 2 1 4; do
ZKMI_FS_TPB=$t timeout -k 10 240 python bench.py --steps 30 --warmup 5 --no-rtt \
  > gpurun_out/r3h_get.json 2> gpurun_out/r3h_get.err \
  || { tail -20 gpurun_out/r3h_get.err; exit 1; }
echo "[tpb=$t]"; cut -c90-200 gpurun_out/r3h_get.json
done
