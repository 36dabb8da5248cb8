#!/bin/bash
# fs_rows lengths from starts, single-block finish: full GPU tests, benches, profile
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests -m gpu > gpurun_out/r2l_tests.log 2>&1 || { tail -40 gpurun_out/r2l_tests.log; exit 1; }
tail -3 gpurun_out/r2l_tests.log
for w in get mix storm chain; do
timeout -k 10 240 python bench.py --workload $w --steps 20 --warmup 5 --no-rtt \
  > gpurun_out/r2l_$w.json 2> gpurun_out/r2l_$w.err \
  || { tail -20 gpurun_out/r2l_$w.err; exit 1; }
echo "[$w]"; cut -c90-220 gpurun_out/r2l_$w.json
done
timeout -k 10 240 python bench.py --steps 10 --warmup 3 --no-rtt --data-dist uniform:0-1024 \
  > gpurun_out/r2l_var.json 2> gpurun_out/r2l_var.err \
  || { tail -20 gpurun_out/r2l_var.err; exit 1; }
echo "[var]"; cut -c90-220 gpurun_out/r2l_var.json
PROF=r2v25 WORKLOADS="get" bash tools/prof_stats.sh
