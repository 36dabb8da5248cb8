#!/bin/bash
# request parse fused into tree_serve: tests + benches
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests -m gpu > gpurun_out/r2p_tests.log 2>&1 || { tail -40 gpurun_out/r2p_tests.log; exit 1; }
tail -2 gpurun_out/r2p_tests.log
for w in get get mix storm chain; do
timeout -k 10 240 python bench.py --workload $w --steps 30 --warmup 5 --no-rtt \
  > gpurun_out/r2p_$w.json 2> gpurun_out/r2p_$w.err \
  || { tail -20 gpurun_out/r2p_$w.err; exit 1; }
echo "[$w]"; cut -c90-220 gpurun_out/r2p_$w.json
done
