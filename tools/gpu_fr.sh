#!/bin/bash
# Forced-route RCCL capture probes: one rank, one GPU, each in a fresh
# process under its own time limit; stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 200 python bench.py --no-rtt --force-route --streams 1 > $OUT/fr_bench1.log 2>&1 || { echo "bench1 rc=$?"; tail -c 1500 $OUT/fr_bench1.log; exit 1; }
echo "bench1 rc=$?"; tail -c 600 $OUT/fr_bench1.log
timeout -k 10 200 python -u -m pytest tests/test_sharded.py -x -v -k "forced_route and 2" \
  --timeout 120 --timeout-method thread > $OUT/fr_t2.log 2>&1 || { echo "t2 rc=$?"; exit 1; }
echo t2 ok
timeout -k 10 200 python bench.py --no-rtt --force-route > $OUT/fr_bench2.log 2>&1
echo "bench2 rc=$?"; tail -c 600 $OUT/fr_bench2.log
