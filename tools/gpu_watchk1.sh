#!/bin/bash
# The watch step whose notification scan needs the long repair: its K1
# counters and stream shape; under its own time limit.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 300 python -u tools/microbench/watch_k1_probe.py --steps 120 > $OUT/wk1.log 2>&1
rc=$?; cut -c1-300 $OUT/wk1.log | tail -12; exit $rc
