#!/bin/bash
# Kernel trace of the watch workload over its first slow step (step ~90 from
# a fresh tree), eager; under its own time limit.
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
OUT=$R/gpurun_out
mkdir -p $OUT
cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $OUT/wt_trace -o tr \
  -- python3 $R/tools/microbench/sustain_probe.py --workload watch --steps 100 --chunk 20 --eager \
  > $OUT/wt_trace.log 2>&1
echo "trace rc=$?"
