#!/bin/bash
# rocprofv3 kernel stats for the storm and chain workloads (kernel trace
# only, one run each, own time limit).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for w in storm chain; do
  cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv \
    -d $R/gpurun_out/prof_$w -o prof -- python3 $R/bench.py --workload $w \
    --steps 5 --warmup 1 --no-rtt > $R/gpurun_out/prof_$w.log 2>&1
  rc=$?; echo "$w rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
