#!/bin/bash
# fs_link A/B on the link-repair streams: tools/fl_ab.sh VAR "V1 V2" "CASES"
# (each probe under its own time limit; the first failure ends the run)
set -o pipefail
VAR=$1; VALS=${2:-"1 0"}; CASES=${3:-"period phantom dense1 nospec"}
mkdir -p gpurun_out
for v in $VALS; do
  for c in $CASES; do
    echo "== $VAR=$v $c"
    env $VAR=$v ZKMI_FS_DBG=1 timeout -k 10 120 python -u \
      tools/microbench/fl_probe.py --case $c --reps 3 > gpurun_out/fl_ab_run.log 2>&1 \
      || { tail -20 gpurun_out/fl_ab_run.log; exit 1; }
    grep -v amdgpu.ids gpurun_out/fl_ab_run.log | tail -2
  done
done
