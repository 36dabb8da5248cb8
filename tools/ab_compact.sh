#!/bin/bash
# ZKMI_FREE_COMPACT on / off per write workload (gpurun_out/ab_compact_<wl>.log)
set -o pipefail
for wl in ${WLS:-mix nest storm}; do
  AB_TAG=compact_$wl AB_VAR=ZKMI_FREE_COMPACT AB_VALUES="1 0" ROUNDS=2 BENCH_ARGS="--workload $wl" bash tools/gpu_ab_env.sh > gpurun_out/ab_compact_run.log 2>&1 || exit 1
done
