#!/bin/bash
# Blocking call_sync round trips: requests sent from the caller's thread
# (request_direct, default) vs hopping to the loop thread first
# (ZKMI_DIRECT=0), alternated.  Output: gpurun_out/direct_ab.log
set -o pipefail
mkdir -p gpurun_out
OUT=gpurun_out/direct_ab.log
: > $OUT
for i in 1 2 3; do
  for d in 1 0; do
    echo -n "direct=$d " >> $OUT
    ZKMI_DIRECT=$d timeout -k 10 120 python tools/rtt_cpu.py --n 20000 \
      >> $OUT 2>&1 || exit $?
  done
done
cat $OUT
