#!/bin/bash
# Interactive-path A/B on a GPU box: the native completion path (reply
# router + coalesced writes) against the Python path, alternated so box
# drift hits both; then the bench's conditions (1M-node server, GPU
# initialised in the process).  Output: gpurun_out/rtt_ab.log
set -o pipefail
mkdir -p gpurun_out
OUT=gpurun_out/rtt_ab.log
: > $OUT
for i in 1 2 3; do
  for cfg in "1 1" "0 0" "1 0"; do
    set -- $cfg
    ZKMI_LOOP_CORK=$1 ZKMI_ROUTE=$2 timeout -k 10 120 python tools/rtt_cpu.py \
      --n 20000 >> $OUT 2>&1 || exit $?
  done
done
timeout -k 10 200 python tools/rtt_cpu.py --n 20000 --nodes 1000000 >> $OUT 2>&1 || exit $?
timeout -k 10 200 python tools/rtt_cpu.py --n 20000 --nodes 1000000 \
  --torch-gpu >> $OUT 2>&1 || exit $?
cat $OUT
