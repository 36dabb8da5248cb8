#!/bin/bash
# interactive RTT: native loop busy-poll window A/B (no GPU work)
set -o pipefail
mkdir -p gpurun_out
for s in 0 50 0 50 200; do
ZKMI_LOOP_SPIN_US=$s timeout -k 10 120 python tools/diag/rtt_cmp.py > gpurun_out/r3j_rtt.log 2>&1 \
  || { tail -5 gpurun_out/r3j_rtt.log; exit 1; }
echo "[spin=$s]"; cat gpurun_out/r3j_rtt.log
done
