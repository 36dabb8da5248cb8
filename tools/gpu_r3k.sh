#!/bin/bash
# interactive RTT: loop busy-poll (default on here) x call_sync poll window
set -o pipefail
mkdir -p gpurun_out
for s in 0 30 100 0 30; do
ZKMI_SYNC_SPIN_US=$s timeout -k 10 120 python tools/diag/rtt_cmp.py > gpurun_out/r3k_rtt.log 2>&1 \
  || { tail -5 gpurun_out/r3k_rtt.log; exit 1; }
echo "[sync_spin=$s]"; cat gpurun_out/r3k_rtt.log
done
