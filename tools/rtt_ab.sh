#!/bin/bash
# Interactive-path A/B of an environment switch (tools/rtt_cpu.py after GPU
# init, as bench.py runs it), alternated ROUNDS times:
#   RTT_VAR=ZKMI_SYNC_WAITER RTT_VALUES="1 0" bash tools/rtt_ab.sh
set -o pipefail
mkdir -p gpurun_out
OUT=gpurun_out/rtt_ab_${RTT_VAR}.log
: > $OUT
for i in $(seq ${ROUNDS:-3}); do
  for v in ${RTT_VALUES:-1 0}; do
    echo -n "$RTT_VAR=$v " >> $OUT
    env $RTT_VAR=$v timeout -k 10 120 python tools/rtt_cpu.py --torch-gpu \
      2>/dev/null | tail -1 >> $OUT || exit 1
  done
done
cat $OUT
