#!/bin/bash
# Kernel stats of the GET step with uniform 0-1024 B payloads and with fixed
# 512 B ones; each profile under its own time limit.
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
OUT=$R/gpurun_out
mkdir -p $OUT
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/vp_var -o prof \
  -- python3 $R/bench.py --steps 10 --warmup 2 --no-rtt --no-sustain --data-dist uniform:0-1024 \
  > $OUT/vp_var.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/vp_512 -o prof \
  -- python3 $R/bench.py --steps 10 --warmup 2 --no-rtt --no-sustain --data-bytes 512 \
  > $OUT/vp_512.log 2>&1 || exit $?

timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/vp_storm -o prof \
  -- python3 $R/bench.py --steps 10 --warmup 2 --no-rtt --no-sustain --workload storm \
  > $OUT/vp_storm.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/vp_chain -o prof \
  -- python3 $R/bench.py --steps 10 --warmup 2 --no-rtt --no-sustain --workload chain \
  > $OUT/vp_chain.log 2>&1 || exit $?
echo done2
