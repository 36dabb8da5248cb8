#!/bin/bash
# Watch workload slow steps: chunked step times from a zxid inside the
# slow stretch, then kernel stats there; each step under its own limit.
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
OUT=$R/gpurun_out
mkdir -p $OUT
P=$R/tools/microbench/sustain_probe.py
timeout -k 10 150 python -u $P --workload watch --steps 60 --chunk 5 --zxid 0xA000000 > $OUT/wp_sus.log 2>&1 || exit $?
grep steps $OUT/wp_sus.log | cut -c1-60
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/wp_prof -o prof \
  -- python3 $P --workload watch --steps 20 --chunk 5 --zxid 0xA000000 --eager > $OUT/wp_prof.log 2>&1
echo "prof rc=$?"
