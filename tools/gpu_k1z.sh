#!/bin/bash
# K1 over GET reply streams whose header zxid falls in byte ranges that
# read as frame lengths; each run under its own time limit.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
TAG=${TAG:-k1z}
for z in 0x100 0x1000005 0x8000005 0x20000005; do
  timeout -k 10 120 python tools/microbench/k1_bench.py --reps 3 --zxid $z \
    > $OUT/${TAG}_$z.log 2>&1
  rc=$?; echo "zxid $z rc=$rc"; grep -E "request|reply|EXACT|MISMATCH" $OUT/${TAG}_$z.log
  [ $rc -eq 0 ] || exit $rc
done
ZKMI_FS_DBG=1 timeout -k 10 120 python tools/microbench/k1_bench.py --reps 3 \
  --zxid 0x8000005 > $OUT/${TAG}_dbg.log 2>&1
rc=$?; tail -6 $OUT/${TAG}_dbg.log; exit $rc
