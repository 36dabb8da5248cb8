#!/bin/bash
# K1 over the mix workload's streams, at a small zxid and inside the slow
# range; each run under its own time limit.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
TAG=${TAG:-k1m}
for z in 0x100 0x8000005; do
  timeout -k 10 120 python tools/microbench/k1_bench.py --workload mix --reps 2 --zxid $z \
    > $OUT/${TAG}_$z.log 2>&1
  rc=$?; echo "zxid $z rc=$rc"; grep -E "request|reply|EXACT|MISMATCH|Error" $OUT/${TAG}_$z.log
  [ $rc -eq 0 ] || exit $rc
  ZKMI_FS_DBG=1 timeout -k 10 120 python tools/microbench/k1_bench.py --workload mix \
    --reps 1 --zxid $z > $OUT/${TAG}_dbg_$z.log 2>&1
  rc=$?; tail -6 $OUT/${TAG}_dbg_$z.log; [ $rc -eq 0 ] || exit $rc
done
