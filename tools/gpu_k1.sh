#!/bin/bash
# K1 A/B on one GPU box: the frame-scan microbenchmark (tools/microbench/
# k1_bench.py) over the GET streams for the tree in ab_old/ (if present)
# and this one, the phase clock, a kernel-stats profile and the K1 tests.
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
OUT=$R/gpurun_out
mkdir -p $OUT
TAG=${TAG:-k1}
if [ -d ab_old ]; then
  (cd ab_old && timeout -k 10 180 python tools/microbench/k1_bench.py $K1ARGS \
    > $OUT/${TAG}_old.log 2>&1)
  rc=$?; tail -4 $OUT/${TAG}_old.log; [ $rc -eq 0 ] || exit $rc
  (cd ab_old && ZKMI_FS_DBG=1 timeout -k 10 180 \
    python tools/microbench/k1_bench.py --reps 3 $K1ARGS \
    > $OUT/${TAG}_old_dbg.log 2>&1)
  rc=$?; tail -6 $OUT/${TAG}_old_dbg.log; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 180 python tools/microbench/k1_bench.py $K1ARGS > $OUT/${TAG}_new.log 2>&1
rc=$?; tail -4 $OUT/${TAG}_new.log; [ $rc -eq 0 ] || exit $rc
ZKMI_FS_DBG=1 timeout -k 10 180 python tools/microbench/k1_bench.py --reps 3 $K1ARGS \
    > $OUT/${TAG}_new_dbg.log 2>&1
rc=$?; tail -6 $OUT/${TAG}_new_dbg.log; [ $rc -eq 0 ] || exit $rc
for g in 1 2; do
  timeout -k 10 180 python tools/microbench/k1_bench.py --group $g $K1ARGS \
    > $OUT/${TAG}_g$g.log 2>&1
  rc=$?; tail -3 $OUT/${TAG}_g$g.log; [ $rc -eq 0 ] || exit $rc
done
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats \
  --output-format csv -d $OUT/${TAG}_prof -o prof -- \
  python3 $R/tools/microbench/k1_bench.py --reps 10 $K1ARGS \
  > $OUT/${TAG}_prof.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd $R
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 300 python -u -m pytest tests/test_frame_repair.py \
    tests/test_kernels.py -x -q -m gpu --timeout 120 \
    --timeout-method thread > $OUT/${TAG}_tests.log 2>&1
  rc=$?; tail -5 $OUT/${TAG}_tests.log; exit $rc
fi
