#!/bin/bash
# K1 node-filter check: the mix streams at both zxids, the K1 GPU tests,
# the long-run step times; each step under its own time limit.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
TAG=${TAG:-k1f}
for z in 0x100 0x8000005; do
  timeout -k 10 120 python tools/microbench/k1_bench.py --workload mix --reps 5 --zxid $z \
    > $OUT/${TAG}_mix_$z.log 2>&1
  rc=$?; echo "mix zxid $z rc=$rc"; grep -E "request|reply|EXACT|MISMATCH|Error" $OUT/${TAG}_mix_$z.log
  [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 120 python tools/microbench/k1_bench.py > $OUT/${TAG}_get.log 2>&1
rc=$?; echo "get rc=$rc"; tail -3 $OUT/${TAG}_get.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_frame_repair.py tests/test_kernels.py \
  -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $OUT/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
P=tools/microbench/sustain_probe.py
timeout -k 10 150 python -u $P --workload mix --steps 400 > $OUT/${TAG}_sus_mix.log 2>&1 || exit $?
timeout -k 10 150 python -u $P --workload watch --steps 40 --chunk 4 > $OUT/${TAG}_sus_watch.log 2>&1 || exit $?
timeout -k 10 200 python -u $P --workload nest --steps 200 --chunk 20 > $OUT/${TAG}_sus_nest.log 2>&1 || exit $?
timeout -k 10 150 python -u $P --workload chain --steps 200 --chunk 20 > $OUT/${TAG}_sus_chain.log 2>&1 || exit $?
echo sustain ok
