#!/bin/bash
# A/B of two kernel-library builds on the default GET bench: the .so is
# swapped between runs (ab/libzkmi_hip_{base,xcd}.so), runs alternate.
set -o pipefail
OUT=gpurun_out/ab
mkdir -p $OUT
timeout -k 10 200 python -m pytest tests/test_kernels.py -x -q -m gpu > $OUT/tests.log 2>&1
rc=$?; tail -1 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for v in base xcd; do
    cp ab/libzkmi_hip_$v.so zkmi/ops/libzkmi_hip.so || exit 1
    timeout -k 10 120 python bench.py --no-rtt --steps 50 --warmup 5 \
      > $OUT/$v$r.log 2>&1
    rc=$?; [ $rc -eq 0 ] || exit $rc
    echo "$v $r $(tail -1 $OUT/$v$r.log | python tools/ms_per_step.py)"
    for w in mix storm; do
      timeout -k 10 120 python bench.py --no-rtt --workload $w --steps 30 \
        --warmup 3 > $OUT/$v$r$w.log 2>&1
      rc=$?; [ $rc -eq 0 ] || exit $rc
      echo "$v $r $w $(tail -1 $OUT/$v$r$w.log | python tools/ms_per_step.py)"
    done
  done
done
