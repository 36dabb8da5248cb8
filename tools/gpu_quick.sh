#!/bin/bash
# GPU tests + the three bench workloads, each step under its own limit; the
# chain stops at the first failure.  BENCH_ARGS is passed to every bench.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 \
    --timeout-method thread > $OUT/gpu_tests.log 2>&1
  rc=$?; tail -3 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
fi
for w in ${WORKLOADS:-get mix storm}; do
  timeout -k 10 300 python bench.py --no-rtt --workload $w ${BENCH_ARGS:-} \
    > $OUT/bench_$w.log 2>&1
  rc=$?; tail -2 $OUT/bench_$w.log; [ $rc -eq 0 ] || exit $rc
done
