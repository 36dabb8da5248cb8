#!/bin/bash
# One gpurun call: build check, full test suite (gpu + cpu), smoke, bench,
# rocprofv3 kernel stats.  Every GPU step has its own time limit and the
# chain stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 300 python -m pytest tests -x -q -m gpu > $OUT/gpu_tests.log 2>&1
rc=$?; tail -3 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
if [ -z "$SKIP_CPU" ]; then
  timeout -k 10 600 python -m pytest tests -x -q -m "not gpu" > $OUT/cpu_tests.log 2>&1
  rc=$?; tail -3 $OUT/cpu_tests.log; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; tail -1 $OUT/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py ${BENCH_ARGS:-} > $OUT/bench.log 2>&1
rc=$?; tail -1 $OUT/bench.log; [ $rc -eq 0 ] || exit $rc
if [ -n "$PROF" ]; then
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d $GRAFT_REPO_ROOT/$OUT/$PROF -o prof -- python3 $GRAFT_REPO_ROOT/bench.py \
    --steps 5 --warmup 1 --no-rtt > $GRAFT_REPO_ROOT/$OUT/$PROF.log 2>&1
  echo "prof rc=$?"
fi
