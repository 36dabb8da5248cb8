#!/bin/bash
# GPU tests, then the three bench workloads (get / mix / storm), then an
# optional rocprofv3 kernel-stats run per workload (PROF=<tag>).  Each GPU
# step has its own time limit; the chain stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 300 python -m pytest tests -x -q -m gpu > $OUT/gpu_tests.log 2>&1
rc=$?; tail -3 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
for w in get mix storm; do
  timeout -k 10 300 python bench.py --no-rtt --workload $w ${BENCH_ARGS:-} > $OUT/bench_$w.log 2>&1
  rc=$?; tail -2 $OUT/bench_$w.log; [ $rc -eq 0 ] || exit $rc
done
if [ -n "$PROF" ]; then
  for w in get mix storm; do
    cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
      -d $GRAFT_REPO_ROOT/$OUT/${PROF}_$w -o prof -- python3 $GRAFT_REPO_ROOT/bench.py \
      --workload $w --steps 5 --warmup 1 --no-rtt > $GRAFT_REPO_ROOT/$OUT/${PROF}_$w.log 2>&1
    rc=$?; echo "prof $w rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
fi
