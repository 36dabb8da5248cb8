#!/bin/bash
# rocprofv3 kernel stats for the bench workloads: PROF=<tag> WORKLOADS=...
set -o pipefail
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $OUT
for w in ${WORKLOADS:-get mix storm}; do
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d $OUT/${PROF}_$w -o prof -- python3 $GRAFT_REPO_ROOT/bench.py \
    --workload $w --steps 5 --warmup 1 --no-rtt ${BENCH_ARGS:-} > $OUT/${PROF}_$w.log 2>&1
  rc=$?; echo "prof $w rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
