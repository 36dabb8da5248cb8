#!/bin/bash
# Round-4 validation on one GPU box: GPU tests, smoke, the headline bench
# (with RTT and bulk TCP), the forced-route RCCL GET, the other workloads,
# and a kernel-stats profile of GET.  Each GPU step has its own time limit;
# the chain stops at the first failure.  TAG names the outputs.
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
OUT=$R/gpurun_out
mkdir -p $OUT
TAG=${TAG:-r4}
step() {   # step <seconds> <log> <cmd...>
  local t=$1 log=$2; shift 2
  timeout -k 10 $t "$@" > $OUT/${TAG}_$log.log 2>&1
  local rc=$?; echo "== $log rc=$rc"; tail -${TAILN:-2} $OUT/${TAG}_$log.log
  [ $rc -eq 0 ] || exit $rc
}
if [ -z "$NO_TESTS" ]; then
  TAILN=4 step 420 gpu_tests python -u -m pytest tests -x -q -m gpu \
    --timeout 120 --timeout-method thread
fi
step 200 smoke python -c "import __graft_entry__ as g; g.smoke()"
step 300 bench python bench.py
step 200 bench_route python bench.py --no-rtt --force-route
step 200 bench_var python bench.py --no-rtt --data-dist uniform:0-1024
step 200 bench_512 python bench.py --no-rtt --data-bytes 512
for w in ${WORKLOADS:-mix storm watch chain nest}; do
  step 200 bench_$w python bench.py --no-rtt --workload $w
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
  -d $OUT/${TAG}_prof_get -o prof -- python3 $R/bench.py \
  --steps 5 --warmup 1 --no-rtt > $OUT/${TAG}_prof_get.log 2>&1
echo "prof rc=$?"
