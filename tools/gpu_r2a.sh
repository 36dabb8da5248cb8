#!/bin/bash
# round-2 checks: new GPU tests, sharded / ensemble benches, a 2-rank gloo
# rehearsal of the sharded bench on the one GPU.  Each step time-limited.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_sharded.py tests/test_ensemble.py -m gpu > $OUT/r2a_tests.log 2>&1
rc=$?; tail -5 $OUT/r2a_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --no-rtt --workload get --sharded > $OUT/r2a_sharded1.log 2>&1
rc=$?; tail -1 $OUT/r2a_sharded1.log; [ $rc -eq 0 ] || exit $rc
ZKMI_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29555 bench.py --no-rtt \
  --workload get --sharded --batch 262144 --steps 5 > $OUT/r2a_sharded2g.log 2>&1
rc=$?; tail -1 $OUT/r2a_sharded2g.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --workload ensemble --steps 8 --warmup 1 > $OUT/r2a_ens.log 2>&1
rc=$?; tail -1 $OUT/r2a_ens.log; [ $rc -eq 0 ] || exit $rc
