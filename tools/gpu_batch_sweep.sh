#!/bin/bash
# GET throughput vs requests per step (1 GPU, graph replay, 1M-znode tree).
set -o pipefail
OUT=gpurun_out/bsweep
mkdir -p $OUT
for b in 262144 524288 1048576 2097152 4194304; do
  timeout -k 10 150 python bench.py --no-rtt --batch $b --steps 30 --warmup 3 \
    > $OUT/b$b.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "batch $b rc=$rc"; tail -5 $OUT/b$b.log; exit $rc; }
  echo "batch $b $(tail -1 $OUT/b$b.log | python tools/ms_per_step.py) ms"
done
