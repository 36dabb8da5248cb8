#!/bin/bash
# GET: connection 0 on a high-priority stream or not, alternating, each run
# under its own time limit.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
for r in 1 2; do
  for m in base prio; do
    extra=""; [ $m = prio ] && extra="--stream-priority"
    timeout -k 10 150 python bench.py --no-rtt $extra > $OUT/prio_${m}_$r.log 2>&1 || exit $?
    python3 -c "
import json; d=json.loads(open('$OUT/prio_${m}_$r.log').read().strip().split('\n')[-1])
print('%-5s %d %.4f ms/step sustained %.4f' % ('$m', $r, d['ms_per_step'], d['sustained']['ms_per_step']))"
  done
done
for g in 8 4; do
  timeout -k 10 120 python tools/microbench/k1_bench.py --group $g > $OUT/k1g${g}.log 2>&1 || exit $?
  echo "group $g: $(grep reply $OUT/k1g${g}.log)"
done
bash tools/gpu_varprof.sh
