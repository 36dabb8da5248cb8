#!/bin/bash
# K1 on the variable-payload reply stream (long-frame mode at a 1 KiB window
# vs a 2 KiB window), then the GPU tests and the headline bench with 8-tile
# groups; each step under its own time limit.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
for w in 1024 2048; do
  timeout -k 10 150 python tools/microbench/k1_bench.py --data-dist 0-1024 --win-max $w --reps 5 \
    > $OUT/k1v_$w.log 2>&1 || exit $?
  echo "win-max $w:"; grep -E "request|reply|EXACT|MISMATCH" $OUT/k1v_$w.log
done
timeout -k 10 420 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread \
  > $OUT/r4d_gpu_tests.log 2>&1 || { tail -30 $OUT/r4d_gpu_tests.log; exit 1; }
tail -2 $OUT/r4d_gpu_tests.log
timeout -k 10 200 python bench.py --no-rtt > $OUT/r4d_bench.log 2>&1 || exit $?
python3 -c "
import json; d=json.loads(open('$OUT/r4d_bench.log').read().strip().split('\n')[-1])
print('bench %.4f ms/step sustained %.4f' % (d['ms_per_step'], d['sustained']['ms_per_step']))"
for v in "--data-bytes 512" "--data-dist uniform:0-1024"; do
  timeout -k 10 200 python bench.py --no-rtt --no-sustain $v > $OUT/r4d_var.log 2>&1 || exit $?
  python3 -c "
import json; d=json.loads(open('$OUT/r4d_var.log').read().strip().split('\n')[-1])
print('bench $v %.4f ms/step' % d['ms_per_step'])"
done
