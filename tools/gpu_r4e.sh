#!/bin/bash
# The 2 KiB automatic K1 window: the K1 / K13 GPU tests, the GET payload
# variants and the headline; each step under its own time limit.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_frame_repair.py tests/test_kernels.py -x -q -m gpu \
  --timeout 120 --timeout-method thread > $OUT/r4e_tests.log 2>&1 || { tail -30 $OUT/r4e_tests.log; exit 1; }
tail -1 $OUT/r4e_tests.log
timeout -k 10 150 python tools/microbench/k1_bench.py --data-dist 0-1024 --reps 5 > $OUT/r4e_k1v.log 2>&1 || exit $?
grep reply $OUT/r4e_k1v.log
for v in "" "--data-bytes 512" "--data-dist uniform:0-1024" "--data-dist uniform:0-200"; do
  timeout -k 10 200 python bench.py --no-rtt $v > $OUT/r4e_b.log 2>&1 || exit $?
  python3 -c "
import json; d=json.loads(open('$OUT/r4e_b.log').read().strip().split('\n')[-1])
print('bench [$v] %.4f ms/step sustained %.4f value %.4g' % (d['ms_per_step'], d['sustained']['ms_per_step'], d['value']))"
done
