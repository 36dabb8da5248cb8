#!/bin/bash
# GET connections per GPU with 8-tile groups; the watch workload's long run
# eager and replayed; each step under its own time limit.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
for s in 2 3 4 2; do
  timeout -k 10 150 python bench.py --no-rtt --no-sustain --streams $s > $OUT/r4g_s.log 2>&1 || exit $?
  python3 -c "
import json; d=json.loads(open('$OUT/r4g_s.log').read().strip().split('\n')[-1])
print('streams $s %.4f ms/step' % d['ms_per_step'])"
done
P=tools/microbench/sustain_probe.py
timeout -k 10 200 python -u $P --workload watch --steps 240 --chunk 20 > $OUT/r4g_w.log 2>&1 || exit $?
echo graph; grep steps $OUT/r4g_w.log | cut -c1-40
timeout -k 10 200 python -u $P --workload watch --steps 240 --chunk 20 --eager > $OUT/r4g_we.log 2>&1 || exit $?
echo eager; grep steps $OUT/r4g_we.log | cut -c1-40
