#!/bin/bash
# A/B bench.py argument sets on one box, alternated ROUNDS times (default 2)
# so box drift hits every set alike.
#   AB_ARGS="--workload,storm,--hash-factor,4 --workload,storm,--hash-factor,2"
# (commas stand for spaces).  Output: gpurun_out/ab_${AB_TAG:-args}.log,
# one line per run (set, ms per step, sustained ms per step, ops/s).
set -o pipefail
mkdir -p gpurun_out
OUT=gpurun_out/ab_${AB_TAG:-args}.log
: > $OUT
for i in $(seq ${ROUNDS:-2}); do
  for set in $AB_ARGS; do
    timeout -k 10 300 python bench.py --no-rtt $(echo "$set" | tr ',' ' ') \
      > gpurun_out/ab_run.log 2>&1 || { tail -20 gpurun_out/ab_run.log; exit 1; }
    python - "$set" gpurun_out/ab_run.log >> $OUT <<'PY'
import json, sys
line = [l for l in open(sys.argv[2]) if l.startswith('{')][-1]
d = json.loads(line)
s = d.get('sustained') or {}
print(sys.argv[1], '%.4f ms' % d['ms_per_step'],
      'sustained %.4f ms' % s.get('ms_per_step', float('nan')),
      '%.3f G ops/s' % (d['value'] / 1e9))
PY
  done
done
cat $OUT
