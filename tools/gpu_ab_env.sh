#!/bin/bash
# A/B an environment switch on the GET bench: AB_VAR=<name> (values 1 and
# 0), alternated ROUNDS times (default 3); BENCH_ARGS passed through.
# Output: gpurun_out/ab_<name>.log (one JSON line per run, tagged).
set -o pipefail
mkdir -p gpurun_out
OUT=gpurun_out/ab_${AB_VAR}.log
: > $OUT
for i in $(seq ${ROUNDS:-3}); do
  for v in 1 0; do
    env $AB_VAR=$v timeout -k 10 300 python bench.py --no-rtt ${BENCH_ARGS:-} \
      > gpurun_out/ab_run.log 2>&1 || { tail -20 gpurun_out/ab_run.log; exit 1; }
    python - "$AB_VAR=$v" gpurun_out/ab_run.log >> $OUT <<'PY'
import json, sys
line = [l for l in open(sys.argv[2]) if l.startswith('{')][-1]
d = json.loads(line)
print(sys.argv[1], '%.4f ms' % d['ms_per_step'], '%.3f G ops/s' % (d['value'] / 1e9))
PY
  done
done
cat $OUT
