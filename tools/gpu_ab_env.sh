#!/bin/bash
# A/B environment settings on a bench workload, alternated ROUNDS times
# (default 3) so box drift hits every setting alike.
#   AB_VAR=<name> AB_VALUES="1 0"     one variable over values, or
#   AB_SETS="A=1,B=2 -"               whole settings ("-" = the defaults)
# BENCH_ARGS is passed through (e.g. AB_VAR=ZKMI_FREE_COMPACT
# AB_VALUES="1 0" BENCH_ARGS="--workload nest" for the free-ring compaction
# A/B).  Output: gpurun_out/ab_<tag>.log, one line per run (setting, ms per
# step, sustained ms per step, ops/s).
set -o pipefail
mkdir -p gpurun_out
if [ -n "$AB_SETS" ]; then
  SETS="$AB_SETS"; TAG=${AB_TAG:-sets}
else
  SETS=""
  for v in ${AB_VALUES:-1 0}; do SETS="$SETS $AB_VAR=$v"; done
  TAG=${AB_TAG:-$AB_VAR}
fi
OUT=gpurun_out/ab_${TAG}.log
: > $OUT
for i in $(seq ${ROUNDS:-3}); do
  for set in $SETS; do
    envs=""
    [ "$set" != "-" ] && envs=$(echo "$set" | tr ',' ' ')
    env $envs timeout -k 10 300 python bench.py --no-rtt ${BENCH_ARGS:-} \
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
