#!/bin/bash
# Graph vs eager for each write workload, back to back; each run under its
# own time limit, stopping at the first failure.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
for w in mix storm watch chain nest; do
  for m in graph eager; do
    extra=""; [ $m = eager ] && extra="--no-graph"
    timeout -k 10 150 python bench.py --no-rtt --no-sustain --workload $w $extra \
      > $OUT/r4c_${w}_$m.log 2>&1 || exit $?
    python3 -c "
import json; d=json.loads(open('$OUT/r4c_${w}_$m.log').read().strip().split('\n')[-1])
print('%-6s %-5s %.4f ms/step graph=%s' % ('$w', '$m', d['ms_per_step'], d['hip_graph']))"
  done
done
