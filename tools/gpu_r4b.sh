#!/bin/bash
# GET connections-per-GPU sweep, GET PMC passes, long watch run; each GPU
# step under its own time limit, stopping at the first failure.
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
OUT=$R/gpurun_out
mkdir -p $OUT
for s in 1 3 4; do
  timeout -k 10 150 python bench.py --no-rtt --no-sustain --streams $s > $OUT/r4b_streams$s.log 2>&1 || exit $?
  echo "streams $s: $(tail -1 $OUT/r4b_streams$s.log | cut -c1-400)"
done
timeout -k 10 200 python -u tools/microbench/sustain_probe.py --workload watch --steps 400 --chunk 40 > $OUT/r4b_sus_watch.log 2>&1 || exit $?
bash tools/pmc_passes.sh get
