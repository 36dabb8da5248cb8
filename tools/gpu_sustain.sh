#!/bin/bash
# Per-chunk step times of the write workloads over long runs; each under
# its own time limit; stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
P=tools/microbench/sustain_probe.py
timeout -k 10 150 python -u $P --workload mix --steps 800 > $OUT/sus_mix.log 2>&1 || exit $?
timeout -k 10 150 python -u $P --workload watch --steps 40 --chunk 4 > $OUT/sus_watch.log 2>&1 || exit $?
timeout -k 10 200 python -u $P --workload nest --steps 200 --chunk 20 > $OUT/sus_nest.log 2>&1 || exit $?
timeout -k 10 150 python -u $P --workload mix --steps 400 --eager > $OUT/sus_mix_eager.log 2>&1 || exit $?
