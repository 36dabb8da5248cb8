#!/bin/bash
# Which part of the two-connection forced-route capture faults: each mode in
# a fresh process under its own time limit; stops at the first failure.
set -o pipefail
export TMPDIR=/tmp PYTHONPATH=$(pwd)
OUT=gpurun_out
mkdir -p $OUT
for m in copy origin comm; do
  timeout -k 10 120 python -u tools/microbench/fr_probe.py --mode $m > $OUT/frp_$m.log 2>&1
  rc=$?; echo "$m rc=$rc"; grep -E "ok|captured|done" $OUT/frp_$m.log
  [ $rc -eq 0 ] || exit $rc
done
