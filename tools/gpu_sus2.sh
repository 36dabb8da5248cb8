#!/bin/bash
# Which kernel the slow zxid range costs: the mix started inside it, with a
# kernel-stats profile.  Each GPU step under its own time limit.
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
OUT=$R/gpurun_out
mkdir -p $OUT
P=$R/tools/microbench/sustain_probe.py
timeout -k 10 120 python -u $P --workload mix --steps 20 --chunk 5 --zxid 0x8000000 > $OUT/sus2_mix.log 2>&1 || exit $?
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv \
  -d $OUT/sus2_prof -o prof -- python3 $P --workload mix --steps 10 --chunk 5 \
  --zxid 0x8000000 --eager > $OUT/sus2_prof.log 2>&1
echo "prof rc=$?"
