#!/bin/bash
# PMC counters for the tree / codec kernels of one workload (default mix):
# L2 hit/miss and memory-side read/write/atomic requests per dispatch.
# Counters only with --kernel-trace (no sys/runtime traces: see the pool rules).
set -o pipefail
W=${1:-mix}
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/pmc_$W
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv \
  --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum \
  -d $OUT -o pmc -- python3 ${GRAFT_REPO_ROOT:-/root/repo}/bench.py \
  --workload $W --steps 3 --warmup 1 --no-rtt > $OUT/run.log 2>&1
echo "pmc rc=$?"
