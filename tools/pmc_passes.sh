#!/bin/bash
# PMC counter passes over one bench workload (default get), one rocprofv3 run
# per pass (a pass holds at most 4 TCC counters: FETCH_SIZE uses 3 and
# WRITE_SIZE 2, so they get separate passes).  Counters only with
# --kernel-trace (no sys/runtime traces, per the pool rules).  Summarise
# with tools/pmc_summary.py.
set -o pipefail
W=${1:-get}
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/pmc_$W
REPO=${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
pass() {
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv \
    --pmc "$@" -d $OUT/$name -o pmc -- python3 $REPO/bench.py \
    --workload $W --steps 3 --warmup 1 --no-rtt --no-sustain > $OUT/$name.log 2>&1
  local rc=$?
  echo "pass $name rc=$rc"
  return $rc
}
pass fetch FETCH_SIZE && \
pass write WRITE_SIZE && \
pass sq SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD \
  SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES && \
pass lds SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES \
  GRBM_GUI_ACTIVE
