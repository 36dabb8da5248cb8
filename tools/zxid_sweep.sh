#!/bin/bash
# K1 across zxid ranges: the write workloads' reply streams carry the
# tree's zxids, whose bytes can read as frame lengths (round 4: zxids in
# [2^27, 2^28) cost a 200 ms repair a scan).  Each workload is started at
# several zxids and timed in chunks (tools/microbench/sustain_probe.py);
# gpurun_out/zxid_sweep.log gets one line per (workload, zxid) with the
# slowest chunk.
set -o pipefail
OUT=gpurun_out/zxid_sweep.log
mkdir -p gpurun_out
: > $OUT
for wl in ${WLS:-mix watch storm}; do
  [ "$wl" = storm ] && continue      # (the probe drives mix / nest / chain / watch)
  for z in ${ZXIDS:-0x100000 0x1000000 0x8000000 0xC000000 0x10000000 0x40000000 0x7F000000}; do
    timeout -k 10 180 python tools/microbench/sustain_probe.py --workload $wl \
      --steps ${STEPS:-60} --chunk 20 --zxid $z > gpurun_out/zxid_run.log 2>&1 \
      || { tail -20 gpurun_out/zxid_run.log; exit 1; }
    python - "$wl" "$z" gpurun_out/zxid_run.log >> $OUT <<'PY'
import re, sys
ms = [float(m.group(1)) for m in
      re.finditer(r'steps\s+\d+\s+([0-9.]+) ms/step', open(sys.argv[3]).read())]
print(sys.argv[1], sys.argv[2], 'chunks', ' '.join('%.3f' % x for x in ms),
      'max %.3f' % max(ms))
PY
  done
done
cat $OUT
