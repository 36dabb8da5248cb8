#!/bin/bash
# round-end style (r3n): full GPU suite, smoke, default bench, all workloads
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests -m gpu > gpurun_out/r3n_tests.log 2>&1 || { tail -40 gpurun_out/r3n_tests.log; exit 1; }
tail -2 gpurun_out/r3n_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
  > gpurun_out/r3n_smoke.log 2>&1 \
  || { tail -20 gpurun_out/r3n_smoke.log; exit 1; }
tail -1 gpurun_out/r3n_smoke.log
timeout -k 10 400 python bench.py > gpurun_out/r3n_default.json 2> gpurun_out/r3n_default.err \
  || { tail -20 gpurun_out/r3n_default.err; exit 1; }
cat gpurun_out/r3n_default.json
for w in mix storm chain; do
timeout -k 10 240 python bench.py --workload $w --steps 20 --warmup 5 --no-rtt \
  > gpurun_out/r3n_$w.json 2> gpurun_out/r3n_$w.err \
  || { tail -20 gpurun_out/r3n_$w.err; exit 1; }
done
for v in "--data-bytes 512" "--data-dist uniform:0-1024" "--data-dist uniform:0-200"; do
timeout -k 10 240 python bench.py --steps 20 --warmup 3 --no-rtt $v \
  >> gpurun_out/r3n_var.json 2>> gpurun_out/r3n_var.err \
  || { tail -20 gpurun_out/r3n_var.err; exit 1; }
done
timeout -k 10 240 python bench.py --workload ensemble --steps 8 --warmup 1 \
  > gpurun_out/r3n_ens.json 2> gpurun_out/r3n_ens.err \
  || { tail -20 gpurun_out/r3n_ens.err; exit 1; }
timeout -k 10 240 python bench.py --sharded --steps 10 --warmup 2 --no-rtt \
  > gpurun_out/r3n_sharded.json 2> gpurun_out/r3n_sharded.err \
  || { tail -20 gpurun_out/r3n_sharded.err; exit 1; }
echo done
