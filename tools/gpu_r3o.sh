#!/bin/bash
# fresh clean-built artifacts: GPU suite, smoke, default bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests -m gpu > gpurun_out/r3o_tests.log 2>&1 || { tail -40 gpurun_out/r3o_tests.log; exit 1; }
tail -2 gpurun_out/r3o_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
  > gpurun_out/r3o_smoke.log 2>&1 || { tail -20 gpurun_out/r3o_smoke.log; exit 1; }
tail -1 gpurun_out/r3o_smoke.log
timeout -k 10 400 python bench.py > gpurun_out/r3o_default.json 2> gpurun_out/r3o_default.err \
  || { tail -20 gpurun_out/r3o_default.err; exit 1; }
cut -c1-260 gpurun_out/r3o_default.json
