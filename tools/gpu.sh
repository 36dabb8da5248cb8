#!/bin/bash
# The one GPU runner for gpurun calls: a list of steps, each under its own
# time limit; the chain stops at the first failure (no step is retried).
#
#   tools/gpu.sh STEP [STEP ...]
#
# A step is NAME or NAME=ARGS; ARGS is one word, commas stand for spaces.
#   tests[=ARGS]        pytest -m gpu over tests/ (ARGS: what to run
#                       instead, e.g. tests/test_frame_repair.py,-k,garbage)
#   cpu                 pytest -m "not gpu"
#   smoke               __graft_entry__.smoke()
#   bench[=ARGS]        bench.py ARGS (default: the driver's config)
#   prof=TAG[,WL...]    rocprofv3 --kernel-trace --stats of bench.py
#                       --steps 5 for each workload WL (default get)
#   profb=TAG,ARGS      rocprofv3 --kernel-trace --stats of bench.py ARGS
#   pmc=WL              tools/pmc_passes.sh WL (one counter pass a run)
#   sustain=WL[,STEPS[,CHUNK]]   tools/microbench/sustain_probe.py
#   py=SCRIPT[,ARGS]    python -u SCRIPT ARGS
#   multi               tools/gpu_rehearse_multi.sh (gloo ranks on 1 GPU)
# Logs: gpurun_out/<n>_<name>.log.  TLIM overrides every step's limit (s).
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
n=0
run() {           # run LIMIT LOG CMD...: one GPU step
  local lim=${TLIM:-$1} log=$2; shift 2
  timeout -k 10 $lim "$@" > $log 2>&1
  local rc=$?
  echo "[$n $(basename $log .log)] rc=$rc"
  tail -${TAILN:-3} $log | cut -c1-600
  return $rc
}
for step in "$@"; do
  n=$((n + 1))
  name=${step%%=*}
  args=""
  [ "$name" != "$step" ] && args=$(echo "${step#*=}" | tr ',' ' ')
  log=$OUT/${n}_$name.log
  case $name in
    tests)
      run 900 $log python -u -m pytest ${args:-tests} -x -q -m gpu \
        --timeout 120 --timeout-method thread ;;
    cpu)
      run 600 $log python -m pytest tests -x -q -m "not gpu" $args ;;
    smoke)
      run 200 $log python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench)
      run 300 $log python bench.py $args ;;
    prof)
      set -- $args
      tag=$1; shift
      rc=0
      for w in ${@:-get}; do
        (cd /tmp && run 300 $OUT/${n}_${tag}_$w.log rocprofv3 --kernel-trace \
          --stats --output-format csv -d $OUT/${tag}_$w -o prof -- \
          python3 $R/bench.py --workload $w --steps 5 --warmup 1 --no-rtt) \
          || { rc=$?; break; }
      done
      [ $rc -eq 0 ] ;;
    profb)
      set -- $args
      tag=$1; shift
      (cd /tmp && run 300 $OUT/${n}_$tag.log rocprofv3 --kernel-trace --stats \
        --output-format csv -d $OUT/$tag -o prof -- python3 $R/bench.py "$@") ;;
    pmc)
      run 600 $log bash $R/tools/pmc_passes.sh $args ;;
    sustain)
      set -- $args
      run 300 $log python -u $R/tools/microbench/sustain_probe.py \
        --workload ${1:-mix} --steps ${2:-400} --chunk ${3:-20} ;;
    py)
      run 300 $log python -u $args ;;
    multi)
      run 1200 $log bash $R/tools/gpu_rehearse_multi.sh ;;
    *)
      echo "unknown step: $step"; false ;;
  esac
  rc=$?
  [ $rc -eq 0 ] || exit $rc
done
