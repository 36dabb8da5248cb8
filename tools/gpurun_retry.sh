#!/bin/bash
# gpurun_retry.sh <out-file> <command...>: one gpurun call, re-issued only
# when gpurun reports an infrastructure failure before anything ran
# (status=transient / exit 3: no box, nothing charged), after the back-off
# it names.  A command that ran and failed is never re-run.
out=$1; shift
for i in $(seq 1 ${TRIES:-10}); do
  timeout 3000 /usr/local/graft/bin/gpurun --timeout ${GPT:-900} -- "$@" > $out 2>&1
  rc=$?
  if [ $rc -eq 3 ] || grep -q "status=transient" $out; then
    wait_s=$(grep -o "retry in [0-9]*s" $out | grep -o "[0-9]*" | tail -1)
    sleep $(( ${wait_s:-60} + 15 ))
    continue
  fi
  exit $rc
done
exit 3
