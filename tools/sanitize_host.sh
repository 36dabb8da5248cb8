#!/bin/bash
# Run the host-codec and event-loop suites against the AddressSanitizer +
# UBSan builds of csrc/host (host code only; GPU sanitizers are not used on
# this pool).
set -eo pipefail
cd "$(dirname "$0")/.."
read -r SO LOOP_SO _WATCH_SO _FSM_SO MACH_SO < <(python tools/build_native.py --sanitize | tail -1)
export LD_PRELOAD="$(gcc -print-file-name=libasan.so):$(gcc -print-file-name=libubsan.so)"
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=1
export UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1
export ZKMI_HOST_CODEC_PATH="$SO"
export ZKMI_NATIVE_LOOP_PATH="$LOOP_SO"
export ZKMI_MACHINES_PATH="$MACH_SO"
python -m pytest -q -x -p no:cacheprovider tests/test_host_codec.py \
  tests/test_proto.py tests/test_fuzz_codec.py tests/test_native_loop.py \
  tests/test_basic.py tests/test_completion.py tests/test_machines.py \
  tests/test_nasty.py "$@"
unset ZKMI_MACHINES_PATH

# ThreadSanitizer over the threaded host code (the native event loop): the
# loop, client and fault-injection suites
TSAN_SO=$(python tools/build_native.py --tsan | tail -1)
LD_PRELOAD="$(gcc -print-file-name=libtsan.so)" \
TSAN_OPTIONS="halt_on_error=1 report_signal_unsafe=0" \
ZKMI_HOST_CODEC_PATH= ZKMI_NATIVE_LOOP_PATH="$TSAN_SO" \
  python -m pytest -q -x -p no:cacheprovider tests/test_native_loop.py \
  tests/test_basic.py tests/test_nasty.py tests/test_completion.py "$@"
