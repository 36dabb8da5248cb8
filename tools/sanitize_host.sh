#!/bin/bash
# Run the host-codec suites against the AddressSanitizer + UBSan build of
# csrc/host (host code only; GPU sanitizers are not used on this pool).
set -eo pipefail
cd "$(dirname "$0")/.."
SO=$(python tools/build_native.py --sanitize | tail -1)
export LD_PRELOAD="$(gcc -print-file-name=libasan.so):$(gcc -print-file-name=libubsan.so)"
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=1
export UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1
export ZKMI_HOST_CODEC_PATH="$SO"
python -m pytest -q -x -p no:cacheprovider tests/test_host_codec.py \
  tests/test_proto.py tests/test_fuzz_codec.py "$@"
