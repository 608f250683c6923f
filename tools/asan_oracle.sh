#!/bin/bash
# tests/test_oracle.py against the AddressSanitizer + UBSan build of the C port (oracle/cpu_ref.c), host only:
# libasan preloaded into python (the interpreter itself is not instrumented), leak checks off (python's allocator).
set -eo pipefail
cd "$(dirname "$0")/.."
make -s -C oracle asan
ASAN=$(gcc -print-file-name=libasan.so)
LD_PRELOAD=$ASAN ASAN_OPTIONS=detect_leaks=0:abort_on_error=1 UBSAN_OPTIONS=print_stacktrace=1 \
  QOC_CPUREF_LIB=$PWD/oracle/build/asan/libqoc_cpuref.so \
  python -m pytest tests/test_oracle.py -q -m "not gpu" -p no:cacheprovider "$@"
