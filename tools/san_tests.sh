#!/bin/bash
# AddressSanitizer + UBSan run of the CPU suite (-m "not gpu"): the host producers and C ABI
# (libsrt_amd_san.so, host code instrumented) and the oracle (liboracle_san.so), loaded by the
# ordinary tests through SRT_LIB_PATH / ORACLE_LIB_PATH with the sanitizer runtimes preloaded.
set -e
cd "$(dirname "$0")/.."
make -s -C simple-ray-tracer_amd SAN=1 -j8 2>&1 | grep -v hip-link || true
make -s -C oracle SAN=1
export SRT_LIB_PATH=$PWD/simple-ray-tracer_amd/libsrt_amd_san.so
export ORACLE_LIB_PATH=$PWD/oracle/_build/liboracle_san.so
export LD_PRELOAD="$(gcc -print-file-name=libasan.so):$(gcc -print-file-name=libubsan.so)"
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=1
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
# the given test files, or the whole CPU suite except the test that runs this script
if [ $# -gt 0 ]; then set -- "$@"; else set -- tests --deselect tests/test_sanitizers.py; fi
python -m pytest -x -q -m "not gpu" -p no:cacheprovider "$@"
