#!/bin/bash
# The CPU test suite (-m "not gpu") against AddressSanitizer + UndefinedBehaviorSanitizer builds of the
# oracle (oracle/_asan/liboracle.so) and of libbcw.so's host code (bitcaskdb_amd/libbcw_asan.so; the
# device code is unchanged and not run here). CPU only.
set -e
cd "$(dirname "$0")/.."
make -C oracle sanitize > /dev/null
python bitcaskdb_amd/build.py --sanitize 2> /dev/null
# clang's shared ASan runtime (with the UBSan handlers) serves both libraries
ASAN_RT=$(/opt/rocm/lib/llvm/bin/clang -print-file-name=libclang_rt.asan-x86_64.so)
export ORACLE_LIB=$PWD/oracle/_asan/liboracle.so BCW_LIB=$PWD/bitcaskdb_amd/libbcw_asan.so
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=1 UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
LD_PRELOAD="$ASAN_RT" python -m pytest tests -q -x -m "not gpu" -p no:cacheprovider "$@"
