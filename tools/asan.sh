#!/bin/bash
# Host sanitizers (SURVEY.md §5 "race detection / sanitizers"): the host-only C/C++ of the path --
# the N5 chunk codec (csrc/cc_n5.cpp, parses chunk headers from disk) and the C oracle
# (oracle/cc_oracle.c) -- built with -fsanitize=address,undefined and loaded into the CPU tests
# through LD_PRELOAD of the ASan runtime (python itself is not instrumented; leak checks off).
# UBSan errors abort (-fno-sanitize-recover).  CPU only; no GPU code is involved.
# Usage: tools/asan.sh [LOG]   (default profiles/r03_asan.log)
set -e -o pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/build/asan
LOG=${1:-$ROOT/profiles/r03_asan.log}
mkdir -p "$OUT"
SAN="-fsanitize=address,undefined -fno-sanitize-recover=all -fno-omit-frame-pointer -g -O1"
g++ $SAN -std=c++17 -fPIC -shared -Wall -o "$OUT/libcc_n5.so" "$ROOT/cluster_tools_amd/csrc/cc_n5.cpp" -lz -pthread
gcc $SAN -fPIC -shared -ffp-contract=off -fno-fast-math -Wall -Wextra -Wno-unused-parameter \
    -o "$OUT/libcc_oracle.so" "$ROOT/oracle/cc_oracle.c" -lpthread -lm
ASAN_RT=$(gcc -print-file-name=libasan.so)
UBSAN_RT=$(gcc -print-file-name=libubsan.so)
cd "$ROOT"
{
  echo "# $(date -u +%FT%TZ)  gcc $(gcc -dumpfullversion)  flags: $SAN"
  echo "# LD_PRELOAD=$ASAN_RT:$UBSAN_RT  ASAN_OPTIONS=detect_leaks=0:abort_on_error=1"
  CC_N5_LIB_PATH=$OUT/libcc_n5.so CC_ORACLE_LIB=$OUT/libcc_oracle.so \
  LD_PRELOAD=$ASAN_RT:$UBSAN_RT ASAN_OPTIONS=detect_leaks=0:abort_on_error=1 \
  UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 \
    python -m pytest -q -m "not gpu" -p no:cacheprovider tests/test_n5.py tests/test_oracle_golden.py \
        tests/test_threshold.py tests/test_distributed_cpu.py tests/test_large_golden.py -k "not c1_less and not c2" 2>&1
} | tee "$LOG"
