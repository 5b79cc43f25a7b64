#!/bin/bash
# Build libcc_mi355x.so of the CURRENT tree with extra compile flags into tools/ab/lib_NAME.so,
# for same-box A/B timing (tools/gpu_ab_libs.sh; bench.py honours CC_LIB_PATH).
# Usage: tools/ab_variant.sh NAME [-DFLAG=value ...]
set -e
NAME=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
S=$ROOT/cluster_tools_amd/csrc
mkdir -p "$ROOT/tools/ab"
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-function $*"
/opt/rocm/bin/hipcc $F -c "$S/cc_lib.hip" -o "/tmp/ab_${NAME}_lib.o" &
P=$!
/opt/rocm/bin/hipcc $F -c "$S/cc_aux.hip" -o "/tmp/ab_${NAME}_aux.o"
wait $P
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o "$ROOT/tools/ab/lib_$NAME.so" "/tmp/ab_${NAME}_lib.o" "/tmp/ab_${NAME}_aux.o"
rm -f "/tmp/ab_${NAME}_lib.o" "/tmp/ab_${NAME}_aux.o"
echo "$ROOT/tools/ab/lib_$NAME.so"
