#!/bin/bash
# Build libcc_mi355x.so of another git revision into tools/ab/lib_<rev>.so for same-box A/B
# timing (bench.py honours CC_LIB_PATH and then skips the provenance check).
# Usage: tools/ab_build.sh REV
set -e -o pipefail
REV=$1
ROOT=$(cd "$(dirname "$0")/.." && pwd)
W=/tmp/ab_$REV
rm -rf "$W"
mkdir -p "$W" "$ROOT/tools/ab"
git -C "$ROOT" archive "$REV" cluster_tools_amd/csrc include | tar -x -C "$W"
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-function"
if [ -f "$W/cluster_tools_amd/csrc/cc_aux.hip" ]; then     # two translation units (cc_aux.hip)
  /opt/rocm/bin/hipcc $F -c "$W/cluster_tools_amd/csrc/cc_lib.hip" -o "$W/lib.o" &
  P=$!
  /opt/rocm/bin/hipcc $F -c "$W/cluster_tools_amd/csrc/cc_aux.hip" -o "$W/aux.o"
  wait $P
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o "$ROOT/tools/ab/lib_$REV.so" "$W/lib.o" "$W/aux.o"
else
  /opt/rocm/bin/hipcc $F -shared -o "$ROOT/tools/ab/lib_$REV.so" "$W/cluster_tools_amd/csrc/cc_lib.hip"
fi
rm -rf "$W"
echo "$ROOT/tools/ab/lib_$REV.so"
