#!/bin/bash
# Build libcc_mi355x.so of another git revision into tools/ab/lib_<rev>.so for same-box A/B
# timing (bench.py honours CC_LIB_PATH and then skips the provenance check).
# Usage: tools/ab_build.sh REV
set -e
REV=$1
ROOT=$(cd "$(dirname "$0")/.." && pwd)
W=/tmp/ab_$REV
rm -rf "$W"
git -C "$ROOT" worktree add -f "$W" "$REV" > /dev/null 2>&1 || { git -C "$ROOT" worktree prune; git -C "$ROOT" worktree add -f "$W" "$REV" > /dev/null; }
mkdir -p "$ROOT/tools/ab"
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-function"
if [ -f "$W/cluster_tools_amd/csrc/cc_aux.hip" ]; then     # two translation units (cc_aux.hip)
  /opt/rocm/bin/hipcc $F -c "$W/cluster_tools_amd/csrc/cc_lib.hip" -o "$W/lib.o" &
  /opt/rocm/bin/hipcc $F -c "$W/cluster_tools_amd/csrc/cc_aux.hip" -o "$W/aux.o"
  wait
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o "$ROOT/tools/ab/lib_$REV.so" "$W/lib.o" "$W/aux.o"
else
  /opt/rocm/bin/hipcc $F -shared -o "$ROOT/tools/ab/lib_$REV.so" "$W/cluster_tools_amd/csrc/cc_lib.hip"
fi
git -C "$ROOT" worktree remove --force "$W"
echo "$ROOT/tools/ab/lib_$REV.so"
