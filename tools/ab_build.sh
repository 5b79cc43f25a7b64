#!/bin/bash
# Build libcc_mi355x.so of another git revision into tools/ab/libcc_<rev>.so for same-box A/B
# timing (bench.py honours CC_LIB_PATH and then skips the provenance check).
# Usage: tools/ab_build.sh REV
set -e
REV=$1
ROOT=$(cd "$(dirname "$0")/.." && pwd)
W=/tmp/ab_$REV
rm -rf "$W"
git -C "$ROOT" worktree add -f "$W" "$REV" > /dev/null 2>&1 || { git -C "$ROOT" worktree prune; git -C "$ROOT" worktree add -f "$W" "$REV" > /dev/null; }
mkdir -p "$ROOT/tools/ab"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wno-unused-function \
    -o "$ROOT/tools/ab/libcc_$REV.so" "$W/cluster_tools_amd/csrc/cc_lib.hip"
git -C "$ROOT" worktree remove --force "$W"
echo "$ROOT/tools/ab/libcc_$REV.so"
