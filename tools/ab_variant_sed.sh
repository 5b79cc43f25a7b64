#!/bin/bash
# Like ab_variant.sh, but builds from a COPY of csrc with one sed expression applied (A/B of a
# constant that has no -D hook) -- the tree's sources stay untouched, so the library hash and the
# stamped traffic files stay valid.  Usage: tools/ab_variant_sed.sh NAME FILE 'sed-expr'
set -e
NAME=$1; FILE=$2; EXPR=$3
ROOT=$(cd "$(dirname "$0")/.." && pwd)
D=$(mktemp -d /tmp/absed_XXXX)
mkdir -p "$D/pkg/csrc" "$D/include"
cp -r "$ROOT/cluster_tools_amd/csrc/." "$D/pkg/csrc/"
cp -r "$ROOT/include/." "$D/include/"
T=$D/pkg/csrc
sed -i "$EXPR" "$T/$FILE"
if cmp -s "$T/$FILE" "$ROOT/cluster_tools_amd/csrc/$FILE"; then echo "sed changed nothing" >&2; exit 1; fi
mkdir -p "$ROOT/tools/ab"
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-function"
/opt/rocm/bin/hipcc $F -c "$T/cc_lib.hip" -o "$T/lib.o" &
P=$!
/opt/rocm/bin/hipcc $F -c "$T/cc_aux.hip" -o "$T/aux.o"
wait $P
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o "$ROOT/tools/ab/lib_$NAME.so" "$T/lib.o" "$T/aux.o"
rm -rf "$D"
echo "$ROOT/tools/ab/lib_$NAME.so"
