#!/bin/bash
# rocprofv3 kernel trace + stats, then one PMC pass each for FETCH_SIZE and WRITE_SIZE (separate
# runs, MI355X_MICROARCH.md), of an arbitrary python3 command; summary via tools/prof_summary.py.
# Usage: [NARROW=KERNEL=BYTES] tools/profile_cmd.sh TAG script.py [args...]   -> gpurun_out/prof_TAG/
# (NARROW: byte-wide reads of that kernel, counted exactly by FETCH_SIZE: prof_summary.py --narrow)
set -e -o pipefail
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
SCRIPT=$1; shift
case "$SCRIPT" in /*) ;; *) SCRIPT=$ROOT/$SCRIPT;; esac
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 "$SCRIPT" "$@" > "$OUT/out_trace.json" 2> "$OUT/trace.err"
if [ -z "$NO_PMC" ]; then
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- \
    python3 "$SCRIPT" "$@" > /dev/null 2> "$OUT/fetch.err"
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- \
    python3 "$SCRIPT" "$@" > /dev/null 2> "$OUT/write.err"
python3 "$ROOT/tools/prof_summary.py" --trace "$OUT/trace" --fetch "$OUT/fetch" --write "$OUT/write" \
    ${NARROW:+--narrow "$NARROW"} -o "$OUT/summary.json" > "$OUT/summary.txt"
else
python3 "$ROOT/tools/prof_summary.py" --trace "$OUT/trace" -o "$OUT/summary.json" > "$OUT/summary.txt"
fi
head -12 "$OUT/summary.txt"
