#!/bin/bash
# Profile the device evaluation (tools/bench_eval.py, C3 seg vs gt) on the GPU box: kernel trace
# + stats, then one PMC pass each for FETCH_SIZE and WRITE_SIZE (separate runs).
# Usage: tools/profile_eval.sh TAG   -> gpurun_out/prof_eval_TAG/{trace,fetch,write}, summary.json
set -e -o pipefail
TAG=${1:-cur}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/prof_eval_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 "$ROOT/tools/bench_eval.py" --steps 10 --warmup 2 > "$OUT/bench_eval_trace.json" 2> "$OUT/trace.err"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- \
    python3 "$ROOT/tools/bench_eval.py" --steps 2 --warmup 1 > /dev/null 2> "$OUT/fetch.err"
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- \
    python3 "$ROOT/tools/bench_eval.py" --steps 2 --warmup 1 > /dev/null 2> "$OUT/write.err"
python3 "$ROOT/tools/prof_summary.py" --trace "$OUT/trace" --fetch "$OUT/fetch" --write "$OUT/write" \
    -o "$OUT/summary.json" > "$OUT/summary.txt"
cat "$OUT/summary.txt"
