#!/bin/bash
# Profile one bench configuration on the GPU box: kernel trace + stats, then one PMC pass each
# for FETCH_SIZE and WRITE_SIZE (separate runs: MI355X_MICROARCH.md §rocprofv3 PMC slots).
# Usage: tools/profile.sh TAG [bench.py args...]   -> gpurun_out/prof_TAG/{trace,fetch,write}, summary.json
set -e -o pipefail
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 "$ROOT/bench.py" --no-cpu-baseline "$@" > "$OUT/bench_trace.json" 2> "$OUT/trace.err"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- \
    python3 "$ROOT/bench.py" --no-cpu-baseline --steps 2 --warmup 1 "$@" > /dev/null 2> "$OUT/fetch.err"
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- \
    python3 "$ROOT/bench.py" --no-cpu-baseline --steps 2 --warmup 1 "$@" > /dev/null 2> "$OUT/write.err"
# byte-wide mask reads are counted exactly by FETCH_SIZE (prof_summary.py --narrow): with --mask,
# k_spec<true, ...> reads one mask byte per voxel of the workload
NARROW=()
case " $* " in *" --mask "*) NARROW=(--narrow "k_spec<true=${CC_NVOX:-4294967296}");; esac
python3 "$ROOT/tools/prof_summary.py" --trace "$OUT/trace" --fetch "$OUT/fetch" --write "$OUT/write" \
    "${NARROW[@]}" --bench-json "$OUT/bench_trace.json" -o "$OUT/summary.json" > "$OUT/summary.txt"
cat "$OUT/summary.txt"
