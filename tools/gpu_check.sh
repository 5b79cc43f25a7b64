#!/bin/bash
# GPU-box check used during development: parity tests, C3 bench (greater / less) and one SQ
# counter pass.  Each GPU step has its own time limit; results go to gpurun_out/.
# Usage (from this container): gpurun --timeout 600 -- tools/gpu_check.sh [TAG]
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=${1:-chk}
cd "$ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -3 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench.json || exit 1
timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --mode less > gpurun_out/bench_less.json || exit 1
tools/pmc_bench.sh "pmc_$TAG"
