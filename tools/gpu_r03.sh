#!/bin/bash
# GPU box: a pytest selection (-k EXPR, empty = whole -m gpu suite), then a default bench line.
# Usage: gpurun --timeout 1200 -- tools/gpu_r03.sh TAG 'k-expr' [bench args ...]
set -e -o pipefail
TAG=$1; K=$2; shift 2
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$ROOT"
mkdir -p gpurun_out
KARG=()
if [ -n "$K" ]; then KARG=(-k "$K"); fi
if [ "$K" != "none" ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -v --maxfail=3 --timeout 400 --timeout-method thread "${KARG[@]}" \
      > gpurun_out/tests_$TAG.log 2>&1 || { tail -60 gpurun_out/tests_$TAG.log; exit 1; }
  tail -3 gpurun_out/tests_$TAG.log
fi
timeout -k 10 180 python -u bench.py --no-cpu-baseline "$@" > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
cat gpurun_out/bench_$TAG.json
