#!/bin/bash
# GPU box: a pytest selection, then the stage-path bench (tools/bench_stage.py) with its rocprof
# kernel trace + FETCH / WRITE passes.  Usage: gpurun -- tools/gpu_r03_stage.sh TAG 'k-expr'
set -e -o pipefail
TAG=$1; K=$2
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$ROOT"
mkdir -p gpurun_out
if [ -n "$K" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail=3 --timeout 400 --timeout-method thread -k "$K" \
      > gpurun_out/tests_$TAG.log 2>&1 || { tail -60 gpurun_out/tests_$TAG.log; exit 1; }
  tail -3 gpurun_out/tests_$TAG.log
fi
timeout -k 10 300 python -u tools/bench_stage.py greater > gpurun_out/stage_$TAG.json
cat gpurun_out/stage_$TAG.json
timeout -k 10 300 python -u tools/bench_stage.py less > gpurun_out/stage_less_$TAG.json
cat gpurun_out/stage_less_$TAG.json
"$ROOT/tools/profile_cmd.sh" stage_$TAG tools/bench_stage.py greater
