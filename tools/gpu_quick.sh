#!/bin/bash
# GPU box: a pytest selection (-k EXPR, optional) then bench lines; outputs in gpurun_out/.
# Usage: gpurun -- tools/gpu_quick.sh TAG 'pytest -k expr' [bench args ...]
set -e -o pipefail
TAG=$1; K=$2; shift 2
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$ROOT"
mkdir -p gpurun_out
if [ -n "$K" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail=3 --timeout 400 --timeout-method thread -k "$K" \
      > gpurun_out/tests_$TAG.log 2>&1 || { tail -60 gpurun_out/tests_$TAG.log; exit 1; }
  tail -3 gpurun_out/tests_$TAG.log
fi
