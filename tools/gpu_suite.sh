#!/bin/bash
# GPU box: the full -m gpu suite (incl. the full-size parity tests), then a default bench line and
# a continuous-input bench line.  Each GPU step has its own time limit; outputs in gpurun_out/.
# Usage (from this container): gpurun --timeout 1200 -- tools/gpu_suite.sh TAG
set -e -o pipefail
TAG=${1:-cur}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail=3 --timeout 400 --timeout-method thread \
    > gpurun_out/tests_$TAG.log 2>&1 || { tail -30 gpurun_out/tests_$TAG.log; exit 1; }
tail -3 gpurun_out/tests_$TAG.log
timeout -k 10 120 python -u bench.py --no-cpu-baseline > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
timeout -k 10 120 python -u bench.py --no-cpu-baseline --dither > gpurun_out/bench_cont_$TAG.json 2> gpurun_out/bench_cont_$TAG.err
cat gpurun_out/bench_$TAG.json gpurun_out/bench_cont_$TAG.json
