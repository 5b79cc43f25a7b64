#!/bin/bash
# Refresh the committed evidence for the current tree on the GPU box: rocprofv3 kernel trace +
# FETCH_SIZE / WRITE_SIZE passes for C3 and C3 + mask, then the default bench line (with the CPU
# baseline).  Each GPU step has its own time limit; outputs land in gpurun_out/.
# Usage (from this container): gpurun --timeout 900 -- tools/refresh_profiles.sh TAG
set -e -o pipefail
TAG=${1:-cur}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$ROOT"
mkdir -p gpurun_out
tools/profile.sh "${TAG}_c3" --steps 10 --warmup 3
tools/profile.sh "${TAG}_c3_mask" --steps 10 --warmup 3 --mask
timeout -k 10 300 python3 bench.py > gpurun_out/bench_default_$TAG.json 2> gpurun_out/bench_default_$TAG.err
cat gpurun_out/bench_default_$TAG.json
