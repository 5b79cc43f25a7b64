#!/bin/bash
# GPU box, round-2 evidence: channel tests, HBM ceilings (tools/roof), rocprof kernel trace +
# FETCH/WRITE passes for C3, C3 + mask and continuous C3, then the default bench line (with the
# CPU baseline).  Each GPU step has its own time limit; outputs in gpurun_out/.
# Usage (from this container): gpurun --timeout 1200 -- tools/gpu_r02.sh TAG
set -e -o pipefail
TAG=${1:-r02}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$ROOT"
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 300 python -u -m pytest tests/test_channel.py -m gpu -k workflow -v --maxfail=3 --timeout 200 --timeout-method thread \
    > gpurun_out/tests_channel_$TAG.log 2>&1 || { tail -40 gpurun_out/tests_channel_$TAG.log; exit 1; }
tail -2 gpurun_out/tests_channel_$TAG.log
fi
timeout -k 10 200 tools/roof 1024 2048 2048 10 > gpurun_out/roof_$TAG.txt
cat gpurun_out/roof_$TAG.txt
tools/profile.sh "${TAG}_c3" --steps 10 --warmup 3
tools/profile.sh "${TAG}_c3_mask" --steps 10 --warmup 3 --mask
tools/profile.sh "${TAG}_c3_cont" --steps 10 --warmup 3 --dither
timeout -k 10 300 python3 bench.py > gpurun_out/bench_default_$TAG.json 2> gpurun_out/bench_default_$TAG.err
cat gpurun_out/bench_default_$TAG.json
