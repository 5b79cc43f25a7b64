#!/bin/bash
# GPU box, end-of-round evidence: the whole -m gpu suite, smoke(), rocprof kernel trace + FETCH /
# WRITE passes of the bench workloads (C3, C3 + mask, continuous C3), then the default bench line
# with the fresh traffic figure.  Outputs in gpurun_out/ (final_*, prof_TAG_*).
# Usage (from this container): gpurun --timeout 1200 -- tools/gpu_final.sh TAG [skip-tests]
set -e -o pipefail
TAG=${1:-r02}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$ROOT"
mkdir -p gpurun_out
if [ -z "$2" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread \
      > gpurun_out/final_tests.log 2>&1 || { tail -40 gpurun_out/final_tests.log; exit 1; }
  tail -2 gpurun_out/final_tests.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.log 2>&1
  tail -3 gpurun_out/final_smoke.log
fi
P=tools/profile_cmd.sh
$P ${TAG}_c3 bench.py --steps 20 --warmup 3 --no-cpu-baseline
tools/profile.sh ${TAG}_c3_mask --steps 20 --warmup 3 --mask      # byte-wide mask reads: --narrow
$P ${TAG}_c3_cont bench.py --steps 20 --warmup 3 --no-cpu-baseline --dither
timeout -k 10 300 python -u bench.py --traffic-json gpurun_out/prof_${TAG}_c3/summary.json \
    > gpurun_out/final_bench.json 2> gpurun_out/final_bench.err
cat gpurun_out/final_bench.json
