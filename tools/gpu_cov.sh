#!/bin/bash
# GPU box: rocprof kernel-trace + FETCH/WRITE summaries for the secondary kernels (Threshold task,
# relabel, evaluation, z-slab sharded schedule, input preparation) and the C1 drop-in timing.
# Usage (from this container): gpurun --timeout 1200 -- tools/gpu_cov.sh TAG
set -e -o pipefail
TAG=${1:-r02}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$ROOT"
mkdir -p gpurun_out
P=tools/profile_cmd.sh
${ONLY_C1:+true} $P ${TAG}_threshold tools/bench_threshold.py
${ONLY_C1:+true} $P ${TAG}_relabel tools/bench_relabel.py
${ONLY_C1:+true} $P ${TAG}_eval tools/bench_eval.py --steps 4 --warmup 1
${ONLY_C1:+true} $P ${TAG}_sharded tools/dev_sharded_prof.py 2 256 4096 4096
${ONLY_C1:+true} $P ${TAG}_prefilter tools/bench_prefilter.py --steps 3
timeout -k 10 400 python3 tools/bench_c1.py --repeats 2 > gpurun_out/c1_$TAG.json 2> gpurun_out/c1_$TAG.err
cat gpurun_out/c1_$TAG.json
