#!/bin/bash
# GPU box: the round-3 measurements of the kernels committed without a profile -- stage path,
# Threshold task (speculative and two-pass), C1 cold start, sharded-slab readiness (8 slabs).
# Usage: gpurun --timeout 1200 -- tools/gpu_r03_measure.sh TAG
set -e -o pipefail
TAG=$1
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$ROOT"
mkdir -p gpurun_out
O=gpurun_out/m_$TAG
mkdir -p $O
timeout -k 10 300 python -u tools/bench_stage.py greater > $O/stage_greater.json; cat $O/stage_greater.json
timeout -k 10 300 python -u tools/bench_threshold.py > $O/thr_spec.json; cat $O/thr_spec.json
CC_THRESHOLD_TWO_PASS=1 timeout -k 10 300 python -u tools/bench_threshold.py > $O/thr_two.json; cat $O/thr_two.json
timeout -k 10 300 python -u bench.py --workload c1 --no-cpu-baseline > $O/c1_cold.json; cat $O/c1_cold.json
timeout -k 10 300 python -u tools/bench_sharded_slabs.py 8 c4 5 > $O/slabs8_c4.json; cat $O/slabs8_c4.json
timeout -k 10 300 python -u tools/bench_sharded_slabs.py 8 c3 5 > $O/slabs8_c3.json; cat $O/slabs8_c3.json
"$ROOT/tools/profile_cmd.sh" stage_$TAG tools/bench_stage.py greater
"$ROOT/tools/profile_cmd.sh" thr_$TAG tools/bench_threshold.py
