#!/bin/bash
# Round-end evidence for the current tree (GPU box): rocprof kernel trace + FETCH / WRITE passes of
# every single-GPU workload, the default bench line with the fresh C3 traffic, the other workloads'
# lines and the 8-slab schedule.  Outputs in gpurun_out/ (prof_TAG_*, final_*_TAG.json).
# Usage (from this container): gpurun --timeout 1200 -- tools/gpu_r06_final.sh TAG
set -e -o pipefail
TAG=${1:-r06f}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$ROOT"; mkdir -p gpurun_out
O=gpurun_out
tools/gpu_steps.sh $TAG boxinfo
tools/profile.sh ${TAG}_c3 --steps 10 --warmup 3
CC_NVOX=4294967296 tools/profile.sh ${TAG}_c4 --workload c4 --steps 10 --warmup 3 --mask
tools/profile.sh ${TAG}_c3_cont --steps 10 --warmup 3 --dither
tools/profile.sh ${TAG}_c2 --workload c2 --steps 20 --warmup 5
tools/profile.sh ${TAG}_c1 --workload c1 --steps 20 --warmup 5
tools/profile.sh ${TAG}_c5 --workload c5 --steps 10 --warmup 3
timeout -k 10 300 python -u bench.py --traffic-json $O/prof_${TAG}_c3/summary.json > $O/final_bench_$TAG.json 2> $O/final_bench_$TAG.err
cat $O/final_bench_$TAG.json
for w in c4 c2 c1 c5; do
  timeout -k 10 240 python -u bench.py --no-cpu-baseline --workload $w --traffic-json $O/prof_${TAG}_$w/summary.json \
      > $O/final_bench_${w}_$TAG.json 2> $O/final_bench_${w}_$TAG.err
  tail -c 400 $O/final_bench_${w}_$TAG.json; echo
done
tools/gpu_steps.sh $TAG slabs8_c3 slabs8_c4
