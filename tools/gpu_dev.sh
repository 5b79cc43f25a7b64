#!/bin/bash
# GPU box dev loop: parity subset, roof probe, C3 / continuous C3 bench lines.  gpurun_out/.
set -e -o pipefail
TAG=${1:-dev}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q --maxfail=3 --timeout 300 --timeout-method thread \
    -k "${K:-golden or speculated or continuous or synthetic or noise or runs or mask_vs or normalisation}" \
    > gpurun_out/tests_$TAG.log 2>&1 || { tail -40 gpurun_out/tests_$TAG.log; exit 1; }
tail -2 gpurun_out/tests_$TAG.log
[ -n "$ROOF" ] && timeout -k 10 200 tools/roof 1024 2048 2048 10 > gpurun_out/roof_$TAG.txt && cat gpurun_out/roof_$TAG.txt
for w in "" "--dither"; do
  timeout -k 10 150 python -u bench.py --no-cpu-baseline $w > gpurun_out/bench_$TAG$w.json 2> gpurun_out/bench_$TAG$w.err
  python3 -c "
import json; d=json.loads(open('gpurun_out/bench_$TAG$w.json').read().strip().splitlines()[-1])
print('$w', d['value'], d['ms_per_step'], d['e2e_roofline']['frac'], d['result'].get('n_relabelled_tiles'), {k: v for k, v in list(d['kernels_ms_per_step'].items())[:8]})"
done
