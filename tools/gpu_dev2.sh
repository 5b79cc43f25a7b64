#!/bin/bash
# GPU box, development loop: a pytest selection (-k EXPR; '' = skip) then N default C3 bench
# lines (extra bench args after N).  Outputs in gpurun_out/dev_TAG_*.
# Usage: gpurun -- tools/gpu_dev2.sh TAG 'pytest -k expr' N [bench args ...]
set -e -o pipefail
TAG=$1; K=$2; N=${3:-1}; shift 3
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$ROOT"
mkdir -p gpurun_out
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -k "$K" \
      > gpurun_out/dev_${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/dev_${TAG}_tests.log; exit 1; }
  tail -2 gpurun_out/dev_${TAG}_tests.log
fi
for i in $(seq 1 $N); do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline "$@" > gpurun_out/dev_${TAG}_bench$i.json 2> gpurun_out/dev_${TAG}_bench$i.err
  python3 -c "
import json; d=json.loads(open('gpurun_out/dev_${TAG}_bench$i.json').read().strip().splitlines()[-1])
k=d['kernels_ms_per_step']; print('ms %.3f e2e %.4f' % (d['ms_per_step'], d['e2e_roofline']['frac']), ' '.join('%s=%.3f' % (a, b) for a, b in list(k.items())[:8]))"
done
