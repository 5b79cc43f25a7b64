#!/bin/bash
# GPU box: A/B of environment settings on the C3 bench, alternating, same box.  gpurun_out/.
# Usage: tools/gpu_ab.sh "ENV_A" "ENV_B" [rounds] [bench args]
set -e -o pipefail
A=$1; B=$2; N=${3:-3}; shift 3 || true
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$ROOT"; mkdir -p gpurun_out
for i in $(seq 1 $N); do
  for v in A B; do
    if [ $v = A ]; then E=$A; else E=$B; fi
    env $E timeout -k 10 150 python -u bench.py --no-cpu-baseline --steps 10 "$@" > gpurun_out/ab_$v$i.json 2> gpurun_out/ab_$v$i.err
    python3 -c "
import json; d=json.loads(open('gpurun_out/ab_$v$i.json').read().strip().splitlines()[-1])
print('$v [$E]', d['ms_per_step'], {k: v for k, v in list(d['kernels_ms_per_step'].items())[:4]})"
  done
done
