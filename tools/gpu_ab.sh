#!/bin/bash
# GPU box: A/B(/C...) of environment settings on the bench, round-robin, same box.  gpurun_out/.
# Usage: ROUNDS=3 tools/gpu_ab.sh "ENV_A" "ENV_B" [...] -- [bench args]
set -e -o pipefail
V=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do V+=("$1"); shift; done
[ "$1" = "--" ] && shift
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$ROOT"; mkdir -p gpurun_out
for i in $(seq 1 ${ROUNDS:-3}); do
  for j in "${!V[@]}"; do
    E=${V[$j]}
    env $E timeout -k 10 150 python -u bench.py --no-cpu-baseline --steps 10 "$@" > gpurun_out/ab_$j.json 2> gpurun_out/ab_$j.err
    python3 -c "
import json; d=json.loads(open('gpurun_out/ab_$j.json').read().strip().splitlines()[-1])
print('$j [$E]'[-60:], d['ms_per_step'], {k: v for k, v in list(d['kernels_ms_per_step'].items())[:4]})"
  done
done
