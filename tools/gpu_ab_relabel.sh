#!/bin/bash
# GPU box: round-robin A/B of library builds on tools/bench_relabel.py.  gpurun_out/.
# Usage: ROUNDS=2 tools/gpu_ab_relabel.sh LIB_A LIB_B ...
set -e -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$ROOT"; mkdir -p gpurun_out
for i in $(seq 1 ${ROUNDS:-2}); do
  for L in "$@"; do
    CC_LIB_PATH=$L timeout -k 10 200 python -u tools/bench_relabel.py > gpurun_out/abr.json
    python3 -c "
import json; d=json.loads(open('gpurun_out/abr.json').read().strip().splitlines()[-1])
print('$L'[-30:], d['ms_per_step'], d['kernels_ms_per_step'])"
  done
done
